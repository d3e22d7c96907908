#!/bin/bash
# One GPU-box call, as named stages run in order; the first failing stage
# ends the call (every GPU step has its own time limit, steps chain with &&).
#   tests        pytest -m gpu (one process, per-test timeout)
#   smoke        __graft_entry__.smoke()
#   bench1       bench.py at N=1 (the driver's BENCH shape)
#   rehearse:K   K ranks on the box's one GPU (torchrun, --skip-rccl: RCCL
#                refuses ranks that share a GPU), every N>1 leg, small steps
#   pytest:FILE  one GPU test file (tests/FILE.py)
#   bench:ARGS   bench.py ARGS (comma-separated), one JSON + a leg summary
#   run:ARGS     python ARGS (comma-separated), output in run_N.txt
#   kt:ARGS      rocprofv3 kernel trace of bench.py ARGS (comma-separated)
# Output lands in gpurun_out/<tag>/ (tag = $TAG, default "run").
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=gpurun_out/${TAG:-run}; mkdir -p $T
nb=0
nr=0
for st in "$@"; do
  case $st in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > $T/pytest_gpu.txt 2>&1 || { tail -30 $T/pytest_gpu.txt; exit 1; }
      tail -3 $T/pytest_gpu.txt ;;
    smoke)
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $T/smoke.txt 2>&1 || { tail $T/smoke.txt; exit 1; }
      tail -1 $T/smoke.txt ;;
    bench1)
      timeout -k 10 600 python -u bench.py > $T/bench1.log 2>&1 || { tail -20 $T/bench1.log; exit 1; }
      grep '^{"metric"' $T/bench1.log > $T/bench1.json; cut -c1-400 $T/bench1.json ;;
    rehearse:*)
      k=${st#rehearse:}
      timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node $k --master-addr 127.0.0.1 \
        --master-port 29533 bench.py --gpus $k --skip-rccl --steps 5 --warmup 1 --requests-per-step 20000 \
        --requests-per-step-64k 4000 --requests-per-step-1m 400 --requests-per-step-grpc 400 \
        --requests-per-step-fanout 200 --latency-sample-s 2 --sweep-seconds 0.2 \
        > $T/rehearse$k.log 2>&1 || { tail -20 $T/rehearse$k.log; exit 1; }
      grep '^{"metric"' $T/rehearse$k.log > $T/rehearse$k.json; cut -c1-400 $T/rehearse$k.json ;;
    pytest:*)
      f=${st#pytest:}
      timeout -k 10 600 python -u -m pytest tests/${f%%::*}.py -m gpu -x -q --timeout 120 --timeout-method thread \
        > $T/pytest_${f%%::*}.txt 2>&1 || { tail -40 $T/pytest_${f%%::*}.txt; exit 1; }
      tail -2 $T/pytest_${f%%::*}.txt ;;
    bench:*)
      args=${st#bench:}; nb=$((nb+1))
      timeout -k 10 600 python -u bench.py ${args//,/ } > $T/bench_$nb.log 2>&1 || { tail -20 $T/bench_$nb.log; exit 1; }
      grep '^{"metric"' $T/bench_$nb.log > $T/bench_$nb.json; echo "bench_$nb: $args"; python benchmarks/leg_summary.py $T/bench_$nb.json ;;
    run:*)
      args=${st#run:}; nr=$((nr+1))
      timeout -k 10 600 python -u ${args//,/ } > $T/run_$nr.txt 2>&1 || { tail -30 $T/run_$nr.txt; exit 1; }
      echo "run_$nr: $args"; tail -40 $T/run_$nr.txt ;;
    kt:*)
      args=${st#kt:}
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $T/kt -o kt -- python3 bench.py ${args//,/ } \
        > $T/kt.log 2>&1 || { tail -20 $T/kt.log; exit 1; }
      python benchmarks/rocprof_summary.py $T/kt > $T/kt_summary.txt 2>&1; head -40 $T/kt_summary.txt ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
