#!/bin/bash
# Checkpoint 12: all GPU tests, smoke, default bench, then a kernel trace of
# the codec legs (stops at the first failure).
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/ck12; rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $P/pytest_gpu.log 2>&1; rc=$?
tail -3 $P/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $P/smoke.log 2>&1 || exit $?
tail -1 $P/smoke.log
timeout -k 10 600 python bench.py > $P/bench.log 2>&1 || exit $?
grep '^{"metric"' $P/bench.log > $P/bench.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$P/prof" -o codec -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --skip-64k --skip-rccl --skip-1m --skip-sweep --skip-stream --latency-sample-s 0 > "$GRAFT_REPO_ROOT/$P/rocprof.log" 2>&1 || exit $?
echo done
cd "$GRAFT_REPO_ROOT" && python3 benchmarks/rocprof_summary.py $P/prof --prune > $P/rocprof_summary.txt 2>&1; head -30 $P/rocprof_summary.txt
