#!/bin/bash
# Two bench ranks on this box's GPU, each started DIRECTLY under rocprofv3
# (the program after `--`, rank variables exported by this script), with
# the kernel and HIP runtime traces: when did each pull kernel run, against
# when it was launched and when the event poller saw it complete.
#   bash benchmarks/xproc_trace.sh [outdir]
set -o pipefail
OUT=${1:-gpurun_out/xtrace}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd - > /dev/null
export WORLD_SIZE=2 LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561 GROUP_RANK=0
ARGS="--gpus 2 --steps 2 --warmup 1 --requests-per-step-64k 4000 --only echo_64KB --skip-rccl --latency-sample-s 0
      --time-budget-s 100 --hard-deadline-s 140"
# PROF=0: the same two ranks without the profiler
ARGS="$ARGS ${EXTRA:-}"
for r in 0 1; do
    if [ "${PROF:-1}" = 1 ]; then
        RANK=$r LOCAL_RANK=$r timeout -k 10 200 rocprofv3 ${PROFARGS:---kernel-trace --hip-runtime-trace} --output-format csv \
            -d $OUT/r$r -o r$r -- python3 bench.py $ARGS > $OUT/r$r.out 2> $OUT/r$r.err &
    else
        RANK=$r LOCAL_RANK=$r timeout -k 10 200 python3 bench.py $ARGS > $OUT/r$r.out 2> $OUT/r$r.err &
    fi
    pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=$?; done
exit $rc
