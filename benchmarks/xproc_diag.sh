#!/bin/bash
# Cross-process device-path diagnosis: the same HBM echo
# legs in one process and in N ranks sharing this box's GPU, each run's
# JSON (with the per-leg `diag` breakdown) under gpurun_out/xproc/.
#   bash benchmarks/xproc_diag.sh [N] [extra bench args...]
set -o pipefail
N=${1:-2}
shift || true
OUT=gpurun_out/xproc
mkdir -p $OUT
COMMON="--steps 5 --warmup 1 --requests-per-step-64k 20000 --requests-per-step-1m 4000 --only echo_64KB,echo_1MB
        --skip-rccl --latency-sample-s 0 --time-budget-s 150 --hard-deadline-s 200"
run() {  # name, env..., -- args
    local name=$1; shift
    echo "== $name $(date +%T)"
    timeout -k 10 240 env "$@" $COMMON > $OUT/$name.json 2> $OUT/$name.err
    local rc=$?
    python3 benchmarks/leg_summary.py $OUT/$name.json 2>/dev/null || tail -c 400 $OUT/$name.json
    return $rc
}
run n1 python3 bench.py --gpus 1 "$@" &&
run n${N} python3 bench.py --gpus $N "$@"
