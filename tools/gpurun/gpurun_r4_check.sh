#!/bin/bash
# Checkpoint: every GPU test, smoke, then the default bench (stops at the
# first failure). Usage: gpurun_r4_check.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/${1:-chk}; rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $P/pytest_gpu.log 2>&1; rc=$?
tail -3 $P/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $P/smoke.log 2>&1 || exit $?
tail -1 $P/smoke.log
timeout -k 10 600 python -u bench.py > $P/bench.log 2> $P/bench.err || exit $?
grep '^{"metric"' $P/bench.log > $P/bench.json
python3 -c "import json,sys; d=json.load(open('$P/bench.json')); print({k: d[k] for k in ('value','p99_us','qps_64KB','rccl_64KB_qps','rccl_1MB_gbytes_per_s','rccl_aborts','errors_64KB_gpu_handler')})"
