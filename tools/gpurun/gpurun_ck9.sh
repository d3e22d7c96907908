#!/bin/bash
# Checkpoint 9: GPU tests, smoke, default bench (stops at the first fault/timeout).
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/ck9; rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $P/pytest_gpu.log 2>&1; rc=$?
tail -3 $P/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $P/smoke.log 2>&1 || exit $?
tail -1 $P/smoke.log
timeout -k 10 600 python bench.py > $P/bench.log 2>&1 || exit $?
grep '^{"metric"' $P/bench.log > $P/bench.json
echo done
