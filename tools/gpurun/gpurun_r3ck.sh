#!/bin/bash
# full checkpoint: GPU tests, smoke, bench, kernel stats of the bench
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/ck
rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $P/pytest_gpu.log 2>&1; rc=$?; tail -3 $P/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $P/smoke.log 2>&1; rc=$?; tail -2 $P/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > $P/bench.log 2>&1; rc=$?; grep '^{"metric"' $P/bench.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
