#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/t
P="$GRAFT_REPO_ROOT/gpurun_out/t"
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $P/t.log 2>&1; rc=$?; grep -E "passed|failed|Error|assert" $P/t.log | tail -12; exit $rc
