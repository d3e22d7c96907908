#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/v
P="$GRAFT_REPO_ROOT/gpurun_out/v"
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > $P/t.log 2>&1; rc=$?; grep -E "passed|failed|Error|assert" $P/t.log | tail -6; [ $rc -eq 0 ] || exit $rc
run() { local name=$1; shift; env "$@" timeout -k 10 60 python benchmarks/profile_leg.py --no-profile --seconds 3 $LEGARGS > $P/$name.log 2>&1; local rc=$?; echo "$name rc=$rc $(grep -E '^leg|^copy|^resident' $P/$name.log | tr '\n' ' ')"; return $rc; }
LEGARGS="--leg dev_64k" run dev_resident RESIDENT=1 &&
LEGARGS="--leg dev_64k" run dev_resident_g4 RESIDENT=1 RESIDENT_GROUPS=4 &&
LEGARGS="--leg gpu_handler" run h_resident RESIDENT=1 &&
LEGARGS="--leg dev_64k --concurrency 1" run dev_qd1_resident RESIDENT=1 &&
LEGARGS="--leg gpu_handler --concurrency 1" run h_qd1_resident RESIDENT=1
