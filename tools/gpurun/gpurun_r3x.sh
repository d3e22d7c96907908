#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/x
P="$GRAFT_REPO_ROOT/gpurun_out/x"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --skip-grpc --skip-stream --verbose-sweep > $P/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep -E "^sweep|Error|error|exhausted|refusing" $P/bench.log | cut -c1-300 | head -40; exit $rc
