#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/p
P="$GRAFT_REPO_ROOT/gpurun_out/p"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_snappy_vectors.py tests/test_gpu_json.py tests/test_gpu_ops.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $P/t.log 2>&1; rc=$?; grep -E "passed|failed|FAILED|Error" $P/t.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 90 python benchmarks/latency_trace.py --seconds 3 --top 5 --dump 1 --qps 0 --concurrency 16 --attachment 16777216 --device-attachment > $P/dev16m.log 2>&1; rc=$?; grep -v "amdgpu.ids\|^I1" $P/dev16m.log | head -24; exit $rc
