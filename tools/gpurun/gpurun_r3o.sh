#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/o
P="$GRAFT_REPO_ROOT/gpurun_out/o"
export TMPDIR=/tmp
timeout -k 10 90 python benchmarks/latency_trace.py --seconds 3 --top 5 --dump 3 --qps 0 --concurrency 16 --attachment 16777216 --device-attachment > $P/dev16m.log 2>&1; rc=$?; grep -v "amdgpu.ids\|^I1" $P/dev16m.log | head -60; exit $rc
