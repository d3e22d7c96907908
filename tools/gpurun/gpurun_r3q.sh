#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/q
P="$GRAFT_REPO_ROOT/gpurun_out/q"
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 90 python benchmarks/latency_trace.py --seconds 2 --top 4 --dump 1 --qps 0 "$@" > $P/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "amdgpu.ids\|^I1" $P/$name.log | head -30; return $rc; }
run handler --concurrency 50 --attachment 65520 --gpu-process &&
run host --concurrency 50 --attachment 65520 &&
run handler_qd1 --concurrency 1 --attachment 65520 --gpu-process
