#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/m
P="$GRAFT_REPO_ROOT/gpurun_out/m"
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 60 python benchmarks/latency_trace.py --seconds 3 --top 8 "$@" > $P/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "amdgpu.ids\|^I1" $P/$name.log | head -20; return $rc; }
run dev1m_qd1 --qps 0 --concurrency 1 --attachment 1048576 --device-attachment &&
run dev64k_qd1 --qps 0 --concurrency 1 --attachment 65536 --device-attachment &&
run host1m_qd1 --qps 0 --concurrency 1 --attachment 1048576
