#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/j
P="$GRAFT_REPO_ROOT/gpurun_out/j"
export TMPDIR=/tmp
run() { local name=$1; shift; env "$@" timeout -k 10 60 python benchmarks/latency_trace.py --seconds 10 --top 6 > $P/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "amdgpu.ids\|^I1" $P/$name.log; return $rc; }
run nap50 NAP_US=50 &&
run nap50_wnap50 NAP_US=50 WORKER_NAP_US=50 &&
run nap50_wnap50_norpcz NAP_US=50 WORKER_NAP_US=50 NO_RPCZ=1 &&
run nap50_norpcz NAP_US=50 NO_RPCZ=1 &&
run nap50_wnap20 NAP_US=20 WORKER_NAP_US=20
