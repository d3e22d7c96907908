#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/l
P="$GRAFT_REPO_ROOT/gpurun_out/l"
export TMPDIR=/tmp
run() { local name=$1; shift; env "$@" timeout -k 10 60 python benchmarks/latency_trace.py --seconds 10 --top 6 > $P/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v "amdgpu.ids\|^I1" $P/$name.log | head -12; return $rc; }
run nap50 NAP_US=50 &&
run nap50_norpcz NAP_US=50 NO_RPCZ=1 &&
timeout -k 10 400 python bench.py > $P/bench.log 2>&1; echo "bench rc=$?"; grep -oE '"p(50|99|999)_us_at_100qps": [0-9.]+|"cpu_pct_at_100qps": [0-9.]+|"placement_rank0": \{[^}]*\}|"qps_1MB": [0-9.]+|"timed_s_1MB": [0-9.]+' $P/bench.log
