#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/h
P="$GRAFT_REPO_ROOT/gpurun_out/h"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; grep -oE '"p(50|99|999)_us_at_100qps": [0-9.]+|"cpu_pct_at_100qps": [0-9.]+|^leg=.*' "$P/$name.log" | tr '\n' ' '; echo; if [ $rc -ne 0 ]; then tail -5 "$P/$name.log"; exit $rc; fi; }
NAP_US=0 step lat_nap0 60 python benchmarks/profile_leg.py --no-profile --leg lat_100qps --seconds 6
NAP_US=50 step lat_nap50 60 python benchmarks/profile_leg.py --no-profile --leg lat_100qps --seconds 6
NAP_US=0 SPIN_US=0 step lat_nap0_spin0 60 python benchmarks/profile_leg.py --no-profile --leg lat_100qps --seconds 6
NAP_US=50 SPIN_US=0 step lat_nap50_spin0 60 python benchmarks/profile_leg.py --no-profile --leg lat_100qps --seconds 6
NAP_US=20 step lat_nap20 60 python benchmarks/profile_leg.py --no-profile --leg lat_100qps --seconds 6
step lat_first 300 python bench.py --steps 3 --warmup 1 --latency-first --skip-64k --skip-grpc --skip-rccl --skip-1m --skip-sweep --skip-stream
echo done
