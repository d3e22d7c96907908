#!/bin/bash
# Where does the bench's 100-QPS p99 come from? Same sample in isolation,
# first in the bench, and last in the bench without the RCCL legs.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/f
P="$GRAFT_REPO_ROOT/gpurun_out/f"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; grep -oE '"p(50|99|999)_us_at_100qps": [0-9.]+|"cpu_pct_at_100qps": [0-9.]+|^leg=.*' "$P/$name.log" | tr '\n' ' '; echo; if [ $rc -ne 0 ]; then tail -5 "$P/$name.log"; exit $rc; fi; }
step gpujson 120 python -u -m pytest tests/test_gpu_json.py -x -v --timeout 60 --timeout-method thread -p no:cacheprovider -k jsonout
step lat_iso 60 python benchmarks/profile_leg.py --no-profile --leg lat_100qps --seconds 6
step lat_first 300 python bench.py --steps 3 --warmup 1 --latency-first --skip-64k --skip-grpc --skip-rccl --skip-1m --skip-sweep --skip-stream
step lat_first_all 400 python bench.py --steps 5 --warmup 1 --latency-first --skip-sweep
step lat_last_norccl 400 python bench.py --steps 5 --warmup 1 --skip-rccl --skip-sweep
echo done
