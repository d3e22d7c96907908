#!/bin/bash
# GPU tests after the bulk packed parse, then the 32 B headline + 100-QPS sample (widened placement).
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/lat2; rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $P/pytest_gpu.log 2>&1; rc=$?
tail -2 $P/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --skip-64k --skip-grpc --skip-rccl --skip-1m --skip-sweep --skip-stream --latency-sample-s 5 > $P/bench.log 2>&1 || exit $?
grep '^{"metric"' $P/bench.log > $P/bench.json
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/lat2/bench.json"))
print("32B", d["value"], "p99", d["p99_us"], "| 100qps p50/p99/p999", d.get("p50_us_at_100qps"), d.get("p99_us_at_100qps"), d.get("p999_us_at_100qps"))
print(json.dumps(d.get("placement_at_100qps_rank0")))
PY
