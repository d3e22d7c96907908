#!/bin/bash
# Device pack (K2) and pb2json arrays (K6): tests, then the codec legs only.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/k2; rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pb_pack.py tests/test_gpu_snappy.py tests/test_gpu_json.py > $P/pytest.log 2>&1; rc=$?
tail -3 $P/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --skip-64k --skip-rccl --skip-1m --skip-sweep --skip-stream --latency-sample-s 1 > $P/bench.log 2>&1 || exit $?
grep '^{"metric"' $P/bench.log > $P/bench.json
python - <<'PY'
import json
d = json.load(open("gpurun_out/k2/bench.json"))
for k, v in d.items():
    if any(x in k for x in ("snappy", "json", "grpc")) and not isinstance(v, dict): print(k, v)
print(json.dumps(d.get("cpu_us_per_rpc")))
PY
