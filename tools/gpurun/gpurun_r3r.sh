#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r
P="$GRAFT_REPO_ROOT/gpurun_out/r"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "gpu_process or handler or crc" > $P/t.log 2>&1; rc=$?; grep -E "passed|failed|FAILED|Error" $P/t.log | tail -5; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
timeout -k 10 90 python benchmarks/latency_trace.py --seconds 2 --top 2 --qps 0 --concurrency 50 --attachment 65520 --gpu-process > $P/handler.log 2>&1; rc=$?; grep -v "amdgpu.ids\|^I1" $P/handler.log | head -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --skip-sweep > $P/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $P/bench.log; exit $rc; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r/bench.log") if l.startswith('{"metric"')][-1])
print({k: d[k] for k in d if "handler" in k or "host_attachment" in k or k in ("value", "qps_64KB", "qps_1MB")})
print(d["cpu_us_per_rpc"])
PY
