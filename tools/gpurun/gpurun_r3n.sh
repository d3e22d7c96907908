#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/n
P="$GRAFT_REPO_ROOT/gpurun_out/n"
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "split or lending" > $P/t.log 2>&1; rc=$?; tail -5 $P/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --skip-grpc --skip-stream > $P/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 $P/bench.log; exit $rc; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/n/bench.log") if l.startswith('{"metric"')][-1])
for p in d.get("sweep", []): print(p)
print({k: d[k] for k in d if "1MB" in k})
print(d["transport"])
print({k: d[k] for k in d if "100qps" in k})
PY
