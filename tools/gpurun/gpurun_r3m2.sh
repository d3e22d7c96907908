#!/bin/bash
# two ranks sharing the one GPU of the box: the N>1 legs (fan-out, scatter,
# route, relay, streams) over cross-process HBM lending on real hardware
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/m2
rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --skip-rccl --skip-sweep --steps 3 --warmup 1 --latency-sample-s 2 > $P/bench2.log 2>&1; rc=$?
grep '^{"metric"' $P/bench2.log > $P/bench2.json
python - <<'PY'
import json
try:
    d = json.loads(open("gpurun_out/m2/bench2.json").read())
except Exception as e:
    print("no json", e)
else:
    keys = [k for k in d if any(s in k for s in ("fanout", "scatter", "route", "pipeline", "stream", "errors", "qps_64KB"))]
    print({k: d[k] for k in keys})
    print(d.get("transport"))
PY
grep -v "^I1\|amdgpu" $P/bench2.log | tail -15
exit $rc
