#!/bin/bash
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/z3
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 120 python benchmarks/profile_leg.py --leg grpc_gpu --seconds 3 --no-profile > $P/grpc_gpu_noprof.txt 2>&1 || exit $?
grep "^leg=" $P/grpc_gpu_noprof.txt
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --skip-64k --skip-rccl --skip-1m --skip-sweep --skip-stream --latency-sample-s 10 > $P/bench_grpc.log 2>&1 || exit $?
python - <<'PY'
import json
line = [l for l in open("gpurun_out/z3/bench_grpc.log") if l.startswith('{"metric"')][-1]
d = json.loads(line)
print({k: v for k, v in d.items() if "grpc" in k or "100qps" in k})
print(d["cpu_us_per_rpc"], d["config"].get("placement_rank0"))
PY
