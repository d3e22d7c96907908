#!/bin/bash
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/z5
rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_snappy.py > $P/pytest.log 2>&1; rc=$?; tail -2 $P/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --skip-64k --skip-rccl --skip-1m --skip-sweep --skip-stream --latency-sample-s 1 > $P/bench_grpc$i.log 2>&1 || exit $?
python - $i <<'PY'
import json, sys
line = [l for l in open("gpurun_out/z5/bench_grpc%s.log" % sys.argv[1]) if l.startswith('{"metric"')][-1]
d = json.loads(line)
print({k: v for k, v in d.items() if "grpc" in k or "json" in k or "baidu" in k}, d["cpu_us_per_rpc"])
PY
done
timeout -k 10 120 python benchmarks/profile_leg.py --leg grpc_gpu --seconds 3 --top 70 > $P/grpc_gpu_prof.txt 2>&1 || exit $?
grep "^leg=" $P/grpc_gpu_prof.txt
