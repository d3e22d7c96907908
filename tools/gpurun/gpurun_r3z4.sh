#!/bin/bash
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/z4
rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_snappy.py tests/test_snappy_vectors.py > $P/pytest.log 2>&1; rc=$?; tail -3 $P/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profz4 -o run -- python3 $GRAFT_REPO_ROOT/benchmarks/profile_leg.py --leg grpc_gpu --seconds 2 --no-profile > $GRAFT_REPO_ROOT/$P/run.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
grep "^leg=" $P/run.log
f=$(find /tmp/profz4 -name "*kernel_stats.csv" | head -1); cp "$f" $P/kernel_stats.csv; cut -d, -f1-4 "$f" | head -12
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --skip-64k --skip-rccl --skip-1m --skip-sweep --skip-stream --latency-sample-s 1 > $P/bench_grpc.log 2>&1 || exit $?
python - <<'PY'
import json
line = [l for l in open("gpurun_out/z4/bench_grpc.log") if l.startswith('{"metric"')][-1]
d = json.loads(line)
print({k: v for k, v in d.items() if "grpc" in k})
print(d["cpu_us_per_rpc"])
PY
