#!/bin/bash
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/z7
rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_snappy.py tests/test_gpu_json.py > $P/pytest.log 2>&1; rc=$?; tail -1 $P/pytest.log; [ $rc -eq 0 ] || exit $rc
for k in 6 8; do
MRPC_FLAGS="--codec_batch_max_inflight=$k" timeout -k 10 300 python bench.py --steps 5 --warmup 1 --skip-64k --skip-rccl --skip-1m --skip-sweep --skip-stream --latency-sample-s 1 > $P/bench_k$k.log 2>&1 || exit $?
python - $k <<'PY'
import json, sys
line = [l for l in open("gpurun_out/z7/bench_k%s.log" % sys.argv[1]) if l.startswith('{"metric"')][-1]
d = json.loads(line)
c = d["cpu_us_per_rpc"]
print("k=%s grpc cpu %.0f gpu %.0f (%.2f/launch, p99 %s) cpu_us %s/%s | baidu_std cpu %.0f gpu %.0f cpu_us %s/%s | json cpu %.0f gpu %.0f" % (
    sys.argv[1], d["grpc_snappy_64KB_qps_cpu_codec"], d["grpc_snappy_64KB_qps_gpu_codec"], d["grpc_gpu_codec_requests_per_launch"],
    d["grpc_snappy_64KB_p99_us_gpu_codec"], c["grpc_snappy_cpu_codec"], c["grpc_snappy_gpu_codec"],
    d["baidu_std_snappy_64KB_qps_cpu"], d["baidu_std_snappy_64KB_qps_gpu"], c["baidu_std_snappy_64KB_cpu"], c["baidu_std_snappy_64KB_gpu"],
    d["http_json_64KB_qps_cpu"], d["http_json_64KB_qps_gpu"]))
PY
done
