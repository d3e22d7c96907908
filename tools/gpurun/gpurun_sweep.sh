#!/bin/bash
# 32 B headline sweep on the GPU box: fiber workers and idle-spin knobs.
# Each run prints one JSON line; summary in gpurun_out/sweep.txt.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/sweep.txt
: > $out
run() {  # label, then env assignments / args
  local label=$1; shift
  echo "== $label" | tee -a $out
  local t0=$(grep -E '^(nr_throttled|throttled_usec|usage_usec)' /sys/fs/cgroup/cpu.stat | tr '\n' ' ')
  timeout -k 10 120 env "$@" > gpurun_out/sweep_run.log 2>&1
  local rc=$?
  local t1=$(grep -E '^(nr_throttled|throttled_usec|usage_usec)' /sys/fs/cgroup/cpu.stat | tr '\n' ' ')
  echo "cpu.stat before: $t0" | tee -a $out
  echo "cpu.stat after:  $t1" | tee -a $out
  grep '^{' gpurun_out/sweep_run.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('value=%.0f p99=%s med=%.0f min=%.0f max=%.0f' % (d['value'], d['p99_us'], d['step_qps_median_32B'], d['step_qps_min_32B'], d['step_qps_max_32B'])); print('steps(k): ' + ' '.join(str(q // 1000) for q in d.get('step_qps_seq_32B', [])))
" | tee -a $out
  if [ $rc -ne 0 ]; then echo "rc=$rc" | tee -a $out; tail -5 gpurun_out/sweep_run.log; exit $rc; fi
}
B="python3 bench.py --skip-64k --skip-grpc --skip-stream --latency-sample-s 0 --steps 20 --warmup 3"
nproc; cat /sys/fs/cgroup/cpu.max || true
L="python3 bench.py --skip-64k --skip-grpc --skip-stream --latency-sample-s 4 --steps 2 --warmup 1 --requests-per-step 2000"
lat() {
  local label=$1; shift
  echo "== $label" | tee -a $out
  timeout -k 10 120 env "$@" > gpurun_out/sweep_run.log 2>&1 || { echo "rc=$?" | tee -a $out; tail -5 gpurun_out/sweep_run.log; exit 1; }
  grep '^{' gpurun_out/sweep_run.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('lat100: p50=%s p99=%s' % (d.get('p50_us_at_100qps'), d.get('p99_us_at_100qps')))
" | tee -a $out
}
G="python3 bench.py --skip-64k --skip-stream --latency-sample-s 0 --steps 5 --warmup 1 --requests-per-step 20000"
grpc() {
  local label=$1; shift
  echo "== $label" | tee -a $out
  timeout -k 10 180 env "$@" > gpurun_out/sweep_run.log 2>&1 || { echo "rc=$?" | tee -a $out; tail -5 gpurun_out/sweep_run.log; exit 1; }
  grep '^{' gpurun_out/sweep_run.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('grpc cpu=%s gpu=%s p99 cpu=%s gpu=%s' % (d.get('grpc_snappy_64KB_qps_cpu_codec'), d.get('grpc_snappy_64KB_qps_gpu_codec'), d.get('grpc_snappy_64KB_p99_us_cpu_codec'), d.get('grpc_snappy_64KB_p99_us_gpu_codec')))
" | tee -a $out
}
for kb in 1 2 4; do grpc "block_kb=$kb" MRPC_FLAGS="--gpu_snappy_block_kb=$kb" $G; done
echo done
