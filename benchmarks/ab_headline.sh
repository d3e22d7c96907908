#!/bin/bash
# Alternating A/B of the 32 B echo headline leg between two trees:
#   bash benchmarks/ab_headline.sh <old_tree_dir> [rounds]
set -o pipefail
OLD=$1
N=${2:-3}
mkdir -p gpurun_out/abh
for i in $(seq 1 $N); do
  timeout -k 10 120 python3 $OLD/bench.py --only echo_32B --steps 20 --warmup 3 > gpurun_out/abh/old_$i.txt 2>/dev/null || exit 1
  echo "old $i $(grep '^{' gpurun_out/abh/old_$i.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("step_qps_median_32B"), d.get("p99_us"), d.get("cpu_us_per_rpc_32B", d.get("echo_32B_cpu_us_per_rpc")))')"
  timeout -k 10 120 python3 bench.py --only echo_32B --steps 20 --warmup 3 > gpurun_out/abh/new_$i.txt 2>/dev/null || exit 1
  echo "new $i $(grep '^{' gpurun_out/abh/new_$i.txt | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("step_qps_median_32B"), d.get("p99_us"), d.get("cpu_us_per_rpc_32B", d.get("echo_32B_cpu_us_per_rpc")))')"
done
