#!/bin/bash
# Idle-spin A/B: -fiber_idle_spin_us 0 vs W (with a spinner present, a ready
# fiber wakes no parked worker). The fiber microbench at both settings, then
# alternating runs of the 32 B echo headline leg and one device leg.
#   bash benchmarks/spin_ab.sh [spin_us] [rounds]
set -o pipefail
W=${1:-50}
N=${2:-3}
mkdir -p gpurun_out/spin
for v in 0 $W; do
  echo "microbench spin=$v"
  timeout -k 10 120 build/bin/mrpc_microbench --seconds 1 --threads 1 --flag fiber_idle_spin_us=$v \
    > gpurun_out/spin/micro_$v.txt || exit 1
  head -3 gpurun_out/spin/micro_$v.txt
done
leg() {
  grep '^{' $1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("p99_us"))'
}
for i in $(seq 1 $N); do
  for v in 0 $W; do
    timeout -k 10 120 python3 bench.py --only echo_32B --steps 20 --warmup 3 --flag fiber_idle_spin_us=$v \
      > gpurun_out/spin/echo_${v}_$i.txt 2>/dev/null || exit 1
    echo "echo32 spin=$v run $i: $(leg gpurun_out/spin/echo_${v}_$i.txt)"
  done
done
