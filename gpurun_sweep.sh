#!/bin/bash
# Worker-count sweep of the 32B echo bench (3 repeats each) + latency sample.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cat /sys/fs/cgroup/cpu.max > gpurun_out/sweep_cpu.txt 2>&1; cat /proc/loadavg >> gpurun_out/sweep_cpu.txt
for w in ${SWEEP_WORKERS:-4 6 8 12 16}; do
  for r in 1 2 3; do
    timeout -k 10 120 python bench.py --workers $w --skip-64k --latency-sample-s ${LAT_S:-0} > gpurun_out/sweep_w${w}_r${r}.json 2>/dev/null || exit 1
  done
done
