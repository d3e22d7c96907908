#!/bin/bash
# Latency-at-100qps + 32B throughput under different spin settings.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cat /proc/loadavg > gpurun_out/lat_load.txt
i=0
for cfg in "default" "nospin" "default" "nospin" "default"; do
  i=$((i+1))
  if [ "$cfg" = nospin ]; then export MRPC_FLAGS="--fiber_idle_spin_us=0 --event_dispatcher_spin_us=0"; else unset MRPC_FLAGS; fi
  timeout -k 10 120 python bench.py --skip-64k --latency-sample-s 4 > gpurun_out/lat_${i}_${cfg}.json 2>gpurun_out/lat_${i}_${cfg}.err || exit 1
done
