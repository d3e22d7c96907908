#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g
for s in /sys/devices/system/cpu/cpu0/cpuidle/state*; do echo "$(cat $s/name 2>/dev/null) latency=$(cat $s/latency 2>/dev/null) residency=$(cat $s/residency 2>/dev/null) disable=$(cat $s/disable 2>/dev/null)"; done
cat /sys/devices/system/cpu/cpuidle/current_governor* 2>/dev/null
uname -r
timeout -k 5 60 ./build/bin/wake_latency --gap_us 10000 --samples 500 --modes block,nap:20,nap:50,nap:100,spin
timeout -k 5 60 taskset -c 64-71 ./build/bin/wake_latency --gap_us 10000 --samples 300 --modes block,nap:50
