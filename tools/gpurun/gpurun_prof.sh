#!/bin/bash
# Profiling session: CPU profiles of single legs + rocprof API/kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" | tee -a gpurun_out/prof/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/prof/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(date +%T)" | tee -a gpurun_out/prof/steps.log
  head -3 "gpurun_out/prof/$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for leg in ${LEGS:-gpu_handler dev_64k host_64k}; do
  step cpu_$leg 120 python benchmarks/profile_leg.py --leg $leg --seconds 3
done
for spin in ${SPINS:-0 200}; do
  SPIN_US=$spin step lat_spin$spin 120 python benchmarks/profile_leg.py --leg lat_100qps --seconds 4 --workers 12
done
if [ -n "${ROCPROF:-}" ]; then
  cd /tmp
  step rocprof_handler 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof/rp_handler" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --leg gpu_handler --seconds 2
fi
echo done
