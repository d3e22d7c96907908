#!/bin/bash
# One GPU session: tests, smoke, bench, kernel microbench, rocprof.
# Stops at the first fault/abort/timeout (exit codes other than 0/1).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  local out="$GRAFT_REPO_ROOT/gpurun_out"
  echo "== $name" | tee -a "$out/steps.log"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$out/steps.log"
  tail -5 "$out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
rocm-smi --showproductname > gpurun_out/rocm_smi.log 2>&1 || true
step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py
step bench_devpayload 600 python bench.py --device-payload --latency-sample-s 0
step kernels 600 python benchmarks/gpu_kernels.py
cd /tmp
step rocprof_kernels 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_kernels" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/gpu_kernels.py"
echo done
