#!/bin/bash
# RCCL plane: GPU tests for the plane, then the bench (rccl leg included).
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
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step rccl_tests 240 python -u -m pytest tests/test_gpu_rccl.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread
step bench_rccl 400 python bench.py --skip-grpc --skip-stream --latency-sample-s 0
echo done
