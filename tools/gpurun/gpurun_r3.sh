#!/bin/bash
# Round-3 GPU session: GPU tests, smoke, bench (+ optional rocprof pass).
# Every step has its own time limit; the script stops at the first fault,
# abort or timeout (any rc other than 0/1).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  local out="$GRAFT_REPO_ROOT/gpurun_out"
  echo "== $name $(date +%T)" | tee -a "$out/steps.log"
  timeout -k 10 "$t" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(date +%T)" | tee -a "$out/steps.log"
  tail -3 "$out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
WHAT=${1:-all}
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  step bench 600 python bench.py
fi
if [ "$WHAT" = prof ]; then
  cd /tmp
  step rocprof_bench 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --latency-sample-s 0
fi
echo done
