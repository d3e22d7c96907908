#!/bin/bash
# Round-2 GPU session: tests, bench (host + device payload), rocprof of the
# device-payload bench. Stops at the first fault/abort/timeout.
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
  tail -3 "$out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 400 python bench.py
  step bench_host 400 python bench.py --host-payload --latency-sample-s 0 --skip-stream
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
  cd /tmp
  step rocprof_dev 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_dev" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --latency-sample-s 0 --skip-stream --steps 5 --warmup 1
  rm -f "$GRAFT_REPO_ROOT/gpurun_out/prof_dev/run_kernel_trace.csv"  # per-launch rows: too big to copy back
fi
echo done
