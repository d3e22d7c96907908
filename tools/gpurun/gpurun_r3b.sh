#!/bin/bash
# Round-3 GPU session B: tests, bench, kernel stats + PMC of the RPC legs.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/b
export TMPDIR=/tmp
P="$GRAFT_REPO_ROOT/gpurun_out/b"
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)" | tee -a "$P/steps.log"
  timeout -k 10 "$t" "$@" > "$P/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(date +%T)" | tee -a "$P/steps.log"
  tail -2 "$P/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
WHAT=${WHAT:-tests,bench,prof}
case ",$WHAT," in *,tests,*)
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ;;
esac
case ",$WHAT," in *,bench,*)
  step bench 600 python bench.py ;;
esac
case ",$WHAT," in *,prof,*)
  for leg in gpu_handler dev_64k host_64k lat_100qps; do
    step cpu_$leg 120 python benchmarks/profile_leg.py --leg $leg --seconds 3
  done
  cd /tmp
  step kt_handler 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/kt_handler" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --leg gpu_handler --seconds 2
  step kt_dev64k 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/kt_dev64k" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --leg dev_64k --seconds 2
  step pmc_fetch_handler 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d "$P/pmc_fetch_handler" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --leg gpu_handler --seconds 1
  step pmc_write_handler 120 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d "$P/pmc_write_handler" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --leg gpu_handler --seconds 1
  step pmc_fetch_dev64k 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d "$P/pmc_fetch_dev64k" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --leg dev_64k --seconds 1
  step pmc_write_dev64k 120 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d "$P/pmc_write_dev64k" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --leg dev_64k --seconds 1
  cd "$GRAFT_REPO_ROOT"
  python benchmarks/rocprof_summary.py "$P"/kt_handler "$P"/kt_dev64k "$P"/pmc_fetch_handler "$P"/pmc_write_handler "$P"/pmc_fetch_dev64k "$P"/pmc_write_dev64k --prune > "$P/rocprof_summary.txt" 2>&1
  du -sh "$P"
  ;;
esac
echo done
