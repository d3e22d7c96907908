#!/bin/bash
# Round-3 checkpoint: whole GPU suite, smoke, bench, kernel stats + PMC of the RPC legs.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/w
P="$GRAFT_REPO_ROOT/gpurun_out/w"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$P/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 600 python bench.py
cd /tmp
step kt_dev64k 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/kt_dev64k" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --no-profile --leg dev_64k --seconds 2
step kt_handler 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/kt_handler" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --no-profile --leg gpu_handler --seconds 2
step pmc_fetch_dev64k 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d "$P/pmc_fetch_dev64k" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --no-profile --leg dev_64k --seconds 1
step pmc_write_dev64k 120 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d "$P/pmc_write_dev64k" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --no-profile --leg dev_64k --seconds 1
cd "$GRAFT_REPO_ROOT"
python benchmarks/rocprof_summary.py "$P"/kt_dev64k "$P"/kt_handler "$P"/pmc_fetch_dev64k "$P"/pmc_write_dev64k --prune > "$P/rocprof_summary.txt" 2>&1
du -sh "$P"
echo done
