#!/bin/bash
# Kernel traces of the device number-codec legs (csv), summarized.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/profk2; rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
for leg in ids_baidu_gpu ids_json_gpu; do
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$P/kt_$leg" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --leg $leg --seconds 2 --no-profile > "$GRAFT_REPO_ROOT/$P/$leg.log" 2>&1) || exit $?
  tail -1 $P/$leg.log
done
for leg in ids_baidu_gpu; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d "$GRAFT_REPO_ROOT/$P/pmc_fetch_$leg" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --leg $leg --seconds 1 --no-profile > "$GRAFT_REPO_ROOT/$P/pmc_fetch_$leg.log" 2>&1) || exit $?
  (cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d "$GRAFT_REPO_ROOT/$P/pmc_write_$leg" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --leg $leg --seconds 1 --no-profile > "$GRAFT_REPO_ROOT/$P/pmc_write_$leg.log" 2>&1) || exit $?
done
python3 benchmarks/rocprof_summary.py $P/kt_ids_baidu_gpu $P/kt_ids_json_gpu $P/pmc_fetch_ids_baidu_gpu $P/pmc_write_ids_baidu_gpu --prune > $P/summary.txt 2>&1
cat $P/summary.txt | head -60
