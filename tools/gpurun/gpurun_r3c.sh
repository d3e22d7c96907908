#!/bin/bash
# Handler-leg experiments: worker count, queue depth, CFS throttling.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c
P="$GRAFT_REPO_ROOT/gpurun_out/c"
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 60 python benchmarks/profile_leg.py --no-profile --seconds 2 "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep '^leg' $P/$name.log)"; if [ $rc -ne 0 ]; then exit $rc; fi; }
cat /sys/fs/cgroup/cpu.max > "$P/cpu_max.txt" 2>&1 || true
for w in 6 8 10 12; do
  run host_w$w --leg host_64k --workers $w
  run handler_w$w --leg gpu_handler --workers $w
done
run host_qd1 --leg host_64k --concurrency 1
run handler_qd1 --leg gpu_handler --concurrency 1
run dev_qd1 --leg dev_64k --concurrency 1
POLL_SPIN_US=0 run handler_nospin --leg gpu_handler
SPIN_US=0 run host_nospin --leg host_64k
echo done
