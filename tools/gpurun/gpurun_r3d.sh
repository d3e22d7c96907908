#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/d
P="$GRAFT_REPO_ROOT/gpurun_out/d"
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 60 python benchmarks/profile_leg.py --no-profile --seconds 2 "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc $(grep -E '^leg|^copy' $P/$name.log | tr '\n' ' ')"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run handler_w10 --leg gpu_handler --workers 10
run handler_qd1 --leg gpu_handler --concurrency 1
run dev_w10 --leg dev_64k --workers 10
run dev_qd1 --leg dev_64k --concurrency 1
echo done
