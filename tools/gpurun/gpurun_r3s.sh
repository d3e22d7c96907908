#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s
P="$GRAFT_REPO_ROOT/gpurun_out/s"
export TMPDIR=/tmp
timeout -k 10 120 python benchmarks/profile_leg.py --leg echo_32b --seconds 3 --top 60 > $P/echo32.log 2>&1; rc=$?; head -3 $P/echo32.log; exit $rc
