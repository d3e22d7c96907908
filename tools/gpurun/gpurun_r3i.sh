#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/i
P="$GRAFT_REPO_ROOT/gpurun_out/i"
export TMPDIR=/tmp
NAP_US=0 timeout -k 10 60 python benchmarks/latency_trace.py --seconds 10 > $P/nap0.log 2>&1 && cat $P/nap0.log &&
NAP_US=50 timeout -k 10 60 python benchmarks/latency_trace.py --seconds 10 > $P/nap50.log 2>&1 && cat $P/nap50.log
