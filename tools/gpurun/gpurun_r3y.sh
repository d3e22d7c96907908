#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/y
export TMPDIR=/tmp
timeout -k 10 120 python benchmarks/rccl_probe.py --points 4194304:16,8388608:16,16777216:1,16777216:4,16777216:16 > gpurun_out/y/probe.log 2>&1; rc=$?; grep -E "^size|Error|abort" gpurun_out/y/probe.log | cut -c1-500; exit $rc
