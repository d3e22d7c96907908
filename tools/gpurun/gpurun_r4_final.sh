#!/bin/bash
# Packed decoder numbers, then the full checkpoint (all GPU tests, smoke, bench).
set -u
cd "$GRAFT_REPO_ROOT"
bash tools/gpurun/gpurun_r4_bw.sh ${1:-fin}_bw || exit $?
bash tools/gpurun/gpurun_r4_check.sh ${1:-fin}_chk
