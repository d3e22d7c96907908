#!/bin/bash
# Number-codec kernels after the load prefetch: tests, then kernel traces of the ids legs.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pb_pack.py tests/test_gpu_json.py tests/test_gpu_snappy.py > gpurun_out/pytest_k2b.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_k2b.log; [ $rc -eq 0 ] || exit $rc
./tools/gpurun/gpurun_prof_k2.sh
