#!/bin/bash
# Packed-run decoder: numerics, then bandwidth and kernel times.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/${1:-bw}; rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_device_codec.py tests/test_gpu_pb_pack.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $P/pytest.log 2>&1; rc=$?
tail -3 $P/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u benchmarks/device_packed_bw.py > $P/bw.jsonl 2>&1 || exit $?
grep shape $P/bw.jsonl
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$P/kt -o kt -- python3 $GRAFT_REPO_ROOT/benchmarks/device_packed_bw.py --iters 5 > $GRAFT_REPO_ROOT/$P/kt.log 2>&1) || exit $?
find $P/kt -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-200 | head -6
