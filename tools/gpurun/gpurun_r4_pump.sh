#!/bin/bash
# Codec-batch pump: the inflight=1 reproduction, the default leg, the codec tests.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/${1:-pump}; rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
for m in 1 1 2 6 6; do
  timeout -k 10 100 python -u benchmarks/profile_leg.py --leg dev_snappy --no-profile --seconds 5 --flags codec_batch_max_inflight=$m > $P/m$m.log 2>&1 || exit $?
  echo "m=$m $(grep -E '^leg=' $P/m$m.log | cut -c1-120)"; grep -E "last_error" $P/m$m.log | cut -c1-200 || true
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_device_codec.py tests/test_gpu_pb_pack.py tests/test_gpu_snappy.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $P/pytest.log 2>&1; rc=$?
tail -3 $P/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u benchmarks/device_packed_bw.py > $P/bw.jsonl 2>&1 || exit $?
cat $P/bw.jsonl
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$P/kt -o kt -- python3 $GRAFT_REPO_ROOT/benchmarks/device_packed_bw.py --iters 5 > $GRAFT_REPO_ROOT/$P/kt.log 2>&1) || exit $?
find $P/kt -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-200 | head -8
