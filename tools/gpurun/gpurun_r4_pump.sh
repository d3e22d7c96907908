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
tail -3 $P/pytest.log; exit $rc
