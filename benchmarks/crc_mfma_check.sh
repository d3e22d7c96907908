set -o pipefail
mkdir -p gpurun_out/crc2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_codec_fused.py tests/test_gpu_device_codec.py -k "crc or fused or verif" > gpurun_out/crc2/pytest.txt 2>&1 || { tail -30 gpurun_out/crc2/pytest.txt; exit 1; }
tail -2 gpurun_out/crc2/pytest.txt
timeout -k 10 180 python3 benchmarks/gpu_kernels.py > gpurun_out/crc2/microbench.jsonl 2>&1 || exit 1
grep crc gpurun_out/crc2/microbench.jsonl
for leg in dev_64k_verify dev_1m_verify; do
  for m in true false; do
    timeout -k 10 60 python3 benchmarks/profile_leg.py --leg $leg --seconds 3 --no-profile --flags copy_engine_crc_mfma=$m > gpurun_out/crc2/leg_${leg}_$m.txt 2>&1 || exit 1
    echo "mfma=$m $(grep '^leg=' gpurun_out/crc2/leg_${leg}_$m.txt)"
  done
done
