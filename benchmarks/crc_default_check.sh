set -o pipefail
mkdir -p gpurun_out/crc3
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_device_codec.py -k "crc or verif" > gpurun_out/crc3/pytest.txt 2>&1 || { tail -30 gpurun_out/crc3/pytest.txt; exit 1; }
tail -2 gpurun_out/crc3/pytest.txt
for leg in dev_64k_verify dev_1m_verify; do
  timeout -k 10 60 python3 benchmarks/profile_leg.py --leg $leg --seconds 3 --no-profile > gpurun_out/crc3/leg_${leg}_default.txt 2>&1 || exit 1
  echo "default $(grep '^leg=' gpurun_out/crc3/leg_${leg}_default.txt | cut -c1-90)"
done
