#!/bin/bash
# Kernel-trace A/B of the verified-pull CRC kernels on the RPC legs:
# copy_crc32c_mfma_kernel (-copy_engine_crc_mfma=true) vs the byte-table
# copy_crc32c_kernel, 64 KiB and 1 MiB HBM attachments.
#   bash benchmarks/crc_kt_ab.sh [outdir]
set -o pipefail
OUT=${1:-gpurun_out/crckt}
mkdir -p $OUT
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for leg in dev_64k_verify dev_1m_verify; do
  for m in true false; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/kt_${leg}_$m -o kt -- \
        python3 $R/benchmarks/profile_leg.py --leg $leg --seconds 2 --no-profile --flags copy_engine_crc_mfma=$m \
        > $R/$OUT/kt_${leg}_$m.log 2>&1 || exit 1
    echo "== $leg mfma=$m: $(grep '^leg=' $R/$OUT/kt_${leg}_$m.log | cut -c1-80)"
    python3 $R/benchmarks/rocprof_summary.py $R/$OUT/kt_${leg}_$m --prune 2>&1 | grep -E "copy_crc32c|batched_copy|overlap" | cut -c1-200
  done
done
