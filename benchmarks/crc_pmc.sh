#!/bin/bash
# Where the verified lending path's CRC kernel stands against HBM (VERDICT r5
# #6): the copy+CRC32C kernel on the -verify_device_payload legs (64 KiB and
# 1 MiB HBM attachments), kernel trace for durations, then one PMC pass per
# TCC counter group (FETCH_SIZE and WRITE_SIZE do not fit one pass).
#   bash benchmarks/crc_pmc.sh [outdir]
set -o pipefail
OUT=${1:-gpurun_out/crc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
cd - > /dev/null
for leg in dev_64k_verify dev_1m_verify; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$leg -o kt -- \
        python3 benchmarks/profile_leg.py --leg $leg --seconds 2 --no-profile > $OUT/kt_$leg.log 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_$leg -o f -- \
        python3 benchmarks/profile_leg.py --leg $leg --seconds 1 --no-profile > $OUT/fetch_$leg.log 2>&1 || exit 1
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write_$leg -o w -- \
        python3 benchmarks/profile_leg.py --leg $leg --seconds 1 --no-profile > $OUT/write_$leg.log 2>&1 || exit 1
done
for leg in dev_64k_verify dev_1m_verify; do
    python3 benchmarks/rocprof_summary.py $OUT/kt_$leg $OUT/fetch_$leg $OUT/write_$leg --prune
done > $OUT/summary.txt 2>&1
timeout -k 10 120 python3 benchmarks/gpu_kernels.py > $OUT/microbench.jsonl 2>&1
exit 0
