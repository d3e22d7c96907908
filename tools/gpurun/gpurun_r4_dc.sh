#!/bin/bash
# Device-payload codec checkpoint: its GPU tests, then the host cost of the
# device-body legs against the CPU codec legs (profile_leg --no-profile),
# then a kernel trace and FETCH/WRITE PMC passes (one counter group per run)
# of the device-body leg and the verified 1 MiB leg. Usage: gpurun_r4_dc.sh <tag>
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"
P=gpurun_out/${1:-dc}; rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_device_codec.py tests/test_gpu_snappy.py -x -v -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $P/pytest.log 2>&1; rc=$?
tail -3 $P/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u benchmarks/snappy_rpc_shapes.py --kinds text,random,const > $P/snappy_b7.txt 2>&1 || exit $?
timeout -k 10 240 python -u benchmarks/snappy_rpc_shapes.py --kinds text,random --bodies 50 --iters 20 \
    > $P/snappy_b50.txt 2>&1 || exit $?
for spec in dev_snappy:text dev_snappy:random grpc_cpu:text grpc_cpu:random dev_64k:text dev_1m_verify:text; do
    leg=${spec%%:*}; body=${spec##*:}
    timeout -k 10 60 python -u benchmarks/profile_leg.py --leg $leg --body $body --seconds 3 --no-profile \
        > $P/leg_${leg}_${body}.txt 2>&1 || exit $?
    head -1 $P/leg_${leg}_${body}.txt
done
cd /tmp
for leg in dev_snappy dev_1m_verify; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$P/kt_$leg" -o run -- \
        python3 "$R/benchmarks/profile_leg.py" --leg $leg --body text --seconds 2 --no-profile \
        > "$R/$P/kt_$leg.log" 2>&1 || exit $?
done
for leg in dev_snappy dev_1m_verify; do
    for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$R/$P/pmc_${c}_${leg}" -o run -- \
            python3 "$R/benchmarks/profile_leg.py" --leg $leg --body text --seconds 1 --no-profile \
            > "$R/$P/pmc_${c}_${leg}.log" 2>&1 || exit $?
    done
done
cd "$R"
for leg in dev_snappy dev_1m_verify; do
    python3 benchmarks/rocprof_summary.py $P/kt_$leg --prune > $P/kt_${leg}_summary.txt 2>&1
done
for leg in dev_snappy dev_1m_verify; do
    python3 benchmarks/rocprof_summary.py $P/pmc_FETCH_SIZE_$leg $P/pmc_WRITE_SIZE_$leg --prune \
        > $P/pmc_${leg}_summary.txt 2>&1
done
echo done
