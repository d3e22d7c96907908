#!/bin/bash
# Kernel microbench + rocprofv3 PMC passes (one counter group per run).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/gpu_kernels.py > gpurun_out/kernels.log 2>&1 || exit 1
cd /tmp
timeout -s KILL 60 rocprofv3 --list-avail > "$GRAFT_REPO_ROOT/gpurun_out/avail.txt" 2>&1 || true
export SIZES=67108864
P="$GRAFT_REPO_ROOT/gpurun_out"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/kt" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/gpu_kernels.py" > "$P/kt.log" 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d "$P/pmc_sq" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/gpu_kernels.py" > "$P/pmc_sq.log" 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P/pmc_fetch" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/gpu_kernels.py" > "$P/pmc_fetch.log" 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$P/pmc_write" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/gpu_kernels.py" > "$P/pmc_write.log" 2>&1 || exit 1
echo done
