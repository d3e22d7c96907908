#!/bin/bash
# GPU tests + kernel microbench + rocprof kernel summary + snappy PMC passes.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python benchmarks/gpu_kernels.py > gpurun_out/kernels.log 2>&1 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_kernels" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/gpu_kernels.py" > "$GRAFT_REPO_ROOT/gpurun_out/rocprof_kernels.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$GRAFT_REPO_ROOT/gpurun_out/pmc1" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/snappy_pmc.py" > "$GRAFT_REPO_ROOT/gpurun_out/pmc1.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU -d "$GRAFT_REPO_ROOT/gpurun_out/pmc2" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/snappy_pmc.py" > "$GRAFT_REPO_ROOT/gpurun_out/pmc2.log" 2>&1 || exit 1
echo done
