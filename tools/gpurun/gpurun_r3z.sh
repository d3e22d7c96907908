#!/bin/bash
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/z
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_snappy.py tests/test_snappy_vectors.py > $P/pytest.log 2>&1; rc=$?; tail -5 $P/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/profile_leg.py --leg grpc_gpu --seconds 3 --top 60 > $P/grpc_gpu.txt 2>&1 || exit $?
timeout -k 10 120 python benchmarks/profile_leg.py --leg grpc_cpu --seconds 3 --top 60 > $P/grpc_cpu.txt 2>&1 || exit $?
head -3 $P/grpc_gpu.txt $P/grpc_cpu.txt
timeout -k 10 400 python benchmarks/latency_domains.py --seconds 4 > $P/domains.txt 2>&1; rc=$?; grep -v amdgpu.ids $P/domains.txt; exit $rc
