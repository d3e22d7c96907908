#!/bin/bash
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/z2
mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 300 python benchmarks/latency_domains.py --seconds 4 > $P/domains.txt 2>&1 || exit $?
grep -v amdgpu.ids $P/domains.txt
timeout -k 10 300 python benchmarks/latency_domains.py --seconds 4 --env WORKER_NAP_US=50 > $P/domains_wnap.txt 2>&1 || exit $?
grep -v amdgpu.ids $P/domains_wnap.txt
