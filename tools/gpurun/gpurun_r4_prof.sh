#!/bin/bash
# Kernel traces (names kept) of the RPC legs that launch kernels: 64 KiB HBM
# echo, the GPU handler, and the gRPC GPU codec on text bodies.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/r4prof; rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
for leg in dev_64k gpu_handler grpc_gpu; do
  cd /tmp
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$P/$leg" -o run -- python3 "$GRAFT_REPO_ROOT/benchmarks/profile_leg.py" --leg $leg --seconds 2 --no-profile > "$GRAFT_REPO_ROOT/$P/$leg.log" 2>&1 || exit $?
  cd "$GRAFT_REPO_ROOT"
  grep '^leg=' $P/$leg.log
  python3 benchmarks/rocprof_summary.py $P/$leg --prune > $P/${leg}_summary.txt 2>&1
  head -12 $P/${leg}_summary.txt
done
echo done
