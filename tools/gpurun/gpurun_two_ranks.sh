#!/bin/bash
# Two ranks on the box's one GPU through torch.distributed.run: every N>1 leg
# (fan-out, scatter, route, streams, codec and ids legs) must complete.
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/two; rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 > $P/bench.log 2>&1; rc=$?
grep '^{"metric"' $P/bench.log > $P/bench.json
tail -3 $P/bench.log | cut -c1-300
exit $rc
