#!/bin/bash
# Round-3 GPU pass: new GPU tests first, then the whole -m gpu suite, smoke, a 1-GPU bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/e
P="$GRAFT_REPO_ROOT/gpurun_out/e"
export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "$P/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step park_dmabuf 300 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "park or dmabuf"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 600 python bench.py
echo done
