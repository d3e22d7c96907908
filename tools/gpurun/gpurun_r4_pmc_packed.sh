#!/bin/bash
# HBM bytes of the packed-run decoder (one counter group per pass).
set -u
cd "$GRAFT_REPO_ROOT"
P=gpurun_out/${1:-pmc_packed}; rm -rf $P; mkdir -p $P
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$P/fetch -o f -- python3 $GRAFT_REPO_ROOT/benchmarks/device_packed_bw.py --iters 2 --sizes-mb 64 > $GRAFT_REPO_ROOT/$P/fetch.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$P/write -o w -- python3 $GRAFT_REPO_ROOT/benchmarks/device_packed_bw.py --iters 2 --sizes-mb 64 > $GRAFT_REPO_ROOT/$P/write.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
for f in $(find $P -name '*counter_collection.csv'); do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(sys.argv[1])):
    k = (r.get("Kernel_Name", "")[:60], r.get("Counter_Name", ""))
    agg[k][0] += 1
    agg[k][1] += float(r.get("Counter_Value", 0) or 0)
for (k, c), (n, v) in sorted(agg.items()):
    if "pb_run" in k:
        print(f"{k:60s} {c:12s} dispatches={n} avg_KiB={v / max(n, 1):.0f}")
PY
done
