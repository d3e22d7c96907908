#!/bin/bash
# A/B of the 100-QPS latency leg (rpc_press -qps=100 analog), alternating
# default vs -fiber_worker_nap_us=50, each run its own process under a limit.
set -o pipefail
out=gpurun_out/lat100_ab; mkdir -p $out
for i in 1 2; do
  for v in default nap50; do
    extra=""; [ $v = nap50 ] && extra="--flag fiber_worker_nap_us=50"
    timeout -k 10 150 python bench.py --only latency_100qps $extra > $out/$v.$i.json 2> $out/$v.$i.err || exit $?
    python -c "
import json,sys;d=json.loads(open('$out/$v.$i.json').read().strip().splitlines()[-1])
print('$v run $i', 'p50', d.get('p50_us_at_100qps'), 'p99', d.get('p99_us_at_100qps'), 'p999', d.get('p999_us_at_100qps'), 'cpu%', d.get('cpu_pct_at_100qps'), 'before_move p99', d.get('p99_us_at_100qps_before_move'))" | tee -a $out/summary.txt
  done
done
