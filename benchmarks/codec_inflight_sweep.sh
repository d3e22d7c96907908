set -o pipefail
mkdir -p gpurun_out/infl
for n in 4 6 8 3 4; do
  timeout -k 10 120 python3 bench.py --only device_snappy_64KB_text --steps 5 --warmup 1 --flag codec_batch_max_inflight=$n > gpurun_out/infl/n$n.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/infl/n$n.json').read())
k='device_snappy_64KB_text'
print('inflight=$n', d.get(k+'_qps'), d.get(k+'_p99_us'), d.get(k+'_device',{}).get('codec_step_us'), d.get(k+'_device',{}).get('codec_requests_per_launch'))"
done
