#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
cat /proc/loadavg; nproc; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null; cat /sys/fs/cgroup/cpu.max 2>/dev/null
head -1 /proc/stat; sleep 2; head -1 /proc/stat
ps -eo pid,psr,pcpu,comm --sort=-pcpu | head -15
python - <<'PY'
import os
# per-CPU busy fraction over 2 s
def snap():
    d = {}
    for l in open('/proc/stat'):
        if l.startswith('cpu') and l[3].isdigit():
            f = l.split(); v = list(map(int, f[1:])); d[int(f[0][3:])] = (sum(v), v[3] + v[4])
    return d
import time
a = snap(); time.sleep(2); b = snap()
busy = {c: 1 - (b[c][1] - a[c][1]) / max(1, b[c][0] - a[c][0]) for c in a}
print('cpus', len(busy), 'mean busy %.1f%%' % (100 * sum(busy.values()) / len(busy)))
print('busy>20%:', sorted((c, round(100 * x)) for c, x in busy.items() if x > 0.2))
for dom in range(0, len(busy), 8):
    print('cpus %d-%d: %.1f%%' % (dom, dom + 7, 100 * sum(busy.get(c, 0) for c in range(dom, dom + 8)) / 8), end='; ')
print()
PY
