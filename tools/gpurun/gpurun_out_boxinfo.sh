cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
{ nproc; python -c "import os; print(len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>&1; cat /proc/cpuinfo | grep "model name" | head -1; cat /proc/loadavg; uptime; } > gpurun_out/boxinfo.txt 2>&1
for w in 4 8 16; do timeout -k 10 120 python bench.py --workers $w --skip-64k --latency-sample-s 2 >> gpurun_out/bench_workers.log 2>&1 || exit 1; done
