#!/bin/bash
# KFD per-process state of this user's GPU processes while a bench runs:
# queues (type, gpu) and eviction time (stats_<gpuid>/evicted_ms), sampled
# twice SECONDS apart.
#   bash benchmarks/kfd_stats.sh DELAY SECONDS -- command...
d=$1; t=$2; shift 3
"$@" &
pid=$!
snap() {
    for p in /sys/class/kfd/kfd/proc/*; do
        pp=$(basename $p)
        # host pids (another pid namespace): every process, ours among them
        ev=""
        for s in $p/stats_*; do [ -d $s ] && ev="$ev $(basename $s):evicted_ms=$(cat $s/evicted_ms 2>/dev/null),cu_occ=$(cat $s/cu_occupancy 2>/dev/null)"; done
        qs=""
        for q in $p/queues/*; do [ -d $q ] && qs="$qs $(cat $q/type 2>/dev/null)@$(cat $q/gpuid 2>/dev/null)"; done
        echo "$(date +%T.%N | cut -c1-12) pid $pp:$ev | queues:$qs"
    done
}
sleep $d; snap; sleep $t; snap
wait $pid
