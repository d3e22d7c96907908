#!/bin/bash
# Lists the KFD user queues of every process of this user while a command
# runs: /sys/class/kfd/kfd/proc/<pid>/queues/<qid>/{type,gpuid,size}.
#   bash benchmarks/kfd_queues.sh SECONDS -- command...
t=$1; shift; shift
"$@" &
pid=$!
sleep $t
for p in /sys/class/kfd/kfd/proc/*; do
    pp=$(basename $p)
    [ -d /proc/$pp ] || continue
    n=$(ls $p/queues 2>/dev/null | wc -l)
    echo "pid $pp ($(tr '\0' ' ' < /proc/$pp/cmdline | cut -c1-80)): $n queues"
    for q in $p/queues/*; do
        [ -d $q ] || continue
        echo "   q$(basename $q) type=$(cat $q/type 2>/dev/null) size=$(cat $q/size 2>/dev/null)"
    done
done
wait $pid
