#!/bin/bash
# The reference's other published echo figures (BASELINE.md rows besides the
# headline), re-measured with build/bin/multi_threaded_echo_main on one host:
# QPS vs client threads at 1 KB, pooled vs single connections at 16 B / 32 KB,
# and 400 fiber senders at 32 B (the TimerThread figure).
#   bash benchmarks/ref_figures.sh > gpurun_out/ref_figures.txt
set -o pipefail
B=build/bin/multi_threaded_echo_main
run() {
  echo -n "$1: "
  shift
  timeout -k 10 60 $B --duration_s 2 "$@" 2>/dev/null | grep "^qps=" || exit 1
}
for t in 1 8 64 256; do run "1KB single, $t pthreads" --thread_num $t --request_size 1024 --connection_type single; done
run "16B single, 50 pthreads" --thread_num 50 --request_size 16 --connection_type single
run "16B pooled, 50 pthreads" --thread_num 50 --request_size 16 --connection_type pooled
run "32KB single, 50 pthreads" --thread_num 50 --request_size 32768 --connection_type single
run "32KB pooled, 50 pthreads" --thread_num 50 --request_size 32768 --connection_type pooled
run "32B single, 400 fibers" --thread_num 400 --use_fiber --request_size 32 --connection_type single
# memcache client against the example's in-process binary-protocol server
# (the reference measured against memcached 1.4.15: 90k single connection)
echo -n "memcache GETs, batches of 10, 1 thread: "; timeout -k 10 60 build/bin/memcache_main --thread_num 1 --duration_s 2 2>/dev/null | grep "^load:" || exit 1
echo -n "memcache GETs, batches of 10, 4 threads: "; timeout -k 10 60 build/bin/memcache_main --thread_num 4 --duration_s 2 2>/dev/null | grep "^load:" || exit 1
# redis client against the framework's own RedisService (the reference
# measured against redis-server: batches of 10 from 1 / 50 / 200 bthreads
# ~16.9k / 38k / 29k QPS single connection, 75.6k pooled with 50)
for t in 1 50 200; do
  echo -n "redis GET batches of 10, $t fibers, single: "; timeout -k 10 60 build/bin/redis_kv_main --thread_num $t --duration_s 2 2>/dev/null | grep "^load:" || exit 1
done
echo -n "redis GET batches of 10, 50 fibers, pooled: "; timeout -k 10 60 build/bin/redis_kv_main --thread_num 50 --connection_type pooled --duration_s 2 2>/dev/null | grep "^load:" || exit 1
# thrift framed echo, framework client -> ThriftService, 60 fibers
# (the reference, docs/en/thrift.md: "hello" 300k QPS / 0.2 ms avg, "hello" x 1000 195k / 0.3 ms, 48 cores)
for r in 1 1000; do
  echo -n "thrift echo, hello x $r, 60 fibers: "; timeout -k 10 60 build/bin/thrift_extension_main --thread_num 60 --repeat $r --duration_s 2 2>/dev/null | grep "^load:" || exit 1
done
