#include "var/collector.h"

#include <pthread.h>
#include <unistd.h>

#include <algorithm>
#include <mutex>
#include <thread>
#include <unordered_set>

#include "base/time.h"
#include "base/util.h"

namespace mrpc {
namespace var {

namespace {
std::atomic<Collected*> g_head{nullptr};
std::atomic<int64_t> g_dumped{0};
std::once_flag g_once;

void collector_loop() {
    pthread_setname_np(pthread_self(), "mrpc_collector");
    size_t round = 0;
    for (;;) {
        usleep(100000);
        ++round;
        Collected* list = g_head.exchange(nullptr, std::memory_order_acquire);
        // Retune the limits of everything seen this round: keep the
        // collected rate near max_per_second.
        std::unordered_set<CollectorSpeedLimit*> limits;
        while (list) {
            Collected* next = list->_next_collected;
            limits.insert(list->speed_limit());
            list->dump_and_destroy(round);
            g_dumped.fetch_add(1, std::memory_order_relaxed);
            list = next;
        }
        const int64_t now = monotonic_us();
        for (CollectorSpeedLimit* sl : limits) {
            const int64_t n = sl->submitted.exchange(0, std::memory_order_relaxed);
            const int64_t since = sl->first_submit_us.exchange(now, std::memory_order_relaxed);
            const double secs = since ? std::max(0.1, (now - since) / 1e6) : 0.1;
            const double rate = n / secs;
            const int64_t want = sl->max_per_second.load(std::memory_order_relaxed);
            int range = sl->sampling_range.load(std::memory_order_relaxed);
            if (rate > 0 && want > 0) {
                // new_range = range * want / rate, moved halfway to damp oscillation
                const double target = range * (double)want / rate;
                range = (int)std::min<double>(COLLECTOR_SAMPLING_BASE, std::max(1.0, (range + target) / 2));
                sl->sampling_range.store(range, std::memory_order_relaxed);
            }
        }
    }
}

void start_collector() {
    std::call_once(g_once, [] { std::thread(collector_loop).detach(); });
}
}  // namespace

bool is_collectable(CollectorSpeedLimit* sl) {
    const int range = sl->sampling_range.load(std::memory_order_relaxed);
    if (range >= COLLECTOR_SAMPLING_BASE) return true;
    return (int)fast_rand_less_than(COLLECTOR_SAMPLING_BASE) < range;
}

void Collected::submit() {
    start_collector();
    CollectorSpeedLimit* sl = speed_limit();
    if (sl->submitted.fetch_add(1, std::memory_order_relaxed) == 0) {
        int64_t zero = 0;
        sl->first_submit_us.compare_exchange_strong(zero, monotonic_us());
    }
    Collected* head = g_head.load(std::memory_order_relaxed);
    do {
        _next_collected = head;
    } while (!g_head.compare_exchange_weak(head, this, std::memory_order_release, std::memory_order_relaxed));
}

int64_t collector_dumped_count() { return g_dumped.load(std::memory_order_relaxed); }

}  // namespace var
}  // namespace mrpc
