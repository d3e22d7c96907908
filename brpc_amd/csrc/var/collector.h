// Speed-limited sampling framework (role of the reference's
// src/bvar/collector.h/.cpp): hot paths ask is_collectable() — a
// thread-local random draw against an adaptive sampling range — and submit()
// the sampled objects to a lock-free list. One background thread grabs the
// list every 100 ms, calls dump_and_destroy() on each object and retunes
// every speed limit so that about max_per_second objects are collected per
// second regardless of traffic. Used by rpc_dump (and available to rpcz,
// contention sampling or user code).
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>

namespace mrpc {
namespace var {

static const int COLLECTOR_SAMPLING_BASE = 16384;

struct CollectorSpeedLimit {
    explicit CollectorSpeedLimit(int64_t max_per_second) : max_per_second(max_per_second) {}
    std::atomic<int64_t> max_per_second;
    // An object is collected when a random draw in [0, BASE) falls below.
    std::atomic<int> sampling_range{COLLECTOR_SAMPLING_BASE};
    std::atomic<int64_t> submitted{0};  // in the current grab window
    std::atomic<int64_t> first_submit_us{0};
};

// Cheap test on the hot path: should this event be sampled?
bool is_collectable(CollectorSpeedLimit* sl);

class Collected {
public:
    virtual ~Collected() {}
    // Called from the collector thread; must delete/recycle *this.
    virtual void dump_and_destroy(size_t round) = 0;
    // Called instead of dump when the collector drops the object.
    virtual void destroy() { delete this; }
    virtual CollectorSpeedLimit* speed_limit() = 0;
    // Hand over to the collector thread.
    void submit();

    Collected* _next_collected = nullptr;
};

int64_t collector_dumped_count();

}  // namespace var
}  // namespace mrpc
