// Public API of the M:N fiber runtime (role of bthread/bthread.h:43-328,
// unstable.h:40-124).
//
// Fibers are user-level threads multiplexed on N worker pthreads with
// work-stealing run queues. Every blocking primitive (mutex, cond, join,
// timed sleep, fd wait, call-id join, and GPU event waits in gpu/stream_wait.h)
// suspends only the fiber, never the worker pthread — this is what lets RPC
// stubs, socket IO and HIP stream completions interleave on few cores.
#pragma once

#include <string>
#include <vector>

#include <time.h>

#include <cstdint>
#include <functional>

namespace mrpc {
namespace fiber {

typedef uint64_t fiber_t;
// errno returned by blocking calls of a stopped fiber (bthread's ESTOP).
static const int ESTOP = -20;
const fiber_t INVALID_FIBER = 0;

enum StackType : uint8_t {
    STACK_UNKNOWN = 0,
    STACK_PTHREAD = 1,  // run in the worker's own pthread stack (no switch)
    STACK_SMALL = 2,    // 32 KB
    STACK_NORMAL = 3,   // 1 MB
    STACK_LARGE = 4,    // 8 MB
};

enum AttrFlags : uint32_t {
    ATTR_NOSIGNAL = 1,      // don't wake workers now; call flush() later
    ATTR_INHERIT_SPAN = 2,  // inherit rpcz span of the creator
    ATTR_LOG_START_AND_FINISH = 4,
};

struct KeyTablePool;

struct Attr {
    StackType stack_type = STACK_NORMAL;
    uint32_t flags = 0;
    KeyTablePool* keytable_pool = nullptr;
    Attr() {}
    Attr(StackType t, uint32_t f) : stack_type(t), flags(f) {}
};
extern const Attr ATTR_NORMAL;
extern const Attr ATTR_SMALL;
extern const Attr ATTR_PTHREAD;

typedef void* (*FiberFn)(void*);

// Create a fiber and switch to it immediately (the caller is re-queued).
int start_urgent(fiber_t* tid, const Attr* attr, FiberFn fn, void* arg);
// Create a fiber and queue it; the caller keeps running.
int start_background(fiber_t* tid, const Attr* attr, FiberFn fn, void* arg);
// Convenience wrapper over std::function.
int start(std::function<void()> fn, bool urgent = false, const Attr* attr = nullptr, fiber_t* tid = nullptr);
// Wake workers for tasks started with ATTR_NOSIGNAL.
void flush();
int join(fiber_t tid, void** ret = nullptr);
// Mark the fiber as stopped and interrupt any blocking call (returns EINTR/ESTOP).
int stop(fiber_t tid);
bool stopped(fiber_t tid);
int interrupt(fiber_t tid);
bool exists(fiber_t tid);
int yield();
// usleep: suspends the fiber (or pthread) for `us`.
int usleep(uint64_t us);
fiber_t self();
bool in_fiber();  // true iff the caller is a fiber (not a worker's main task or a plain pthread)
int worker_index();  // -1 if not in a worker thread

int set_concurrency(int n);  // can only grow
int get_concurrency();
// Start the runtime (idempotent). Called lazily by any start_*.
int init_runtime();

// Placement on shared hosts (fiber/cpu_probe.cc, fiber/runtime.cc).
struct CpuWakeProbe {
    int cpu = -1;
    int64_t wakes = 0;  // -1: the CPU is not in our allowed set
    int64_t late_p50_us = 0, late_p99_us = 0, late_max_us = 0;
    int64_t late_over = 0;     // wake-ups later than the threshold
    int64_t run_delay_us = 0;  // runnable but not running
    int64_t nivcsw = 0;        // involuntary context switches
};
// One pinned thread per CPU sleeps period_us at a time for duration_ms.
std::vector<CpuWakeProbe> ProbeCpuWake(const std::vector<int>& cpus, int duration_ms, int period_us,
                                       int late_threshold_us);
// Re-confines every thread of the process to L3 domain k (the same
// indexing as -cpu_l3_domain) and records k in that flag; 0 on success.
int RebindL3Domain(int k);
// Tell runtime the process is about to quit (skip waiting for fibers).
void about_to_quit();

// ---- fiber-local storage
typedef uint64_t FiberKey;
int key_create(FiberKey* key, void (*dtor)(void*));
int key_create2(FiberKey* key, void (*dtor)(void*, const void*), const void* dtor_arg);
int key_delete(FiberKey key);
int setspecific(FiberKey key, void* data);
void* getspecific(FiberKey key);
// Pool of keytables so that server fibers can reuse fiber-local data
// (role of bthread_keytable_pool_*).
KeyTablePool* keytable_pool_create();
void keytable_pool_destroy(KeyTablePool* p);
size_t keytable_pool_size(KeyTablePool* p);

// ---- timers (run fn in the timer pthread; fn must be quick)
typedef uint64_t TimerId;
int timer_add(TimerId* id, const timespec& abstime, void (*fn)(void*), void* arg);
int timer_add_us(TimerId* id, int64_t delay_us, void (*fn)(void*), void* arg);
// 0: removed before run; 1: already ran or running; -1: invalid.
int timer_del(TimerId id);

// ---- fd waiting (edge/level agnostic; one-shot)
int fd_wait(int fd, unsigned epoll_events);
// Returns -1/ETIMEDOUT on timeout.
int fd_timedwait(int fd, unsigned epoll_events, const timespec* abstime);
// connect(2) that suspends the fiber while the connection is in progress.
int connect(int sockfd, const struct sockaddr* addr, unsigned addrlen, int64_t timeout_ms = -1);
int close_fd(int fd);

// ---- stats
int64_t fiber_count();
// One line per live fiber: tid, entry, arg, saved sp, stack, age (/fibers, gdb).
std::string DescribeFibers(size_t max_lines = 200);
int64_t switch_count();
int64_t steal_count();
double worker_usage();  // in worker-equivalents

}  // namespace fiber
}  // namespace mrpc
