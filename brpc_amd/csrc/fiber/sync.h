// Fiber-aware synchronization primitives built on butex (role of
// bthread/mutex.h, condition_variable.h, countdown_event.h, rwlock.h,
// barrier). They suspend fibers and block pthreads, so they are safe to use
// from either. Contended Mutex waits are sampled into the contention
// profiler (role of bthread ContentionProfiler, reference mutex.cpp:107-337).
#pragma once

#include <time.h>

#include <atomic>
#include <cstdint>
#include <string>

#include "base/macros.h"
#include "fiber/butex.h"

namespace mrpc {
namespace fiber {

class Mutex {
public:
    Mutex();
    ~Mutex();
    MRPC_DISALLOW_COPY(Mutex);
    void lock() {
        int expected = 0;
        if (MRPC_LIKELY(_b->compare_exchange_strong(expected, 1, std::memory_order_acquire))) return;
        lock_contended();
    }
    bool try_lock() {
        int expected = 0;
        return _b->compare_exchange_strong(expected, 1, std::memory_order_acquire);
    }
    // Returns false on timeout.
    bool timed_lock(const timespec* abstime);
    void unlock() {
        if (MRPC_UNLIKELY(_b->exchange(0, std::memory_order_release) == 2)) butex_wake(_b);
    }
    std::atomic<int>* native() { return _b; }

private:
    void lock_contended();
    std::atomic<int>* _b;  // 0 free, 1 locked, 2 contended
};

class ConditionVariable {
public:
    ConditionVariable();
    ~ConditionVariable();
    MRPC_DISALLOW_COPY(ConditionVariable);
    void wait(Mutex& m);
    // Returns ETIMEDOUT or 0
    int wait_until(Mutex& m, const timespec* abstime);
    int wait_for_us(Mutex& m, int64_t us);
    void notify_one();
    void notify_all();

private:
    std::atomic<int>* _seq;
};

class CountdownEvent {
public:
    explicit CountdownEvent(int initial = 1);
    ~CountdownEvent();
    MRPC_DISALLOW_COPY(CountdownEvent);
    void signal(int n = 1);
    void add_count(int n = 1);
    void reset(int v = 1);
    int wait();
    int timed_wait(const timespec* abstime);
    int count() const { return _b->load(std::memory_order_acquire); }

private:
    std::atomic<int>* _b;
};

class RWLock {
public:
    RWLock() : _readers(0), _writer(false) {}
    void rdlock();
    void wrlock();
    void unlock_shared();
    void unlock();
    bool try_rdlock();
    bool try_wrlock();

private:
    Mutex _m;
    ConditionVariable _cv;
    int _readers;
    bool _writer;
    int _waiting_writers = 0;
};

class Barrier {
public:
    explicit Barrier(int count) : _count(count), _arrived(0), _gen(0) {}
    // Returns true for exactly one caller per generation (the "serial" one).
    bool wait();

private:
    Mutex _m;
    ConditionVariable _cv;
    int _count;
    int _arrived;
    int64_t _gen;
};

template <typename M>
class LockGuard {
public:
    explicit LockGuard(M& m) : _m(m) { _m.lock(); }
    ~LockGuard() { _m.unlock(); }
private:
    M& _m;
};

// Contention profiler: samples contended lock waits (duration + call site).
struct ContentionSample {
    int64_t wait_ns;
    void* caller;
    int64_t count;
};
bool ContentionProfilerStart(const char* filename);
void ContentionProfilerStop();
bool IsContentionProfilerRunning();
// Text dump "caller_address count total_wait_ns" lines, most contended first.
std::string ContentionProfilerDump();
// Total contended waits observed (also exported as a metric).
int64_t ContentionCount();
// contended pthread_mutex_lock calls sampled while the profiler ran
int64_t PthreadContentionCount();

}  // namespace fiber
}  // namespace mrpc
