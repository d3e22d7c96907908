#include "fiber/sync.h"

#include <dlfcn.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <map>
#include <mutex>
#include <vector>

#include "base/time.h"
#include "base/util.h"

namespace mrpc {
namespace fiber {

// ------------------------------------------------------------ contention profiler
namespace {
struct ContentionState {
    std::mutex mu;
    bool running = false;
    std::string filename;
    std::map<void*, ContentionSample> samples;
    std::atomic<int64_t> total{0};
};
ContentionState& cstate() {
    static ContentionState* s = new ContentionState;
    return *s;
}
std::atomic<bool> g_profiling{false};
// set while a thread records a sample: the recorder's own locks (which go
// through the pthread_mutex_lock interposer below) are not sampled
thread_local bool tls_in_submit = false;

void submit_contention(void* caller, int64_t wait_ns) {
    ContentionState& s = cstate();
    if (tls_in_submit) return;
    struct Guard {
        Guard() { tls_in_submit = true; }
        ~Guard() { tls_in_submit = false; }
    } in_submit;
    s.total.fetch_add(1, std::memory_order_relaxed);
    if (!g_profiling.load(std::memory_order_relaxed)) return;
    // Sample proportionally to the wait time: long waits are always kept,
    // short ones with probability wait/1ms (like the reference profiler's
    // COLLECTOR_SAMPLING_BASE weighting).
    if (wait_ns < 1000000 && (int64_t)fast_rand_less_than(1000000) > wait_ns) return;
    std::lock_guard<std::mutex> g(s.mu);
    ContentionSample& cs = s.samples[caller];
    cs.caller = caller;
    cs.wait_ns += wait_ns;
    cs.count += 1;
}
}  // namespace

bool ContentionProfilerStart(const char* filename) {
    ContentionState& s = cstate();
    std::lock_guard<std::mutex> g(s.mu);
    if (s.running) return false;
    s.running = true;
    s.filename = filename ? filename : "";
    s.samples.clear();
    g_profiling.store(true);
    return true;
}

void ContentionProfilerStop() {
    ContentionState& s = cstate();
    std::string dump;
    std::string fn;
    {
        std::lock_guard<std::mutex> g(s.mu);
        if (!s.running) return;
        s.running = false;
        g_profiling.store(false);
        fn = s.filename;
    }
    if (!fn.empty()) {
        dump = ContentionProfilerDump();
        FILE* f = fopen(fn.c_str(), "w");
        if (f) {
            fwrite(dump.data(), 1, dump.size(), f);
            fclose(f);
        }
    }
}

bool IsContentionProfilerRunning() { return g_profiling.load(); }

std::string ContentionProfilerDump() {
    ContentionState& s = cstate();
    std::vector<ContentionSample> v;
    {
        std::lock_guard<std::mutex> g(s.mu);
        for (auto& kv : s.samples) v.push_back(kv.second);
    }
    std::sort(v.begin(), v.end(), [](const ContentionSample& a, const ContentionSample& b) {
        return a.wait_ns > b.wait_ns;
    });
    std::string out = "--- contention (caller count total_wait_ns)\n";
    for (auto& cs : v) string_appendf(&out, "%p %ld %ld\n", cs.caller, (long)cs.count, (long)cs.wait_ns);
    return out;
}

int64_t ContentionCount() { return cstate().total.load(std::memory_order_relaxed); }

// ------------------------------------------------------------ pthread mutexes
// The contention profiler sees pthread mutexes too (std::mutex included):
// libmrpc defines pthread_mutex_lock, which binds ahead of libc's for every
// program linked with it (reference: src/bthread/mutex.cpp:367-423). With
// the profiler off it forwards at once; with it on, a failed try-lock means
// contention, and the time to acquire is sampled for the caller.
typedef int (*PthreadMutexOp)(pthread_mutex_t*);
static PthreadMutexOp g_sys_lock = nullptr;
static PthreadMutexOp g_sys_trylock = nullptr;
std::atomic<int64_t> g_pthread_contentions{0};

static void resolve_pthread_mutex() {
    if (!g_sys_lock) g_sys_lock = (PthreadMutexOp)dlsym(RTLD_NEXT, "pthread_mutex_lock");
    if (!g_sys_trylock) g_sys_trylock = (PthreadMutexOp)dlsym(RTLD_NEXT, "pthread_mutex_trylock");
}
__attribute__((constructor)) static void resolve_pthread_mutex_at_load() { resolve_pthread_mutex(); }

int64_t PthreadContentionCount() { return g_pthread_contentions.load(std::memory_order_relaxed); }

}  // namespace fiber
}  // namespace mrpc

extern "C" int pthread_mutex_lock(pthread_mutex_t* m) {
    using namespace mrpc::fiber;
    if (__builtin_expect(!g_sys_lock, 0)) {
        resolve_pthread_mutex();
        if (!g_sys_lock) {  // dlsym not usable yet (very early): spin on try-lock
            while (pthread_mutex_trylock(m) == EBUSY) sched_yield();
            return 0;
        }
    }
    if (!g_profiling.load(std::memory_order_relaxed) || tls_in_submit) return g_sys_lock(m);
    if (g_sys_trylock(m) == 0) return 0;
    const int64_t t0 = mrpc::monotonic_ns();
    const int rc = g_sys_lock(m);
    if (rc == 0) {
        g_pthread_contentions.fetch_add(1, std::memory_order_relaxed);
        submit_contention(__builtin_return_address(0), mrpc::monotonic_ns() - t0);
    }
    return rc;
}

namespace mrpc {
namespace fiber {

// ------------------------------------------------------------ Mutex
Mutex::Mutex() : _b(butex_create()) { _b->store(0, std::memory_order_relaxed); }
Mutex::~Mutex() { butex_destroy(_b); }

MRPC_NOINLINE void Mutex::lock_contended() {
    const int64_t t0 = monotonic_ns();
    while (_b->exchange(2, std::memory_order_acquire) != 0) {
        if (butex_wait(_b, 2, nullptr) < 0 && errno != EWOULDBLOCK && errno != EINTR) {
            // unexpected; keep trying
        }
    }
    submit_contention(__builtin_return_address(0), monotonic_ns() - t0);
}

bool Mutex::timed_lock(const timespec* abstime) {
    if (try_lock()) return true;
    while (_b->exchange(2, std::memory_order_acquire) != 0) {
        if (butex_wait(_b, 2, abstime) < 0 && errno == ETIMEDOUT) return false;
    }
    return true;
}

// ------------------------------------------------------------ ConditionVariable
ConditionVariable::ConditionVariable() : _seq(butex_create()) { _seq->store(0, std::memory_order_relaxed); }
ConditionVariable::~ConditionVariable() { butex_destroy(_seq); }

void ConditionVariable::wait(Mutex& m) {
    const int expected = _seq->load(std::memory_order_relaxed);
    m.unlock();
    butex_wait(_seq, expected, nullptr);
    // Re-acquire as contended so that wakeups are not lost for other waiters
    // requeued onto the mutex.
    while (m.native()->exchange(2, std::memory_order_acquire) != 0) butex_wait(m.native(), 2, nullptr);
}

int ConditionVariable::wait_until(Mutex& m, const timespec* abstime) {
    const int expected = _seq->load(std::memory_order_relaxed);
    m.unlock();
    int rc = 0;
    if (butex_wait(_seq, expected, abstime) < 0 && errno == ETIMEDOUT) rc = ETIMEDOUT;
    while (m.native()->exchange(2, std::memory_order_acquire) != 0) butex_wait(m.native(), 2, nullptr);
    return rc;
}

int ConditionVariable::wait_for_us(Mutex& m, int64_t us) {
    timespec ts = realtime_after_us(us);
    return wait_until(m, &ts);
}

void ConditionVariable::notify_one() {
    _seq->fetch_add(1, std::memory_order_release);
    butex_wake(_seq);
}

void ConditionVariable::notify_all() {
    _seq->fetch_add(1, std::memory_order_release);
    butex_wake_all(_seq);
}

// ------------------------------------------------------------ CountdownEvent
CountdownEvent::CountdownEvent(int initial) : _b(butex_create()) { _b->store(initial, std::memory_order_relaxed); }
CountdownEvent::~CountdownEvent() { butex_destroy(_b); }

void CountdownEvent::signal(int n) {
    // The decrement can release a waiter that destroys this event at once:
    // read the butex pointer first, never a member after the fetch_sub (the
    // butex itself is pooled, so a late wake on a recycled one is only a
    // spurious wake-up, as with bthread's countdown event).
    std::atomic<int>* const b = _b;
    const int prev = b->fetch_sub(n, std::memory_order_release);
    if (prev <= n) butex_wake_all(b);
}

void CountdownEvent::add_count(int n) { _b->fetch_add(n, std::memory_order_release); }
void CountdownEvent::reset(int v) { _b->store(v, std::memory_order_release); }

int CountdownEvent::wait() {
    for (;;) {
        const int v = _b->load(std::memory_order_acquire);
        if (v <= 0) return 0;
        if (butex_wait(_b, v, nullptr) < 0 && errno != EWOULDBLOCK && errno != EINTR) return errno;
    }
}

int CountdownEvent::timed_wait(const timespec* abstime) {
    for (;;) {
        const int v = _b->load(std::memory_order_acquire);
        if (v <= 0) return 0;
        if (butex_wait(_b, v, abstime) < 0 && errno == ETIMEDOUT) return ETIMEDOUT;
    }
}

// ------------------------------------------------------------ RWLock (writer preferring)
void RWLock::rdlock() {
    _m.lock();
    while (_writer || _waiting_writers > 0) _cv.wait(_m);
    ++_readers;
    _m.unlock();
}
bool RWLock::try_rdlock() {
    LockGuard<Mutex> g(_m);
    if (_writer || _waiting_writers > 0) return false;
    ++_readers;
    return true;
}
void RWLock::wrlock() {
    _m.lock();
    ++_waiting_writers;
    while (_writer || _readers > 0) _cv.wait(_m);
    --_waiting_writers;
    _writer = true;
    _m.unlock();
}
bool RWLock::try_wrlock() {
    LockGuard<Mutex> g(_m);
    if (_writer || _readers > 0) return false;
    _writer = true;
    return true;
}
void RWLock::unlock_shared() {
    _m.lock();
    if (--_readers == 0) _cv.notify_all();
    _m.unlock();
}
void RWLock::unlock() {
    _m.lock();
    _writer = false;
    _cv.notify_all();
    _m.unlock();
}

// ------------------------------------------------------------ Barrier
bool Barrier::wait() {
    _m.lock();
    const int64_t gen = _gen;
    if (++_arrived == _count) {
        _arrived = 0;
        ++_gen;
        _cv.notify_all();
        _m.unlock();
        return true;
    }
    while (gen == _gen) _cv.wait(_m);
    _m.unlock();
    return false;
}

}  // namespace fiber
}  // namespace mrpc
