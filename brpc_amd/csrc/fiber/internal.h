// Internals of the fiber scheduler. Design parity with bthread's
// TaskControl/TaskGroup (reference src/bthread/task_control.cpp:59-400,
// task_group.cpp:118-896): per-worker Chase-Lev run queue + remote queue,
// futex parking lots, "remained" callbacks executed right after a context
// switch (so a suspending fiber is enqueued only once it is off its stack),
// stack hand-over between an ending fiber and a fresh one.
#pragma once

#include <linux/futex.h>
#include <pthread.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <deque>
#include <mutex>
#include <vector>

#include "base/flags.h"
#include "base/macros.h"
#include "fiber/fiber.h"

DECLARE_bool(fiber_signal_parked_only);

namespace mrpc {
namespace fiber {

inline int futex_wait_private(void* addr, int expected, const timespec* timeout) {
    return (int)syscall(SYS_futex, addr, FUTEX_WAIT_PRIVATE, expected, timeout, nullptr, 0);
}
inline int futex_wake_private(void* addr, int nwake) {
    return (int)syscall(SYS_futex, addr, FUTEX_WAKE_PRIVATE, nwake, nullptr, nullptr, 0);
}

// Chase-Lev work stealing deque. Owner push/pop at bottom, thieves steal top.
// Slots are relaxed atomics: a thief reads slot `top` before its CAS decides
// whether the read counted, and the owner may be rewriting that slot after a
// wrap-around; the value of a failed steal is discarded, but the read must
// still not be a data race (TSan flags it otherwise).
template <typename T>
class WorkStealingQueue {
public:
    WorkStealingQueue() : _bottom(1), _cap(0), _buf(nullptr), _top(1) {}
    ~WorkStealingQueue() { delete[] _buf; }
    void init(size_t cap) {
        _cap = cap;
        _buf = new std::atomic<T>[cap];
    }
    bool push(const T& x) {
        const size_t b = _bottom.load(std::memory_order_relaxed);
        const size_t t = _top.load(std::memory_order_acquire);
        if (b >= t + _cap) return false;
        _buf[b & (_cap - 1)].store(x, std::memory_order_relaxed);
        _bottom.store(b + 1, std::memory_order_release);
        return true;
    }
    bool pop(T* val) {
        const size_t b = _bottom.load(std::memory_order_relaxed);
        size_t t = _top.load(std::memory_order_relaxed);
        if (t >= b) return false;
        const size_t nb = b - 1;
        _bottom.store(nb, std::memory_order_relaxed);
        std::atomic_thread_fence(std::memory_order_seq_cst);
        t = _top.load(std::memory_order_relaxed);
        if (t > nb) {
            _bottom.store(b, std::memory_order_relaxed);
            return false;
        }
        *val = _buf[nb & (_cap - 1)].load(std::memory_order_relaxed);
        if (t != nb) return true;
        const bool popped = _top.compare_exchange_strong(t, t + 1, std::memory_order_seq_cst, std::memory_order_relaxed);
        _bottom.store(b, std::memory_order_relaxed);
        return popped;
    }
    bool steal(T* val) {
        size_t t = _top.load(std::memory_order_acquire);
        size_t b = _bottom.load(std::memory_order_acquire);
        if (t >= b) return false;
        do {
            std::atomic_thread_fence(std::memory_order_seq_cst);
            b = _bottom.load(std::memory_order_acquire);
            if (t >= b) return false;
            *val = _buf[t & (_cap - 1)].load(std::memory_order_relaxed);
        } while (!_top.compare_exchange_strong(t, t + 1, std::memory_order_seq_cst, std::memory_order_relaxed));
        return true;
    }
    size_t volatile_size() const {
        const size_t b = _bottom.load(std::memory_order_relaxed);
        const size_t t = _top.load(std::memory_order_relaxed);
        return b <= t ? 0 : b - t;
    }

private:
    std::atomic<size_t> _bottom;
    size_t _cap;
    std::atomic<T>* _buf;
    MRPC_CACHELINE_ALIGNED std::atomic<size_t> _top;
};

// Idle workers sleep here. Value = signal count << 1 | stopped bit.
//
// A signal only enters the kernel when a worker is parked: under load every
// worker is running or spinning, and an unconditional FUTEX_WAKE costs a
// syscall per lot tried (signal_task walks up to kParkingLots of them) on
// every ready fiber. Dekker pair, both sides seq_cst: the signaler bumps
// _pending then reads _waiters; a parker bumps _waiters then lets the
// kernel compare _pending. A signaler that saw no waiter is ordered before
// the parker's increment, so the parker's compare sees the new _pending and
// does not sleep.
class MRPC_CACHELINE_ALIGNED ParkingLot {
public:
    struct State {
        int val;
        bool stopped() const { return val & 1; }
    };
    ParkingLot() : _pending(0) {}
    int signal(int n) {
        _pending.fetch_add(n << 1, std::memory_order_seq_cst);
        if (_waiters.load(std::memory_order_seq_cst) == 0 && FLAGS_fiber_signal_parked_only) return 0;
        return futex_wake_private(&_pending, n);
    }
    // moves the state without waking anyone: a worker about to park on a
    // snapshot older than this returns from wait() at once
    void bump() { _pending.fetch_add(2, std::memory_order_seq_cst); }
    State get_state() { return State{_pending.load(std::memory_order_acquire)}; }
    void wait(const State& expected) {
        _waiters.fetch_add(1, std::memory_order_seq_cst);
        futex_wait_private(&_pending, expected.val, nullptr);
        _waiters.fetch_sub(1, std::memory_order_relaxed);
    }
    void wait_for(const State& expected, int64_t timeout_ns) {
        const timespec ts{(time_t)(timeout_ns / 1000000000), (long)(timeout_ns % 1000000000)};
        _waiters.fetch_add(1, std::memory_order_seq_cst);
        futex_wait_private(&_pending, expected.val, &ts);
        _waiters.fetch_sub(1, std::memory_order_relaxed);
    }
    void stop() {
        _pending.fetch_or(1);
        futex_wake_private(&_pending, 10000);
    }

private:
    std::atomic<int> _pending;
    std::atomic<int> _waiters{0};  // workers inside wait()/wait_for()
};

struct KeyTable;
struct ButexWaiter;
struct Stack;

struct TaskMeta {
    std::atomic<ButexWaiter*> current_waiter{nullptr};
    std::atomic<uint64_t> current_sleep{0};
    // Guards publishing current_sleep: a timer id is published only while
    // the sleep that armed it is still the fiber's current one (sleep_gen),
    // so a late publish of an old sleep can never hide a newer timer.
    std::mutex sleep_mu;
    uint64_t sleep_gen = 0;
    // set by other threads (stop/interrupt), read by the fiber's worker
    std::atomic<bool> stop{false};
    std::atomic<bool> interrupted{false};
    // the worker pthread running this fiber right now (0 while it is not
    // running): interrupt() sends it SIGURG so a blocking syscall returns
    std::atomic<pthread_t> running_on{0};
    bool is_main = false;
    std::atomic<int>* version_butex = nullptr;  // current version of this slot
    fiber_t tid = 0;
    FiberFn fn = nullptr;
    void* arg = nullptr;
    void* sp = nullptr;  // saved context
    Stack* stack = nullptr;
    Attr attr;
    KeyTable* local_storage = nullptr;
    void* span = nullptr;  // rpcz parent span (opaque)
    int64_t start_ns = 0;
    void* tsan_fiber = nullptr;  // ThreadSanitizer fiber of this context (TSan builds)
    std::mutex version_lock;
};

class TaskControl;

// Queue of fibers made runnable by threads that are not this worker (event
// dispatcher, timer, GPU poller, foreign pthreads), guarded by the group's
// _remote_mu. A power-of-two ring that only grows: no allocation per push
// once warm (std::deque allocated a node every 64 pushes).
class RemoteQueue {
public:
    RemoteQueue() : _buf(256) {}
    bool empty() const { return _n == 0; }
    size_t size() const { return _n; }
    void push_back(fiber_t t) {
        if (_n == _buf.size()) grow();
        _buf[(_head + _n) & (_buf.size() - 1)] = t;
        ++_n;
    }
    fiber_t front() const { return _buf[_head]; }
    void pop_front() {
        _head = (_head + 1) & (_buf.size() - 1);
        --_n;
    }

private:
    void grow() {
        std::vector<fiber_t> b(_buf.size() * 2);
        for (size_t i = 0; i < _n; ++i) b[i] = _buf[(_head + i) & (_buf.size() - 1)];
        _buf.swap(b);
        _head = 0;
    }
    std::vector<fiber_t> _buf;
    size_t _head = 0, _n = 0;
};

class TaskGroup {
public:
    explicit TaskGroup(TaskControl* c);
    ~TaskGroup();
    int init(size_t rq_cap);

    static int start_foreground(TaskGroup** pg, fiber_t* tid, const Attr* attr, FiberFn fn, void* arg);
    template <bool REMOTE>
    int start_background(fiber_t* tid, const Attr* attr, FiberFn fn, void* arg);

    static void sched(TaskGroup** pg);
    static void yield(TaskGroup** pg);
    static int usleep(TaskGroup** pg, uint64_t us);
    static void sched_to(TaskGroup** pg, TaskMeta* next);
    static void sched_to(TaskGroup** pg, fiber_t next_tid);
    static void sched_to_impl(TaskGroup** pg, TaskMeta* next, bool handover);
    static void ending_sched(TaskGroup** pg);
    static void task_runner(void* arg);
    static int interrupt(fiber_t tid, TaskControl* c);

    void run_main_task();
    void ready_to_run(fiber_t tid, bool nosignal = false);
    void ready_to_run_remote(fiber_t tid, bool nosignal = false);
    void flush_nosignal_tasks();
    void flush_nosignal_tasks_remote();
    bool steal_task(fiber_t* tid);
    bool spin_for_task(fiber_t* tid);
    bool wait_task(fiber_t* tid);

    void set_remained(void (*fn)(void*), void* arg) {
        _last_fn = fn;
        _last_arg = arg;
    }
    TaskMeta* current_task() const { return _cur_meta; }
    fiber_t current_tid() const { return _cur_meta->tid; }
    bool is_current_main_task() const { return _cur_meta == _main_meta; }
    TaskControl* control() const { return _control; }
    int index() const { return _index; }
    int64_t nswitch() const { return _nswitch.load(std::memory_order_relaxed); }
    int64_t idle_ns() const { return _idle_ns.load(std::memory_order_relaxed); }

    // public for the runtime's free functions
    int _index = -1;
    ParkingLot* _pl = nullptr;
    ParkingLot::State _last_pl_state{0};

private:
    friend class TaskControl;
    void run_remained();
    TaskControl* _control;
    TaskMeta* _cur_meta;
    TaskMeta* _main_meta;
    fiber_t _main_tid;
    WorkStealingQueue<fiber_t> _rq;
    std::mutex _remote_mu;
    RemoteQueue _remote_rq;
    std::atomic<int> _remote_size{0};
    void (*_last_fn)(void*) = nullptr;
    void* _last_arg = nullptr;
    int _num_nosignal = 0;
    int _remote_num_nosignal = 0;
    std::atomic<int64_t> _nswitch{0};  // written by the owner, read by stats
    uint64_t _steal_seed;
    size_t _steal_offset;
    std::atomic<int64_t> _idle_ns{0};
    int64_t _last_task_ns = 0;  // when this worker last found a fiber (0: running one)
};

class TaskControl {
public:
    static const int kParkingLots = 4;
    static const int kMaxConcurrency = 1024;
    TaskControl();
    int init(int concurrency);
    int add_workers(int n);
    int concurrency() const { return _concurrency.load(std::memory_order_acquire); }
    TaskGroup* choose_one_group();
    bool steal_task(fiber_t* tid, uint64_t* seed, size_t offset);
    void signal_task(int num_task);
    void stop_and_join();
    int64_t total_switch() const;
    int64_t total_idle_ns() const;
    std::atomic<int64_t> nfibers{0};
    std::atomic<int64_t> nsteal{0};
    int64_t start_ns;

private:
    static void* worker_thread(void* arg);
    std::mutex _mu;
    std::atomic<int> _concurrency{0};
    std::atomic<int> _ngroup{0};
    TaskGroup* _groups[kMaxConcurrency];
    std::vector<pthread_t> _workers;
    ParkingLot _pl[kParkingLots];
    bool _stop = false;
};

TaskControl* get_task_control();        // nullptr if not started
TaskControl* get_or_new_task_control();
TaskGroup* tls_group();                 // volatile TLS read (safe across switches)
TaskMeta* address_meta(fiber_t tid);
inline uint32_t tid_slot(fiber_t tid) { return (uint32_t)(tid >> 32); }
inline uint32_t tid_version(fiber_t tid) { return (uint32_t)tid; }
inline fiber_t make_tid(uint32_t version, uint32_t slot) { return ((uint64_t)slot << 32) | version; }

// Put a fiber back to a run queue from any thread (worker or not).
void ready_to_run_general(fiber_t tid, bool nosignal = false);

}  // namespace fiber
}  // namespace mrpc
