#include "fiber/timer.h"

#include <sys/prctl.h>

#include <algorithm>
#include <climits>
#include <vector>

#include "base/logging.h"
#include "base/pool.h"
#include "base/time.h"
#include "fiber/internal.h"

namespace mrpc {
namespace fiber {

struct TimerThread::Task {
    Task* next = nullptr;
    int64_t run_us = 0;
    void (*fn)(void*) = nullptr;
    void* arg = nullptr;
    uint32_t slot = 0;
    uint32_t initial_version = 0;
    // initial: not run; initial+1: running; initial+2: finished/removed
    std::atomic<uint32_t> version{2};
};

struct MRPC_CACHELINE_ALIGNED TimerThread::Bucket {
    std::mutex mu;
    Task* head = nullptr;
    int64_t nearest_us = INT64_MAX;
};

static inline TimerThread::TaskId make_task_id(uint32_t slot, uint32_t version) {
    return ((uint64_t)slot << 32) | version;
}

TimerThread::TimerThread() : _nearest_run_us(INT64_MAX) {}

TimerThread::~TimerThread() {
    stop_and_join();
    delete[] _buckets;
}

int TimerThread::start(const Options* opt) {
    std::lock_guard<std::mutex> g(_mu);
    if (_started.load()) return 0;
    _nbuckets = opt ? opt->num_buckets : 13;
    _buckets = new Bucket[_nbuckets];
    _thread = std::thread([this] { run(); });
    _started.store(true);
    return 0;
}

void TimerThread::stop_and_join() {
    if (!_started.load() || _stop.exchange(true)) return;
    _nsignals.fetch_add(1);
    futex_wake_private(&_nsignals, 1);
    if (_thread.joinable()) _thread.join();
}

TimerThread::TaskId TimerThread::schedule(void (*fn)(void*), void* arg, const timespec& abstime) {
    if (_stop.load(std::memory_order_relaxed) || !_started.load(std::memory_order_acquire)) return INVALID_TASK_ID;
    uint32_t slot;
    Task* t = get_resource<Task>(&slot);
    if (!t) return INVALID_TASK_ID;
    t->next = nullptr;
    t->run_us = abstime.tv_sec * 1000000LL + abstime.tv_nsec / 1000;
    t->fn = fn;
    t->arg = arg;
    t->slot = slot;
    t->initial_version = t->version.load(std::memory_order_relaxed);
    const TaskId id = make_task_id(slot, t->initial_version);
    static thread_local size_t bucket_hint = (size_t)syscall(SYS_gettid) * 2654435761u;
    Bucket& b = _buckets[bucket_hint % _nbuckets];
    bool earlier = false;
    {
        std::lock_guard<std::mutex> g(b.mu);
        t->next = b.head;
        b.head = t;
        if (t->run_us < b.nearest_us) {
            b.nearest_us = t->run_us;
            earlier = true;
        }
    }
    if (earlier) {
        int64_t cur = _nearest_run_us.load(std::memory_order_relaxed);
        bool wake = false;
        while (t->run_us < cur) {
            if (_nearest_run_us.compare_exchange_weak(cur, t->run_us)) {
                wake = true;
                break;
            }
        }
        if (wake) {
            _nsignals.fetch_add(1, std::memory_order_release);
            futex_wake_private(&_nsignals, 1);
        }
    }
    return id;
}

TimerThread::TaskId TimerThread::schedule_after_us(void (*fn)(void*), void* arg, int64_t delay_us) {
    int64_t t = realtime_us() + delay_us;
    timespec ts;
    ts.tv_sec = t / 1000000;
    ts.tv_nsec = (t % 1000000) * 1000;
    return schedule(fn, arg, ts);
}

int TimerThread::unschedule(TaskId id) {
    const uint32_t slot = (uint32_t)(id >> 32);
    const uint32_t ver = (uint32_t)id;
    Task* t = address_resource<Task>(slot);
    if (!t) return -2;
    uint32_t expected = ver;
    if (t->version.compare_exchange_strong(expected, ver + 2, std::memory_order_acquire)) return 0;
    return expected == ver + 1 ? -1 : 1;
}

void TimerThread::run() {
    pthread_setname_np(pthread_self(), "mrpc_timer");
    // deadlines are kept to the microsecond: without this the kernel may
    // defer every timed futex wait by the default 50 us timer slack
    prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);
    struct Cmp {
        bool operator()(const Task* a, const Task* b) const { return a->run_us > b->run_us; }
    };
    std::vector<Task*> heap;
    while (!_stop.load(std::memory_order_relaxed)) {
        // Reset the nearest time before pulling; concurrent schedules that
        // come after will lower it again and signal us.
        _nearest_run_us.store(INT64_MAX, std::memory_order_relaxed);
        for (size_t i = 0; i < _nbuckets; ++i) {
            Bucket& b = _buckets[i];
            Task* head;
            {
                std::lock_guard<std::mutex> g(b.mu);
                head = b.head;
                b.head = nullptr;
                b.nearest_us = INT64_MAX;
            }
            while (head) {
                Task* n = head->next;
                if (head->version.load(std::memory_order_relaxed) == head->initial_version) {
                    heap.push_back(head);
                    std::push_heap(heap.begin(), heap.end(), Cmp());
                } else {
                    return_resource<Task>(head->slot);  // unscheduled already
                }
                head = n;
            }
        }
        bool pull_again = false;
        while (!heap.empty()) {
            Task* t = heap.front();
            if (_nearest_run_us.load(std::memory_order_relaxed) <= t->run_us) {
                pull_again = true;  // a newer earlier task arrived
                break;
            }
            if (realtime_us() < t->run_us) break;
            std::pop_heap(heap.begin(), heap.end(), Cmp());
            heap.pop_back();
            uint32_t expected = t->initial_version;
            if (t->version.compare_exchange_strong(expected, expected + 1, std::memory_order_acquire)) {
                t->fn(t->arg);
                t->version.store(t->initial_version + 2, std::memory_order_release);
            }
            return_resource<Task>(t->slot);
        }
        if (pull_again) continue;
        int64_t next_run = heap.empty() ? INT64_MAX : heap.front()->run_us;
        const int expected_signal = _nsignals.load(std::memory_order_acquire);
        int64_t nearest = _nearest_run_us.load(std::memory_order_acquire);
        if (nearest <= next_run) {
            continue;
        }
        if (next_run == INT64_MAX) {
            timespec ts = ns_to_timespec(100000000LL);  // 100ms safety wakeup
            futex_wait_private(&_nsignals, expected_signal, &ts);
        } else {
            int64_t now = realtime_us();
            if (next_run > now) {
                timespec ts = ns_to_timespec((next_run - now) * 1000);
                futex_wait_private(&_nsignals, expected_signal, &ts);
            }
        }
    }
    for (Task* t : heap) return_resource<Task>(t->slot);
}

TimerThread* get_global_timer_thread() {
    static TimerThread* tt = [] {
        TimerThread* t = new TimerThread;
        TimerThread::Options opt;
        t->start(&opt);
        return t;
    }();
    return tt;
}

}  // namespace fiber
}  // namespace mrpc
