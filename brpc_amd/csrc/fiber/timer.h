// Timer thread (role of bthread/timer_thread.h, reference
// timer_thread.cpp:40,219,256,315): tasks are sharded into buckets to cut
// contention, pulled into a min-heap by one pthread, ids are versioned so
// unschedule() is O(1) and safe against reuse.
#pragma once

#include <time.h>

#include <atomic>
#include <cstdint>
#include <mutex>
#include <thread>

namespace mrpc {
namespace fiber {

class TimerThread {
public:
    typedef uint64_t TaskId;
    static const TaskId INVALID_TASK_ID = 0;
    struct Options {
        size_t num_buckets = 13;
    };
    TimerThread();
    ~TimerThread();
    int start(const Options* opt);
    void stop_and_join();
    // abstime is CLOCK_REALTIME (like pthread waits).
    TaskId schedule(void (*fn)(void*), void* arg, const timespec& abstime);
    TaskId schedule_after_us(void (*fn)(void*), void* arg, int64_t delay_us);
    // 0: unscheduled before running, 1: already ran, -1: running now, -2: invalid
    int unschedule(TaskId id);

    struct Task;
    struct Bucket;

private:
    void run();
    std::atomic<bool> _started{false};
    std::atomic<bool> _stop{false};
    Bucket* _buckets = nullptr;
    size_t _nbuckets = 0;
    std::atomic<int64_t> _nearest_run_us;
    std::atomic<int> _nsignals{0};
    std::mutex _mu;
    std::thread _thread;
};

TimerThread* get_global_timer_thread();

}  // namespace fiber
}  // namespace mrpc
