// Wake-up probe of candidate CPUs: how promptly does a thread that sleeps
// on each CPU get to run again?
//
// On the shared MI355X hosts the tail of a paced RPC's latency is made of
// our threads being preempted or kept waiting by other tenants' tasks on
// the same CPUs (a per-L3-domain sweep: domains whose threads logged
// thousands of involuntary switches ran the 100-QPS echo at p99 300-1400 us,
// quiet ones at 32-60 us; benchmarks/latency_domains.py). How busy a domain
// looked over the previous 0.2 s barely predicted it. This measures the
// thing itself: one pinned thread per CPU sleeps `period_us` at a time and
// records how late each wake-up came, its runqueue delay
// (/proc/thread-self/schedstat) and its involuntary switches.
#include <pthread.h>
#include <sched.h>
#include <sys/prctl.h>
#include <sys/resource.h>
#include <time.h>

#include <algorithm>
#include <cstdio>
#include <thread>
#include <vector>

#include "fiber/fiber.h"

namespace mrpc {
namespace fiber {

namespace {

int64_t now_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}

void probe_one(int cpu, int duration_ms, int period_us, int late_threshold_us, CpuWakeProbe* out) {
    out->cpu = cpu;
    prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);  // measure the scheduler, not the default 50 us slack
    cpu_set_t one;
    CPU_ZERO(&one);
    CPU_SET(cpu, &one);
    if (pthread_setaffinity_np(pthread_self(), sizeof(one), &one) != 0) {
        out->wakes = -1;  // not allowed to run there
        return;
    }
    long long delay0 = 0, delay1 = 0, run0 = 0, run1 = 0;
    auto read_sched = [](long long* run, long long* delay) {
        if (FILE* f = fopen("/proc/thread-self/schedstat", "r")) {
            if (fscanf(f, "%lld %lld", run, delay) != 2) *run = *delay = 0;
            fclose(f);
        }
    };
    rusage ru0, ru1;
    getrusage(RUSAGE_THREAD, &ru0);
    read_sched(&run0, &delay0);
    std::vector<int64_t> late;
    late.reserve((size_t)duration_ms * 1000 / std::max(1, period_us) + 16);
    const int64_t end = now_ns() + (int64_t)duration_ms * 1000000;
    int64_t next = now_ns();
    while (true) {
        next += (int64_t)period_us * 1000;
        if (next > end) break;
        timespec ts{(time_t)(next / 1000000000), (long)(next % 1000000000)};
        clock_nanosleep(CLOCK_MONOTONIC, TIMER_ABSTIME, &ts, nullptr);
        const int64_t t = now_ns();
        late.push_back(std::max<int64_t>(0, t - next) / 1000);
        if (t > next) next = t;  // a long stall does not turn into a burst
    }
    read_sched(&run1, &delay1);
    getrusage(RUSAGE_THREAD, &ru1);
    out->wakes = (int64_t)late.size();
    out->run_delay_us = (delay1 - delay0) / 1000;
    out->nivcsw = ru1.ru_nivcsw - ru0.ru_nivcsw;
    out->late_over = 0;
    for (int64_t l : late) out->late_over += l > late_threshold_us ? 1 : 0;
    if (!late.empty()) {
        std::sort(late.begin(), late.end());
        out->late_p50_us = late[late.size() / 2];
        out->late_p99_us = late[std::min(late.size() - 1, late.size() * 99 / 100)];
        out->late_max_us = late.back();
    }
}

}  // namespace

std::vector<CpuWakeProbe> ProbeCpuWake(const std::vector<int>& cpus, int duration_ms, int period_us,
                                       int late_threshold_us) {
    std::vector<CpuWakeProbe> out(cpus.size());
    std::vector<std::thread> ths;
    ths.reserve(cpus.size());
    for (size_t i = 0; i < cpus.size(); ++i) {
        ths.emplace_back(probe_one, cpus[i], duration_ms, period_us, late_threshold_us, &out[i]);
    }
    for (auto& t : ths) t.join();
    return out;
}

}  // namespace fiber
}  // namespace mrpc
