// Clocks. Mirrors the role of butil/time.h (reference src/butil/time.h:223,315):
// cheap monotonic nanoseconds for latency accounting and realtime micros for
// spans/logs. Monotonic reads go through the vDSO (~20 ns).
#pragma once

#include <time.h>
#include <sys/time.h>
#include <cstdint>

namespace mrpc {

inline int64_t monotonic_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1000000000LL + ts.tv_nsec;
}
inline int64_t monotonic_us() { return monotonic_ns() / 1000; }
// Jiffy-resolution monotonic time (CLOCK_MONOTONIC_COARSE: a vDSO read of
// the last tick, a few ns instead of ~25): for ages and debug stamps taken on
// every fiber run, never for timeouts or latencies.
inline int64_t monotonic_coarse_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC_COARSE, &ts);
    return ts.tv_sec * 1000000000LL + ts.tv_nsec;
}
inline int64_t monotonic_ms() { return monotonic_ns() / 1000000; }

inline int64_t realtime_us() {
    timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return ts.tv_sec * 1000000LL + ts.tv_nsec / 1000;
}
inline int64_t realtime_ms() { return realtime_us() / 1000; }

inline uint64_t rdtsc() { return __builtin_ia32_rdtsc(); }

inline timespec ns_to_timespec(int64_t ns) {
    timespec ts;
    ts.tv_sec = ns / 1000000000LL;
    ts.tv_nsec = ns % 1000000000LL;
    return ts;
}

// Absolute CLOCK_REALTIME timespec `us` microseconds from now (for pthread waits).
inline timespec realtime_after_us(int64_t us) {
    int64_t t = realtime_us() + us;
    timespec ts;
    ts.tv_sec = t / 1000000;
    ts.tv_nsec = (t % 1000000) * 1000;
    return ts;
}

class Timer {
public:
    Timer() : _start(0), _stop(0) {}
    void start() { _start = monotonic_ns(); _stop = _start; }
    void stop() { _stop = monotonic_ns(); }
    int64_t n_elapsed() const { return _stop - _start; }
    int64_t u_elapsed() const { return n_elapsed() / 1000; }
    int64_t m_elapsed() const { return n_elapsed() / 1000000; }
    double s_elapsed() const { return n_elapsed() / 1e9; }
private:
    int64_t _start, _stop;
};

}  // namespace mrpc
