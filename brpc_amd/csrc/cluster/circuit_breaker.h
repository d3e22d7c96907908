// CircuitBreaker (role of src/brpc/circuit_breaker.cpp:28-230): two
// EMA error-cost recorders (short window 1500 samples / 10%, long window
// 3000 / 5%); when either trips, the server is isolated for a duration that
// doubles on repeated trips (100 ms .. 30 s). Fed from Controller call
// completion when ChannelOptions.enable_circuit_breaker is set.
#pragma once

#include <atomic>
#include <cstdint>
#include <mutex>

#include "net/socket.h"

namespace mrpc {

class CircuitBreaker {
public:
    CircuitBreaker();
    // Returns false when the call makes the breaker trip.
    bool OnCallEnd(int error_code, int64_t latency_us);
    void Reset();
    bool isolated(int64_t now_us) const { return now_us < _isolated_until_us.load(std::memory_order_relaxed); }
    int isolation_duration_ms() const { return _isolation_duration_ms.load(); }
    int64_t isolated_times() const { return _isolated_times.load(); }
    void MarkIsolated(int64_t now_us);

private:
    class EmaErrorRecorder {
    public:
        EmaErrorRecorder(int window_size, int max_error_percent);
        bool OnCallEnd(int error_code, int64_t latency);
        void Reset();
    private:
        int64_t UpdateLatency(int64_t latency);
        bool UpdateErrorCost(int64_t error_cost, int64_t ema_latency);
        const int _window_size;
        const int _max_error_percent;
        const double _smooth;
        std::atomic<int32_t> _sample_count_when_initializing;
        std::atomic<int32_t> _error_count_when_initializing;
        std::atomic<int64_t> _ema_error_cost;
        std::atomic<int64_t> _ema_latency;
    };
    EmaErrorRecorder _long_window;
    EmaErrorRecorder _short_window;
    std::atomic<int64_t> _last_reset_us;
    std::atomic<int> _isolation_duration_ms;
    std::atomic<int64_t> _isolated_times;
    std::atomic<int64_t> _isolated_until_us;
};

// Per-server breakers keyed by SocketId.
void FeedCircuitBreaker(SocketId id, int error_code, int64_t latency_us);
bool IsIsolatedByCircuitBreaker(SocketId id);

}  // namespace mrpc
