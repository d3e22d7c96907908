#include "cluster/circuit_breaker.h"

#include <cmath>
#include <memory>
#include <unordered_map>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"

DEFINE_int32(circuit_breaker_short_window_size, 1500, "short window samples");
DEFINE_int32(circuit_breaker_long_window_size, 3000, "long window samples");
DEFINE_int32(circuit_breaker_short_window_error_percent, 10, "error percent tolerated by the short window");
DEFINE_int32(circuit_breaker_long_window_error_percent, 5, "error percent tolerated by the long window");
DEFINE_int32(circuit_breaker_min_error_cost_us, 500, "ema error cost below this is reset to zero");
DEFINE_int32(circuit_breaker_max_failed_latency_mutiple, 2, "cap of the cost of a failed call (x ema latency)");
DEFINE_int32(circuit_breaker_min_isolation_duration_ms, 100, "minimal isolation");
DEFINE_int32(circuit_breaker_max_isolation_duration_ms, 30000, "maximal isolation");
DEFINE_double(circuit_breaker_epsilon_value, 0.02, "decay epsilon of the ema");

namespace mrpc {

CircuitBreaker::EmaErrorRecorder::EmaErrorRecorder(int window_size, int max_error_percent)
    : _window_size(window_size),
      _max_error_percent(max_error_percent),
      _smooth(std::pow(FLAGS_circuit_breaker_epsilon_value, 1.0 / window_size)),
      _sample_count_when_initializing(0),
      _error_count_when_initializing(0),
      _ema_error_cost(0),
      _ema_latency(0) {}

void CircuitBreaker::EmaErrorRecorder::Reset() {
    _sample_count_when_initializing = 0;
    _error_count_when_initializing = 0;
    _ema_error_cost = 0;
    _ema_latency = 0;
}

int64_t CircuitBreaker::EmaErrorRecorder::UpdateLatency(int64_t latency) {
    int64_t ema = _ema_latency.load(std::memory_order_relaxed);
    for (;;) {
        const int64_t next = ema == 0 ? latency : (int64_t)(ema * _smooth + latency * (1 - _smooth));
        if (_ema_latency.compare_exchange_weak(ema, next)) return next;
    }
}

bool CircuitBreaker::EmaErrorRecorder::UpdateErrorCost(int64_t error_cost, int64_t ema_latency) {
    if (ema_latency != 0) error_cost = std::min<int64_t>(ema_latency * FLAGS_circuit_breaker_max_failed_latency_mutiple, error_cost);
    if (error_cost != 0) {
        const int64_t cost = _ema_error_cost.fetch_add(error_cost) + error_cost;
        const double max_cost = (double)ema_latency * _window_size * (_max_error_percent / 100.0) *
                                (1.0 + FLAGS_circuit_breaker_epsilon_value);
        return cost <= max_cost;
    }
    int64_t cost = _ema_error_cost.load(std::memory_order_relaxed);
    for (;;) {
        if (cost == 0) break;
        const int64_t next = cost < FLAGS_circuit_breaker_min_error_cost_us ? 0 : (int64_t)(cost * _smooth);
        if (_ema_error_cost.compare_exchange_weak(cost, next)) break;
    }
    return true;
}

bool CircuitBreaker::EmaErrorRecorder::OnCallEnd(int error_code, int64_t latency) {
    int64_t ema_latency;
    bool healthy;
    if (error_code == 0) {
        ema_latency = UpdateLatency(latency);
        healthy = UpdateErrorCost(0, ema_latency);
    } else {
        ema_latency = _ema_latency.load(std::memory_order_relaxed);
        healthy = UpdateErrorCost(latency, ema_latency);
    }
    if (_sample_count_when_initializing.load(std::memory_order_relaxed) < _window_size &&
        _sample_count_when_initializing.fetch_add(1) < _window_size) {
        if (error_code != 0) {
            const int32_t errors = _error_count_when_initializing.fetch_add(1);
            return errors < _window_size * _max_error_percent / 100;
        }
        return true;
    }
    return healthy;
}

CircuitBreaker::CircuitBreaker()
    : _long_window(FLAGS_circuit_breaker_long_window_size, FLAGS_circuit_breaker_long_window_error_percent),
      _short_window(FLAGS_circuit_breaker_short_window_size, FLAGS_circuit_breaker_short_window_error_percent),
      _last_reset_us(monotonic_us()),
      _isolation_duration_ms(FLAGS_circuit_breaker_min_isolation_duration_ms),
      _isolated_times(0),
      _isolated_until_us(0) {}

bool CircuitBreaker::OnCallEnd(int error_code, int64_t latency_us) {
    if (isolated(monotonic_us())) return false;
    const bool ok_short = _short_window.OnCallEnd(error_code, latency_us);
    const bool ok_long = _long_window.OnCallEnd(error_code, latency_us);
    return ok_short && ok_long;
}

void CircuitBreaker::Reset() {
    _long_window.Reset();
    _short_window.Reset();
    _last_reset_us = monotonic_us();
}

void CircuitBreaker::MarkIsolated(int64_t now_us) {
    ++_isolated_times;
    // Isolated again soon after the last reset: double the duration.
    const int64_t since_reset_ms = (now_us - _last_reset_us.load()) / 1000;
    int dur = _isolation_duration_ms.load();
    if (since_reset_ms < FLAGS_circuit_breaker_max_isolation_duration_ms) {
        dur = std::min(dur * 2, FLAGS_circuit_breaker_max_isolation_duration_ms);
    } else {
        dur = FLAGS_circuit_breaker_min_isolation_duration_ms;
    }
    _isolation_duration_ms = dur;
    _isolated_until_us = now_us + (int64_t)dur * 1000;
    Reset();
}

namespace {
struct Breakers {
    std::mutex mu;
    std::unordered_map<SocketId, std::unique_ptr<CircuitBreaker>> m;
    std::atomic<int> nisolated{0};
};
Breakers& breakers() {
    static Breakers* b = new Breakers;
    return *b;
}
}  // namespace

void FeedCircuitBreaker(SocketId id, int error_code, int64_t latency_us) {
    Breakers& b = breakers();
    CircuitBreaker* cb;
    {
        std::lock_guard<std::mutex> g(b.mu);
        auto& p = b.m[id];
        if (!p) p.reset(new CircuitBreaker);
        cb = p.get();
    }
    if (!cb->OnCallEnd(error_code, latency_us)) {
        const int64_t now = monotonic_us();
        if (!cb->isolated(now)) {
            cb->MarkIsolated(now);
            b.nisolated.fetch_add(1);
            LOG(WARNING) << "CircuitBreaker isolates server " << id << " for " << cb->isolation_duration_ms() << "ms";
        }
    }
}

bool IsIsolatedByCircuitBreaker(SocketId id) {
    Breakers& b = breakers();
    if (b.nisolated.load(std::memory_order_relaxed) == 0) return false;
    std::lock_guard<std::mutex> g(b.mu);
    auto it = b.m.find(id);
    if (it == b.m.end()) return false;
    if (it->second->isolated(monotonic_us())) return true;
    return false;
}

}  // namespace mrpc
