// Per-method server statistics + admission (role of
// src/brpc/details/method_status.h:33-111): concurrency, latency recorder
// (qps / avg / p50..p99.99), error count and the concurrency limiter hook.
#pragma once

#include <atomic>
#include <memory>
#include <string>

#include "rpc/concurrency_limiter.h"
#include "var/var.h"

namespace mrpc {

class Controller;
class Server;

class MethodStatus {
public:
    MethodStatus();
    ~MethodStatus();
    int Expose(const std::string& prefix);
    // Returns false (and sets *rejected) if the limiter rejects.
    bool OnRequested(int* rejected_cc = nullptr, Controller* cntl = nullptr);
    void OnResponded(int error_code, int64_t latency_us);
    int SetMaxConcurrency(const AdaptiveMaxConcurrency& amc);
    const AdaptiveMaxConcurrency& max_concurrency() const { return _amc; }
    int concurrency() const { return _nconcurrency.load(std::memory_order_relaxed); }
    var::LatencyRecorder& latency_rec() { return _latency_rec; }
    int64_t nerror() const { return _nerror.get_value(); }
    int64_t nprocessing() const { return concurrency(); }
    std::string Describe() const;

private:
    std::atomic<int> _nconcurrency{0};
    var::LatencyRecorder _latency_rec;
    var::Adder<int64_t> _nerror;
    AdaptiveMaxConcurrency _amc;
    std::unique_ptr<ConcurrencyLimiter> _cl;
    std::unique_ptr<var::PassiveStatus<int>> _concurrency_var;
    std::unique_ptr<var::PassiveStatus<int64_t>> _error_var;
};

// RAII: calls OnResponded on destruction (used by protocols).
class ConcurrencyRemover {
public:
    // `server` (when the request was counted in the server's concurrency)
    // is decremented LAST, after the method status was updated: Server::Join
    // waits for that count to drain before the statuses may be destroyed.
    ConcurrencyRemover(MethodStatus* s, Controller* c, int64_t received_us, Server* server = nullptr)
        : _status(s), _server(server), _c(c), _received_us(received_us) {}
    ~ConcurrencyRemover();
private:
    MethodStatus* _status;
    Server* _server;
    Controller* _c;
    int64_t _received_us;
};

}  // namespace mrpc
