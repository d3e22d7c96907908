#include "rpc/method_status.h"

#include "rpc/server.h"

#include "base/time.h"
#include "base/util.h"
#include "rpc/controller.h"

namespace mrpc {

MethodStatus::MethodStatus() {}
MethodStatus::~MethodStatus() {}

int MethodStatus::Expose(const std::string& prefix) {
    _latency_rec.expose(prefix);
    _concurrency_var.reset(new var::PassiveStatus<int>(prefix + "_concurrency", [this] { return concurrency(); }));
    _error_var.reset(new var::PassiveStatus<int64_t>(prefix + "_error", [this] { return nerror(); }));
    return 0;
}

int MethodStatus::SetMaxConcurrency(const AdaptiveMaxConcurrency& amc) {
    _amc = amc;
    _cl.reset(CreateConcurrencyLimiter(amc));
    return 0;
}

bool MethodStatus::OnRequested(int* rejected_cc, Controller* cntl) {
    const int cc = _nconcurrency.fetch_add(1, std::memory_order_relaxed) + 1;
    if (!_cl || _cl->OnRequested(cc, cntl)) return true;
    if (rejected_cc) *rejected_cc = cc;
    return false;
}

void MethodStatus::OnResponded(int error_code, int64_t latency_us) {
    _nconcurrency.fetch_sub(1, std::memory_order_relaxed);
    if (error_code == 0) {
        _latency_rec << latency_us;
    } else {
        _nerror << 1;
    }
    if (_cl) _cl->OnResponded(error_code, latency_us);
}

std::string MethodStatus::Describe() const {
    return string_printf("count=%lld qps=%.0f latency=%lldus p99=%lldus max=%lldus concurrency=%d error=%lld",
                         (long long)_latency_rec.count(), _latency_rec.qps(), (long long)_latency_rec.latency(),
                         (long long)_latency_rec.latency_percentile(0.99), (long long)_latency_rec.max_latency(),
                         concurrency(), (long long)nerror());
}

ConcurrencyRemover::~ConcurrencyRemover() {
    if (_status) _status->OnResponded(_c ? _c->ErrorCode() : 0, monotonic_us() - _received_us);
    if (_server) _server->RemoveConcurrency();
}

}  // namespace mrpc
