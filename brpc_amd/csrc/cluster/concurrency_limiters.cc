// Concurrency limiters: constant, auto (Little's-law based, reference
// docs/cn/auto_concurrency_limiter.md: max_concurrency = max_qps *
// ((2+alpha)*min_latency - latency)), timeout (reject when the expected
// queueing latency exceeds the request deadline).
#include <algorithm>
#include <cmath>
#include <map>
#include <memory>
#include <mutex>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"
#include "rpc/concurrency_limiter.h"
#include "rpc/controller.h"

DEFINE_int32(auto_cl_sample_window_size_ms, 1000, "sample window of the auto limiter");
DEFINE_int32(auto_cl_min_sample_count, 100, "min samples per window");
DEFINE_int32(auto_cl_max_sample_count, 200, "max samples per window");
DEFINE_int32(auto_cl_initial_max_concurrency, 40, "initial max concurrency of the auto limiter");
DEFINE_double(auto_cl_alpha_factor_for_ema, 0.1, "EMA smoothing factor");
DEFINE_double(auto_cl_max_explore_ratio, 0.3, "explore ratio (alpha)");
DEFINE_double(auto_cl_min_explore_ratio, 0.06, "minimal explore ratio");
DEFINE_double(auto_cl_change_rate_of_explore_ratio, 0.02, "step of explore ratio change");
DEFINE_double(auto_cl_reduce_ratio_while_remeasure, 0.9, "multiply max concurrency while remeasuring min latency");
DEFINE_int32(auto_cl_latency_fluctuation_correction_factor, 1, "latency fluctuation correction");
DEFINE_double(auto_cl_fail_punish_ratio, 1.0, "weight of failed requests' latency");
DEFINE_int32(auto_cl_noload_latency_remeasure_interval_ms, 50000, "interval of remeasuring no-load latency");
DEFINE_int32(timeout_cl_initial_avg_latency_us, 500, "initial avg latency of the timeout limiter");
DEFINE_int32(timeout_cl_max_concurrency, 100, "upper bound of the timeout limiter");
DEFINE_int32(timeout_cl_default_timeout_ms, 500, "timeout assumed when the request carries none");

namespace mrpc {

AdaptiveMaxConcurrency::AdaptiveMaxConcurrency(int v) : _value(v <= 0 ? "unlimited" : std::to_string(v)), _max(v > 0 ? v : 0) {}

AdaptiveMaxConcurrency::AdaptiveMaxConcurrency(const std::string& s) : _value(s), _max(0) {
    int64_t v;
    if (parse_int64(s, &v)) {
        _max = v > 0 ? (int)v : 0;
        _value = _max > 0 ? s : "unlimited";
    }
}

const std::string& AdaptiveMaxConcurrency::type() const {
    static const std::string kConstant = "constant", kUnlimited = "unlimited";
    if (_max > 0) return kConstant;
    if (_value == "unlimited" || _value.empty() || _value == "0") return kUnlimited;
    return _value;
}

namespace {

class ConstantLimiter : public ConcurrencyLimiter {
public:
    explicit ConstantLimiter(int max) : _max(max) {}
    bool OnRequested(int cur, Controller*) override { return cur <= _max; }
    void OnResponded(int, int64_t) override {}
    int MaxConcurrency() override { return _max; }
    ConcurrencyLimiter* New(const AdaptiveMaxConcurrency& amc) const override {
        return new ConstantLimiter(amc.max_concurrency());
    }

private:
    int _max;
};

class AutoLimiter : public ConcurrencyLimiter {
public:
    AutoLimiter()
        : _max_concurrency(FLAGS_auto_cl_initial_max_concurrency),
          _remeasure_start_us(NextResetTime(monotonic_us())),
          _reset_latency_us(0),
          _min_latency_us(-1),
          _ema_max_qps(-1),
          _explore_ratio(FLAGS_auto_cl_max_explore_ratio) {
        _w.start_us = 0;
    }
    bool OnRequested(int cur, Controller*) override { return cur <= _max_concurrency.load(std::memory_order_relaxed); }
    void OnResponded(int error_code, int64_t latency_us) override {
        const int64_t now = monotonic_us();
        std::lock_guard<std::mutex> g(_mu);
        if (_reset_latency_us > now) return;  // draining after a reduction
        if (_w.start_us == 0) _w.start_us = now;
        if (error_code == 0) {
            ++_w.succ;
            _w.succ_us += latency_us;
        } else if (error_code != ELIMIT_CODE()) {
            ++_w.fail;
            _w.fail_us += latency_us;
        }
        const int64_t elapsed = now - _w.start_us;
        const int n = _w.succ + _w.fail;
        if (n < FLAGS_auto_cl_min_sample_count) {
            if (elapsed > (int64_t)FLAGS_auto_cl_sample_window_size_ms * 1000) Reset(now);
            return;
        }
        if (elapsed < (int64_t)FLAGS_auto_cl_sample_window_size_ms * 1000 && n < FLAGS_auto_cl_max_sample_count) return;
        if (_w.succ > 0) Update(now, elapsed);
        Reset(now);
    }
    int MaxConcurrency() override { return _max_concurrency.load(std::memory_order_relaxed); }
    ConcurrencyLimiter* New(const AdaptiveMaxConcurrency&) const override { return new AutoLimiter; }

private:
    static int ELIMIT_CODE() { return 2004; }
    static int64_t NextResetTime(int64_t now) {
        return now + (int64_t)(FLAGS_auto_cl_noload_latency_remeasure_interval_ms / 2 +
                               fast_rand_less_than(FLAGS_auto_cl_noload_latency_remeasure_interval_ms / 2 + 1)) * 1000;
    }
    void Reset(int64_t now) {
        _w = Window();
        _w.start_us = now;
    }
    void Update(int64_t now, int64_t elapsed_us) {
        const double fail_punish = FLAGS_auto_cl_fail_punish_ratio * _w.fail_us;
        const int64_t avg_latency = (int64_t)std::ceil((_w.succ_us + fail_punish) / _w.succ);
        const double qps = 1e6 * _w.succ / std::max<int64_t>(elapsed_us, 1);
        const double a = FLAGS_auto_cl_alpha_factor_for_ema;
        if (_remeasure_start_us <= now) {
            // Periodically shrink to let the no-load latency be re-measured.
            _reset_latency_us = now + avg_latency * 2;
            _remeasure_start_us = NextResetTime(now);
            _max_concurrency = std::max(1, (int)(_max_concurrency * FLAGS_auto_cl_reduce_ratio_while_remeasure));
            _min_latency_us = -1;
            return;
        }
        if (_min_latency_us <= 0) _min_latency_us = avg_latency;
        else if (avg_latency < _min_latency_us) _min_latency_us = (int64_t)(avg_latency * a + _min_latency_us * (1 - a));
        if (qps >= _ema_max_qps) _ema_max_qps = qps;
        else _ema_max_qps = qps * (a / 10) + _ema_max_qps * (1 - a / 10);
        if (avg_latency <= _min_latency_us * (1.0 + FLAGS_auto_cl_min_explore_ratio * FLAGS_auto_cl_latency_fluctuation_correction_factor) ||
            qps <= _ema_max_qps / (1.0 + FLAGS_auto_cl_min_explore_ratio)) {
            _explore_ratio = std::min(FLAGS_auto_cl_max_explore_ratio, _explore_ratio + FLAGS_auto_cl_change_rate_of_explore_ratio);
        } else {
            _explore_ratio = std::max(FLAGS_auto_cl_min_explore_ratio, _explore_ratio - FLAGS_auto_cl_change_rate_of_explore_ratio);
        }
        const double next = _min_latency_us * _ema_max_qps / 1e6 * (1 + _explore_ratio);
        _max_concurrency = std::max(1, (int)std::ceil(next));
    }
    struct Window {
        int64_t start_us = 0;
        int succ = 0, fail = 0;
        int64_t succ_us = 0, fail_us = 0;
    };
    std::mutex _mu;
    Window _w;
    std::atomic<int> _max_concurrency;
    int64_t _remeasure_start_us;
    int64_t _reset_latency_us;
    int64_t _min_latency_us;
    double _ema_max_qps;
    double _explore_ratio;
};

class TimeoutLimiter : public ConcurrencyLimiter {
public:
    TimeoutLimiter() : _avg_latency_us(FLAGS_timeout_cl_initial_avg_latency_us) {}
    bool OnRequested(int cur, Controller* cntl) override {
        if (cur > FLAGS_timeout_cl_max_concurrency) return false;
        int64_t timeout_us = (int64_t)FLAGS_timeout_cl_default_timeout_ms * 1000;
        if (cntl && cntl->server_deadline_us() > 0) timeout_us = cntl->server_deadline_us() - monotonic_us();
        // queueing estimate: every in-flight request ahead costs avg latency / parallelism
        return cur * _avg_latency_us.load(std::memory_order_relaxed) / std::max(1, _parallel) <= timeout_us;
    }
    void OnResponded(int error_code, int64_t latency_us) override {
        if (error_code) return;
        int64_t avg = _avg_latency_us.load(std::memory_order_relaxed);
        _avg_latency_us.store((avg * 15 + latency_us) / 16, std::memory_order_relaxed);
    }
    int MaxConcurrency() override { return FLAGS_timeout_cl_max_concurrency; }
    ConcurrencyLimiter* New(const AdaptiveMaxConcurrency&) const override { return new TimeoutLimiter; }

private:
    std::atomic<int64_t> _avg_latency_us;
    int _parallel = 8;
};

struct LimiterRegistry {
    std::mutex mu;
    std::map<std::string, const ConcurrencyLimiter*> m;
};
LimiterRegistry& limiters() {
    static LimiterRegistry* r = new LimiterRegistry;
    return *r;
}
}  // namespace

void RegisterConcurrencyLimiter(const std::string& name, const ConcurrencyLimiter* prototype) {
    std::lock_guard<std::mutex> g(limiters().mu);
    limiters().m[name] = prototype;
}

void RegisterBuiltinConcurrencyLimiters() {
    static std::once_flag once;
    std::call_once(once, [] {
        RegisterConcurrencyLimiter("constant", new ConstantLimiter(0));
        RegisterConcurrencyLimiter("auto", new AutoLimiter);
        RegisterConcurrencyLimiter("timeout", new TimeoutLimiter);
    });
}

ConcurrencyLimiter* CreateConcurrencyLimiter(const AdaptiveMaxConcurrency& amc) {
    RegisterBuiltinConcurrencyLimiters();
    const std::string& type = amc.type();
    if (type == "unlimited") return nullptr;
    std::lock_guard<std::mutex> g(limiters().mu);
    auto it = limiters().m.find(type);
    if (it == limiters().m.end()) {
        LOG(ERROR) << "Unknown concurrency limiter `" << type << "'";
        return nullptr;
    }
    return it->second->New(amc);
}

}  // namespace mrpc
