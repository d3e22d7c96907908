// Sampler thread, Window<> and PerSecond<> (role of bvar/window.h:174,197,
// detail/sampler.h:45): a 1 Hz sampler thread snapshots reducers; windows
// answer "value over the last N seconds" (difference for additive reducers,
// combination of per-second resets for max/min).
#pragma once

#include <deque>
#include <mutex>
#include <string>

#include "base/time.h"
#include "base/util.h"
#include "var/reducer.h"

namespace mrpc {
namespace var {

class Sampler {
public:
    virtual ~Sampler() {}
    virtual void take_sample() = 0;
    void schedule();    // register with the sampler thread
    void unschedule();  // blocks until the sampler thread is not using us
};

// Max seconds of history kept by any window.
const int kMaxWindowSeconds = 3600;

template <typename R>
class ReducerSampler : public Sampler {
public:
    typedef typename R::value_type T;
    typedef typename R::op_type Op;
    explicit ReducerSampler(R* r, int keep_seconds) : _r(r), _keep(keep_seconds) {}
    void take_sample() override {
        T v = Op::inverse_ok() ? _r->get_value() : _r->reset();
        std::lock_guard<std::mutex> g(_mu);
        _samples.push_back(Sample{monotonic_us(), v});
        while ((int)_samples.size() > _keep + 1) _samples.pop_front();
    }
    // Value over the last `window` seconds. *seconds gets the real span.
    T value_over(int window, double* seconds) const {
        std::lock_guard<std::mutex> g(_mu);
        if (Op::inverse_ok()) {
            T cur = _r->get_value();
            int64_t now = monotonic_us();
            if (_samples.empty()) {
                if (seconds) *seconds = 0;
                return cur;
            }
            size_t idx = _samples.size() > (size_t)window ? _samples.size() - 1 - window : 0;
            const Sample& old = _samples[idx];
            if (seconds) *seconds = (now - old.t_us) / 1e6;
            return Op::inverse(cur, old.v);
        }
        T r = Op::identity();
        int n = 0;
        for (auto it = _samples.rbegin(); it != _samples.rend() && n < window; ++it, ++n) r = Op::apply(r, it->v);
        if (seconds) *seconds = n;
        return r;
    }
    // series for /vars charts: per-second values, oldest first
    std::string series_json(bool per_second) const {
        std::lock_guard<std::mutex> g(_mu);
        std::string out = "[";
        for (size_t i = 1; i < _samples.size(); ++i) {
            double v;
            if (Op::inverse_ok()) {
                v = (double)Op::inverse(_samples[i].v, _samples[i - 1].v);
                if (per_second) {
                    double dt = (_samples[i].t_us - _samples[i - 1].t_us) / 1e6;
                    if (dt > 0) v /= dt;
                }
            } else {
                v = (double)_samples[i].v;
            }
            if (i > 1) out += ",";
            string_appendf(&out, "[%zu,%.6g]", i, v);
        }
        out += "]";
        return out;
    }

private:
    struct Sample {
        int64_t t_us;
        T v;
    };
    R* _r;
    int _keep;
    mutable std::mutex _mu;
    std::deque<Sample> _samples;
};

template <typename R>
class Window : public Variable {
public:
    typedef typename R::value_type value_type;
    Window(R* r, int window_seconds) : _sampler(r, window_seconds < 60 ? 60 : window_seconds), _window(window_seconds) {
        _sampler.schedule();
    }
    Window(const std::string& name, R* r, int window_seconds) : Window(r, window_seconds) { this->expose(name); }
    ~Window() {
        hide();
        _sampler.unschedule();
    }
    value_type get_value() const { return get_value(_window); }
    value_type get_value(int w) const {
        value_type v = _sampler.value_over(w, nullptr);
        if (!R::op_type::inverse_ok() && v == R::op_type::identity()) return value_type(0);
        return v;
    }
    void describe(std::ostream& os, bool) const override { os << get_value(); }
    bool get_number(double* out) const override {
        *out = (double)get_value();
        return true;
    }
    std::string series_json() const override { return _sampler.series_json(false); }
    int window_size() const { return _window; }

private:
    ReducerSampler<R> _sampler;
    int _window;
};

template <typename R>
class PerSecond : public Variable {
public:
    typedef typename R::value_type value_type;
    PerSecond(R* r, int window_seconds = 10) : _sampler(r, window_seconds < 60 ? 60 : window_seconds), _window(window_seconds) {
        _sampler.schedule();
    }
    PerSecond(const std::string& name, R* r, int window_seconds = 10) : PerSecond(r, window_seconds) { this->expose(name); }
    ~PerSecond() {
        hide();
        _sampler.unschedule();
    }
    double get_value() const { return get_value(_window); }
    double get_value(int w) const {
        double secs = 0;
        value_type v = _sampler.value_over(w, &secs);
        if (secs <= 0) return 0;
        return (double)v / secs;
    }
    void describe(std::ostream& os, bool) const override {
        double v = get_value();
        if (v == (double)(int64_t)v) os << (int64_t)v;
        else os << v;
    }
    bool get_number(double* out) const override {
        *out = get_value();
        return true;
    }
    std::string series_json() const override { return _sampler.series_json(true); }

private:
    ReducerSampler<R> _sampler;
    int _window;
};

}  // namespace var
}  // namespace mrpc
