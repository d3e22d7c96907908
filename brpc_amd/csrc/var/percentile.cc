#include "var/percentile.h"

#include <algorithm>
#include <cmath>

#include "base/util.h"

namespace mrpc {
namespace var {

namespace {
const size_t kAgentCap = 128;   // samples per interval per thread per second
const size_t kGlobalCap = 254;  // samples per interval per second (like the reference)

inline int interval_of(uint32_t v) { return v == 0 ? 0 : 31 - __builtin_clz(v); }

class SpinLock {
public:
    void lock() {
        while (_f.exchange(true, std::memory_order_acquire)) {
            while (_f.load(std::memory_order_relaxed)) __builtin_ia32_pause();
        }
    }
    void unlock() { _f.store(false, std::memory_order_release); }
private:
    std::atomic<bool> _f{false};
};
}  // namespace

void PercentileInterval::add(uint32_t v, size_t cap) {
    ++added;
    if (samples.size() < cap) {
        samples.push_back(v);
    } else {
        uint64_t r = fast_rand_less_than(added);
        if (r < cap) samples[r] = v;
    }
}

void PercentileInterval::merge(const PercentileInterval& o, size_t cap) {
    if (o.added == 0) return;
    if (samples.size() + o.samples.size() <= cap) {
        samples.insert(samples.end(), o.samples.begin(), o.samples.end());
        added += o.added;
        return;
    }
    // keep proportions: each side contributes cap * its weight
    const uint64_t total = added + o.added;
    size_t from_self = (size_t)std::llround((double)cap * added / total);
    size_t from_o = cap - from_self;
    from_self = std::min(from_self, samples.size());
    from_o = std::min(from_o, o.samples.size());
    std::vector<uint32_t> out;
    out.reserve(from_self + from_o);
    std::vector<uint32_t> a = samples, b = o.samples;
    for (size_t i = 0; i < from_self; ++i) {
        size_t j = i + fast_rand_less_than(a.size() - i);
        std::swap(a[i], a[j]);
        out.push_back(a[i]);
    }
    for (size_t i = 0; i < from_o; ++i) {
        size_t j = i + fast_rand_less_than(b.size() - i);
        std::swap(b[i], b[j]);
        out.push_back(b[i]);
    }
    samples.swap(out);
    added = total;
}

void PercentileSamples::add(uint32_t v, size_t cap) {
    ++total;
    iv[interval_of(v)].add(v, cap);
}

void PercentileSamples::merge(const PercentileSamples& o, size_t cap) {
    total += o.total;
    for (int i = 0; i < kIntervals; ++i) iv[i].merge(o.iv[i], cap);
}

void PercentileSamples::clear() {
    total = 0;
    for (auto& i : iv) {
        i.added = 0;
        i.samples.clear();
    }
}

uint32_t PercentileSamples::get_number(double ratio) const {
    if (total == 0) return 0;
    if (ratio < 0) ratio = 0;
    if (ratio > 1) ratio = 1;
    uint64_t target = (uint64_t)std::ceil(ratio * total);
    if (target == 0) target = 1;
    uint64_t acc = 0;
    for (int i = 0; i < kIntervals; ++i) {
        const PercentileInterval& in = iv[i];
        if (in.added == 0) continue;
        if (acc + in.added >= target) {
            std::vector<uint32_t> s = in.samples;
            if (s.empty()) return 1u << i;
            std::sort(s.begin(), s.end());
            double pos = (double)(target - acc) / in.added * s.size();
            size_t idx = pos <= 0 ? 0 : (size_t)std::ceil(pos) - 1;
            if (idx >= s.size()) idx = s.size() - 1;
            return s[idx];
        }
        acc += in.added;
    }
    return 0xFFFFFFFFu;
}

struct Percentile::Agent : public detail::AgentBase {
    SpinLock lock;
    PercentileSamples s;
    Percentile* owner = nullptr;
    void merge_and_detach() override {
        if (!owner) return;
        std::lock_guard<std::mutex> g(owner->_mu);
        lock.lock();
        if (owner->_history.empty()) owner->_history.emplace_back();
        owner->_history.back().merge(s, kGlobalCap);
        s.clear();
        lock.unlock();
        owner->_agents.erase(std::remove(owner->_agents.begin(), owner->_agents.end(), this), owner->_agents.end());
        owner = nullptr;
    }
};

Percentile::Percentile(int window_seconds) : _window(window_seconds) {
    detail::allocate_combiner_id(&_id, &_gen);
    schedule();
}

Percentile::~Percentile() {
    unschedule();
    std::lock_guard<std::mutex> g(detail::global_agent_mutex());
    std::lock_guard<std::mutex> g2(_mu);
    for (Agent* a : _agents) a->owner = nullptr;
    _agents.clear();
    detail::free_combiner_id(_id);
}

Percentile::Agent* Percentile::agent() {
    detail::AgentBase* a = detail::get_tls_agent(_id, _gen);
    if (a) return static_cast<Agent*>(a);
    Agent* na = new Agent;
    na->gen = _gen;
    na->owner = this;
    {
        std::lock_guard<std::mutex> g(_mu);
        _agents.push_back(na);
    }
    detail::set_tls_agent(_id, na);
    return na;
}

Percentile& Percentile::operator<<(int64_t v) {
    if (v < 0) v = 0;
    uint32_t u = v > 0xFFFFFFFFLL ? 0xFFFFFFFFu : (uint32_t)v;
    Agent* a = agent();
    a->lock.lock();
    a->s.add(u, kAgentCap);
    a->lock.unlock();
    return *this;
}

void Percentile::take_sample() {
    PercentileSamples merged;
    std::lock_guard<std::mutex> g(_mu);
    for (Agent* a : _agents) {
        a->lock.lock();
        merged.merge(a->s, kGlobalCap);
        a->s.clear();
        a->lock.unlock();
    }
    _history.push_back(std::move(merged));
    while ((int)_history.size() > _window) _history.pop_front();
}

PercentileSamples Percentile::merged() const {
    PercentileSamples out;
    std::lock_guard<std::mutex> g(_mu);
    for (const auto& h : _history) out.merge(h, kGlobalCap);
    if (out.total == 0) {
        // Nothing sampled yet (first second): peek at live agents.
        for (Agent* a : _agents) {
            a->lock.lock();
            out.merge(a->s, kGlobalCap);
            a->lock.unlock();
        }
    }
    return out;
}

uint32_t Percentile::get_number(double ratio) const { return merged().get_number(ratio); }

// ---------------------------------------------------------------- LatencyRecorder

LatencyRecorder::LatencyRecorder(int window_seconds)
    : _window(window_seconds),
      _percentile(window_seconds),
      _latency_window(&_latency, window_seconds),
      _max_latency_window(&_max_latency, window_seconds),
      _count(_latency.num_adder()),
      _qps(_latency.num_adder(), window_seconds) {}

LatencyRecorder::LatencyRecorder(const std::string& prefix, int window_seconds) : LatencyRecorder(window_seconds) {
    expose(prefix);
}

LatencyRecorder::~LatencyRecorder() { hide(); }

LatencyRecorder& LatencyRecorder::operator<<(int64_t latency) {
    _latency << latency;
    _max_latency << latency;
    _percentile << latency;
    return *this;
}

int64_t LatencyRecorder::latency() const { return _latency_window.get_value().get_average_int(); }
int64_t LatencyRecorder::max_latency() const { return _max_latency_window.get_value(); }
int64_t LatencyRecorder::count() const { return _count->get_value(); }
double LatencyRecorder::qps() const { return _qps.get_value(); }
int64_t LatencyRecorder::latency_percentile(double ratio) const { return _percentile.get_number(ratio); }

std::string LatencyRecorder::latency_percentiles_json() const {
    PercentileSamples s = _percentile.merged();
    return string_printf("[%u,%u,%u,%u]", s.get_number(0.5), s.get_number(0.9), s.get_number(0.99), s.get_number(0.999));
}

void LatencyRecorder::hide() {
    _exposed.clear();
    _prefix.clear();
}

int LatencyRecorder::expose(const std::string& prefix) {
    hide();
    _prefix = normalize_name(prefix);
    auto add = [this](const std::string& suffix, std::function<double()> fn) {
        auto* v = new PassiveStatus<double>(fn);
        v->expose(_prefix + "_" + suffix);
        _exposed.emplace_back(v);
    };
    add("latency", [this] { return (double)latency(); });
    add("max_latency", [this] { return (double)max_latency(); });
    add("qps", [this] { return qps(); });
    add("count", [this] { return (double)count(); });
    add("latency_80", [this] { return (double)latency_percentile(0.8); });
    add("latency_90", [this] { return (double)latency_percentile(0.9); });
    add("latency_99", [this] { return (double)latency_percentile(0.99); });
    add("latency_999", [this] { return (double)latency_percentile(0.999); });
    add("latency_9999", [this] { return (double)latency_percentile(0.9999); });
    auto* pj = new PassiveStatus<std::string>([this] { return latency_percentiles_json(); });
    pj->expose(_prefix + "_latency_percentiles");
    _exposed.emplace_back(pj);
    return 0;
}

// ---------------------------------------------------------------- LatencyHistogram
// Bucket b: for v < 128 exact; above, 7 bits of mantissa per power of two.
static const int kSubBits = 7;
static const int kSub = 1 << kSubBits;

LatencyHistogram::LatencyHistogram() : _buckets(64 * kSub, 0) {}

int LatencyHistogram::bucket_of(int64_t v) {
    if (v < kSub) return (int)(v < 0 ? 0 : v);
    int e = 63 - __builtin_clzll((uint64_t)v);  // >= kSubBits
    int shift = e - kSubBits;
    int mant = (int)((v >> shift) & (kSub - 1));
    return (shift + 1) * kSub + mant;
}

int64_t LatencyHistogram::bucket_value(int b) {
    if (b < kSub) return b;
    int shift = b / kSub - 1;
    int mant = b % kSub;
    // midpoint of the bucket
    int64_t lo = ((int64_t)(kSub + mant)) << shift;
    return lo + ((int64_t)1 << shift) / 2;
}

void LatencyHistogram::add(int64_t v) {
    if (v < 0) v = 0;
    int b = bucket_of(v);
    if (b >= (int)_buckets.size()) b = (int)_buckets.size() - 1;
    ++_buckets[b];
    ++_count;
    _sum += v;
    if (v < _min) _min = v;
    if (v > _max) _max = v;
}

void LatencyHistogram::merge(const LatencyHistogram& o) {
    for (size_t i = 0; i < _buckets.size(); ++i) _buckets[i] += o._buckets[i];
    _count += o._count;
    _sum += o._sum;
    _min = std::min(_min, o._min);
    _max = std::max(_max, o._max);
}

int64_t LatencyHistogram::percentile(double ratio) const {
    if (_count == 0) return 0;
    uint64_t target = (uint64_t)std::ceil(ratio * _count);
    if (target == 0) target = 1;
    uint64_t acc = 0;
    for (size_t i = 0; i < _buckets.size(); ++i) {
        acc += _buckets[i];
        if (acc >= target) return std::min<int64_t>(std::max<int64_t>(bucket_value((int)i), _min), _max);
    }
    return _max;
}

void LatencyHistogram::clear() {
    std::fill(_buckets.begin(), _buckets.end(), 0);
    _count = _sum = 0;
    _min = INT64_MAX;
    _max = 0;
}

}  // namespace var
}  // namespace mrpc
