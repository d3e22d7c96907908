// Percentile estimation and LatencyRecorder (role of
// bvar/detail/percentile.h:49-505 and latency_recorder.h:75).
//
// Values are bucketed by floor(log2(v)) into 32 intervals; each interval keeps
// a bounded reservoir of samples plus the exact count. Threads write into
// their own agent (spinlock-free fast path); the 1 Hz sampler folds agents
// into per-second buckets that windows merge on demand.
//
// LatencyHistogram is an exact-count log-linear histogram (~1% relative
// resolution) used by the rpc_press tool / bench.py where precise p99s are
// required.
#pragma once

#include <array>
#include <atomic>
#include <cstdint>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "var/recorder.h"
#include "var/reducer.h"
#include "var/window.h"

namespace mrpc {
namespace var {

struct PercentileInterval {
    uint64_t added = 0;
    std::vector<uint32_t> samples;
    void add(uint32_t v, size_t cap);
    void merge(const PercentileInterval& o, size_t cap);
};

struct PercentileSamples {
    static const int kIntervals = 32;
    uint64_t total = 0;
    PercentileInterval iv[kIntervals];
    void add(uint32_t v, size_t cap);
    void merge(const PercentileSamples& o, size_t cap);
    uint32_t get_number(double ratio) const;
    void clear();
};

class Percentile : public Sampler {
public:
    explicit Percentile(int window_seconds = 10);
    ~Percentile();
    Percentile& operator<<(int64_t v);
    // Percentile over the window (ratio in [0,1]).
    uint32_t get_number(double ratio) const;
    PercentileSamples merged() const;
    void take_sample() override;
    int window() const { return _window; }

private:
    struct Agent;
    Agent* agent();
    int _window;
    int _id;
    uint64_t _gen;
    mutable std::mutex _mu;
    std::vector<Agent*> _agents;
    std::deque<PercentileSamples> _history;
};

class LatencyRecorder {
public:
    explicit LatencyRecorder(int window_seconds = 10);
    LatencyRecorder(const std::string& prefix, int window_seconds = 10);
    ~LatencyRecorder();
    LatencyRecorder& operator<<(int64_t latency);
    int expose(const std::string& prefix);
    void hide();

    int64_t latency() const;  // average over window
    int64_t max_latency() const;
    int64_t count() const;
    double qps() const;
    int64_t latency_percentile(double ratio) const;
    std::string latency_percentiles_json() const;
    const std::string& name() const { return _prefix; }
    int window_size() const { return _window; }

private:
    int _window;
    std::string _prefix;
    IntRecorder _latency;
    Maxer<int64_t> _max_latency;
    Percentile _percentile;
    IntRecorderWindow _latency_window;
    Window<Maxer<int64_t>> _max_latency_window;
    Adder<int64_t>* _count;
    PerSecond<Adder<int64_t>> _qps;
    std::vector<std::unique_ptr<Variable>> _exposed;
};

// Exact-count histogram with log-linear buckets (relative error ~1/128).
class LatencyHistogram {
public:
    LatencyHistogram();
    void add(int64_t v);
    void merge(const LatencyHistogram& o);
    int64_t count() const { return _count; }
    int64_t min() const { return _count ? _min : 0; }
    int64_t max() const { return _max; }
    double mean() const { return _count ? (double)_sum / _count : 0; }
    int64_t percentile(double ratio) const;
    void clear();

private:
    static int bucket_of(int64_t v);
    static int64_t bucket_value(int b);
    std::vector<uint64_t> _buckets;
    int64_t _count = 0;
    int64_t _sum = 0;
    int64_t _min = INT64_MAX;
    int64_t _max = 0;
};

}  // namespace var
}  // namespace mrpc
