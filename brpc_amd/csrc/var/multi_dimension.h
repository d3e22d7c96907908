// Labelled metric families (role of the reference's bvar/multi_dimension.h
// and mvariable.h).
#pragma once

#include <map>
#include <memory>
#include <mutex>
#include <ostream>
#include <string>
#include <vector>

#include "base/containers.h"
#include "base/flags.h"
#include "var/percentile.h"
#include "var/recorder.h"

DECLARE_int64(var_max_multi_dimension_stats_count);

namespace mrpc {
namespace var {

// A labelled family of metrics of type M (role of the reference's
// bvar/multi_dimension.h: MultiDimension<Adder/Maxer/IntRecorder/
// LatencyRecorder/...> with Prometheus labels). Lookups of existing label
// tuples are lock-free (DoublyBufferedData of the label map; a writer only
// appears when a tuple is created or deleted), at most
// var_max_multi_dimension_stats_count tuples exist per family, and
// describe() renders Prometheus lines (prefixed with '#' so the dumper
// forwards them verbatim): one gauge series per tuple, or for
// LatencyRecorder the whole family — <name>_latency{...,quantile="0.5".."0.9999"}
// summary, _latency (avg), _max_latency, _qps and _count.

namespace detail {
// What one tuple contributes to the Prometheus text.
template <typename M>
struct MdRender {
    static void render(std::ostream& os, const std::string& name, const std::string& labels, const M& m,
                       bool first) {
        double v = 0;
        if (!m.get_number(&v)) return;
        if (first) os << "# TYPE " << name << " gauge\n";
        os << name << "{" << labels << "} " << v << "\n";
    }
};
template <>
struct MdRender<LatencyRecorder> {
    static void render(std::ostream& os, const std::string& name, const std::string& labels,
                       const LatencyRecorder& m, bool first) {
        static const double kQ[] = {0.5, 0.9, 0.99, 0.999, 0.9999};
        static const char* kQs[] = {"0.5", "0.9", "0.99", "0.999", "0.9999"};
        const std::string sep = labels.empty() ? "" : ",";
        if (first) os << "# TYPE " << name << "_latency summary\n";
        for (int i = 0; i < 5; ++i) {
            os << name << "_latency{" << labels << sep << "quantile=\"" << kQs[i] << "\"} "
               << m.latency_percentile(kQ[i]) << "\n";
        }
        os << name << "_latency_sum{" << labels << "} " << m.latency() * m.count() << "\n";
        os << name << "_latency_count{" << labels << "} " << m.count() << "\n";
        os << name << "_max_latency{" << labels << "} " << m.max_latency() << "\n";
        os << name << "_qps{" << labels << "} " << m.qps() << "\n";
    }
};
}  // namespace detail

template <typename M>
class MultiDimension : public Variable {
public:
    typedef std::vector<std::string> Key;
    typedef std::map<Key, std::shared_ptr<M>> Map;

    MultiDimension(const std::string& name, const Key& labels) : _labels(labels) { expose(name); }
    ~MultiDimension() { hide(); }
    const Key& labels() const { return _labels; }

    // The metric of one label tuple, created on first use. nullptr when the
    // arity is wrong or the family is full.
    M* get_stats(const Key& label_values) {
        if (label_values.size() != _labels.size()) return nullptr;
        {
            typename DoublyBufferedData<Map>::ScopedPtr p;
            if (_map.Read(&p) == 0) {
                auto it = p->find(label_values);
                if (it != p->end()) return it->second.get();
            }
        }
        std::lock_guard<std::mutex> g(_create_mu);  // one creator at a time
        {
            typename DoublyBufferedData<Map>::ScopedPtr p;
            if (_map.Read(&p) == 0) {
                auto it = p->find(label_values);
                if (it != p->end()) return it->second.get();
                if ((int64_t)p->size() >= FLAGS_var_max_multi_dimension_stats_count) return nullptr;
            }
        }
        std::shared_ptr<M> m(new M);
        _map.Modify([&](Map& bg) {
            bg.emplace(label_values, m);
            return (size_t)1;
        });
        return m.get();
    }
    bool has_stats(const Key& lv) const {
        typename DoublyBufferedData<Map>::ScopedPtr p;
        return const_cast<DoublyBufferedData<Map>&>(_map).Read(&p) == 0 && p->count(lv) > 0;
    }
    // Removes the tuple; a pointer returned earlier stays valid until every
    // reader of the old map version is gone (shared ownership), so callers
    // must not keep it past the delete.
    void delete_stats(const Key& lv) {
        std::lock_guard<std::mutex> g(_create_mu);
        _map.Modify([&](Map& bg) { return (size_t)bg.erase(lv); });
    }
    void clear_stats() {
        std::lock_guard<std::mutex> g(_create_mu);
        _map.Modify([&](Map& bg) {
            bg.clear();
            return (size_t)1;
        });
    }
    size_t count_stats() const {
        typename DoublyBufferedData<Map>::ScopedPtr p;
        return const_cast<DoublyBufferedData<Map>&>(_map).Read(&p) == 0 ? p->size() : 0;
    }
    void list_stats(std::vector<Key>* out) const {
        out->clear();
        typename DoublyBufferedData<Map>::ScopedPtr p;
        if (const_cast<DoublyBufferedData<Map>&>(_map).Read(&p) != 0) return;
        for (auto& kv : *p) out->push_back(kv.first);
    }
    void describe(std::ostream& os, bool) const override {
        // snapshot the tuples, render without holding the read side
        std::vector<std::pair<Key, std::shared_ptr<M>>> snap;
        {
            typename DoublyBufferedData<Map>::ScopedPtr p;
            if (const_cast<DoublyBufferedData<Map>&>(_map).Read(&p) != 0) return;
            snap.assign(p->begin(), p->end());
        }
        os << "#";
        bool first = true;
        for (auto& kv : snap) {
            std::string labels;
            for (size_t i = 0; i < _labels.size(); ++i) {
                if (i) labels += ",";
                labels += _labels[i] + "=\"" + escape(kv.first[i]) + "\"";
            }
            detail::MdRender<M>::render(os, name(), labels, *kv.second, first);
            first = false;
        }
    }
    bool get_number(double*) const override { return false; }

private:
    static std::string escape(const std::string& v) {
        std::string o;
        for (char c : v) {
            if (c == '"' || c == '\\') o.push_back('\\');
            if (c == '\n') {
                o += "\\n";
                continue;
            }
            o.push_back(c);
        }
        return o;
    }
    Key _labels;
    std::mutex _create_mu;
    DoublyBufferedData<Map> _map;
};

}  // namespace var
}  // namespace mrpc
