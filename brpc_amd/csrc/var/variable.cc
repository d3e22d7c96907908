#include "var/variable.h"

#include <cstring>

#include <set>

#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <map>
#include <mutex>
#include <thread>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"

DEFINE_bool(var_dump, false, "periodically dump exposed variables to var_dump_file");
DEFINE_int64(var_max_multi_dimension_stats_count, 20000, "max label tuples of one MultiDimension family");
DEFINE_string(var_dump_file, "monitor/mrpc.vars", "file of the periodic dump");
DEFINE_int32(var_dump_interval, 10, "seconds between dumps");
DEFINE_string(var_dump_include, "", "only dump variables matching this wildcard list");

namespace mrpc {
namespace var {

namespace {
struct Entry {
    Variable* var;
    DisplayFilter filter;
};
struct Registry {
    std::mutex mu;
    std::map<std::string, Entry> m;
};
Registry& reg() {
    static Registry* r = new Registry;
    return *r;
}
}  // namespace

std::string normalize_name(const std::string& s) {
    std::string out;
    out.reserve(s.size());
    for (char c : s) {
        if (isalnum((unsigned char)c) || c == '_') {
            out.push_back((char)tolower((unsigned char)c));
        } else if (!out.empty() && out.back() != '_') {
            out.push_back('_');
        }
    }
    while (!out.empty() && out.back() == '_') out.pop_back();
    return out;
}

static bool wildcard_one(const char* p, const char* s) {
    while (*p) {
        if (*p == '*') {
            while (*p == '*') ++p;
            if (!*p) return true;
            for (; *s; ++s) {
                if (wildcard_one(p, s)) return true;
            }
            return false;
        }
        if (!*s) return false;
        if (*p != '?' && *p != *s) return false;
        ++p;
        ++s;
    }
    return *s == 0;
}

bool wildcard_match(const std::string& pattern, const std::string& s) {
    if (pattern.empty()) return true;
    size_t b = 0;
    while (b <= pattern.size()) {
        size_t e = pattern.find_first_of(";,", b);
        if (e == std::string::npos) e = pattern.size();
        std::string one = pattern.substr(b, e - b);
        if (!one.empty() && wildcard_one(one.c_str(), s.c_str())) return true;
        b = e + 1;
    }
    return false;
}

Variable::~Variable() { hide(); }

bool Variable::get_number(double* out) const {
    std::ostringstream os;
    describe(os, false);
    const std::string s = os.str();
    char* end = nullptr;
    double v = strtod(s.c_str(), &end);
    if (end == s.c_str() || *end) return false;
    *out = v;
    return true;
}

std::string Variable::get_description() const {
    std::ostringstream os;
    describe(os, false);
    return os.str();
}

int Variable::expose_impl(const std::string& prefix, const std::string& name, DisplayFilter f) {
    hide();
    std::string full = prefix.empty() ? normalize_name(name) : normalize_name(prefix) + "_" + normalize_name(name);
    if (full.empty()) return -1;
    Registry& r = reg();
    std::lock_guard<std::mutex> g(r.mu);
    auto it = r.m.find(full);
    if (it != r.m.end()) {
        LOG(WARNING) << "variable `" << full << "' already exposed";
        return -1;
    }
    r.m[full] = Entry{this, f};
    _name = full;
    return 0;
}

bool Variable::hide() {
    if (_name.empty()) return false;
    Registry& r = reg();
    std::lock_guard<std::mutex> g(r.mu);
    auto it = r.m.find(_name);
    if (it != r.m.end() && it->second.var == this) r.m.erase(it);
    _name.clear();
    return true;
}

int Variable::count_exposed() {
    Registry& r = reg();
    std::lock_guard<std::mutex> g(r.mu);
    return (int)r.m.size();
}

void Variable::list_exposed(std::vector<std::string>* names) {
    Registry& r = reg();
    std::lock_guard<std::mutex> g(r.mu);
    names->clear();
    for (auto& kv : r.m) names->push_back(kv.first);
}

int Variable::describe_exposed(const std::string& name, std::ostream& os, bool quote_string) {
    Registry& r = reg();
    std::lock_guard<std::mutex> g(r.mu);
    auto it = r.m.find(name);
    if (it == r.m.end()) return -1;
    it->second.var->describe(os, quote_string);
    return 0;
}

std::string Variable::describe_exposed(const std::string& name) {
    std::ostringstream os;
    if (describe_exposed(name, os, false) != 0) return "";
    return os.str();
}

std::string Variable::series_exposed(const std::string& name) {
    Registry& r = reg();
    std::lock_guard<std::mutex> g(r.mu);
    auto it = r.m.find(name);
    if (it == r.m.end()) return "";
    return it->second.var->series_json();
}

int Variable::dump_exposed(std::vector<std::pair<std::string, std::string>>* out, const std::string& filter,
                           DisplayFilter display) {
    Registry& r = reg();
    std::lock_guard<std::mutex> g(r.mu);
    int n = 0;
    for (auto& kv : r.m) {
        if (!(kv.second.filter & display)) continue;
        if (!wildcard_match(filter, kv.first)) continue;
        std::ostringstream os;
        kv.second.var->describe(os, false);
        out->emplace_back(kv.first, os.str());
        ++n;
    }
    return n;
}

// A LatencyRecorder exposed as P renders as one Prometheus summary P (the
// reference's prometheus_metrics_service.cpp:103-182 grouping): quantiles
// 0.8/0.9/0.99/0.999/0.9999 from P_latency_NN, "1" from P_max_latency,
// "avg" from P_latency, P_sum = avg * count and P_count. Members of a
// complete group are not repeated as gauges; P_qps stays a gauge.
namespace {
const char* const kPctSuffix[] = {"_latency_80", "_latency_90", "_latency_99", "_latency_999", "_latency_9999"};
const char* const kPctQuantile[] = {"0.8", "0.9", "0.99", "0.999", "0.9999"};
bool ends_with(const std::string& s, const char* suf, size_t* base_len) {
    const size_t n = strlen(suf);
    if (s.size() <= n || s.compare(s.size() - n, n, suf) != 0) return false;
    *base_len = s.size() - n;
    return true;
}
struct Summary {
    double pct[5] = {0, 0, 0, 0, 0};
    int have = 0;  // bit i: percentile i; bit 5: max; bit 6: avg; bit 7: count
    double max = 0, avg = 0, count = 0;
    bool complete() const { return have == 0xFF; }
};
}  // namespace

std::string Variable::dump_prometheus() {
    Registry& r = reg();
    std::lock_guard<std::mutex> g(r.mu);
    std::map<std::string, Summary> sums;
    auto member = [](const std::string& name, std::string* base, int* bit) {
        size_t bl;
        for (int i = 0; i < 5; ++i) {
            if (ends_with(name, kPctSuffix[i], &bl)) {
                *base = name.substr(0, bl);
                *bit = i;
                return true;
            }
        }
        if (ends_with(name, "_max_latency", &bl)) *bit = 5;
        else if (ends_with(name, "_latency", &bl)) *bit = 6;
        else if (ends_with(name, "_count", &bl)) *bit = 7;
        else return false;
        *base = name.substr(0, bl);
        return true;
    };
    for (auto& kv : r.m) {
        std::string base;
        int bit;
        double v;
        if (!member(kv.first, &base, &bit) || !kv.second.var->get_number(&v)) continue;
        Summary& sm = sums[base];
        sm.have |= 1 << bit;
        if (bit < 5) sm.pct[bit] = v;
        else if (bit == 5) sm.max = v;
        else if (bit == 6) sm.avg = v;
        else sm.count = v;
    }
    std::string out;
    std::set<std::string> emitted;
    char line[512];
    for (auto& kv : r.m) {
        const std::string& name = kv.first;
        std::string base;
        int bit;
        if (member(name, &base, &bit)) {
            auto it = sums.find(base);
            if (it != sums.end() && it->second.complete()) {
                if (emitted.insert(base).second) {
                    const Summary& sm = it->second;
                    out += "# HELP " + base + "\n# TYPE " + base + " summary\n";
                    for (int i = 0; i < 5; ++i) {
                        snprintf(line, sizeof(line), "%s{quantile=\"%s\"} %.10g\n", base.c_str(), kPctQuantile[i],
                                 sm.pct[i]);
                        out += line;
                    }
                    snprintf(line, sizeof(line),
                             "%s{quantile=\"1\"} %.10g\n%s{quantile=\"avg\"} %.10g\n%s_sum %.10g\n%s_count %.10g\n",
                             base.c_str(), sm.max, base.c_str(), sm.avg, base.c_str(), sm.avg * sm.count,
                             base.c_str(), sm.count);
                    out += line;
                }
                continue;
            }
        }
        double v;
        std::ostringstream os;
        kv.second.var->describe(os, false);
        std::string desc = os.str();
        if (desc.size() > 2 && desc[0] == '#') {
            // multi-dimension variables already render prometheus lines
            out += desc.substr(1);
            if (out.back() != '\n') out.push_back('\n');
            continue;
        }
        if (!kv.second.var->get_number(&v)) continue;
        snprintf(line, sizeof(line), "# HELP %s %s\n# TYPE %s gauge\n%s %.10g\n", name.c_str(), name.c_str(),
                 name.c_str(), name.c_str(), v);
        out += line;
    }
    return out;
}

void start_dump_thread_if_needed() {
    static std::once_flag once;
    if (!FLAGS_var_dump) return;
    std::call_once(once, [] {
        std::thread([] {
            for (;;) {
                sleep((unsigned)std::max(1, FLAGS_var_dump_interval));
                if (!FLAGS_var_dump) continue;
                std::vector<std::pair<std::string, std::string>> vars;
                Variable::dump_exposed(&vars, FLAGS_var_dump_include);
                std::string path = FLAGS_var_dump_file;
                size_t slash = path.rfind('/');
                if (slash != std::string::npos) {
                    std::string dir = path.substr(0, slash);
                    std::string cmd = dir;
                    mkdir(dir.c_str(), 0755);
                }
                FILE* f = fopen((path + ".tmp").c_str(), "w");
                if (!f) continue;
                for (auto& kv : vars) fprintf(f, "%s : %s\r\n", kv.first.c_str(), kv.second.c_str());
                fclose(f);
                rename((path + ".tmp").c_str(), path.c_str());
            }
        }).detach();
    });
}

}  // namespace var
}  // namespace mrpc
