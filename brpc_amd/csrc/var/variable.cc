#include "var/variable.h"

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

std::string Variable::dump_prometheus() {
    Registry& r = reg();
    std::lock_guard<std::mutex> g(r.mu);
    std::string out;
    for (auto& kv : r.m) {
        const std::string& name = kv.first;
        // latency percentiles are emitted as a summary
        static const char* kSuffix[] = {"_latency_50", "_latency_90", "_latency_99", "_latency_999", "_latency_9999"};
        static const char* kQuant[] = {"0.5", "0.9", "0.99", "0.999", "0.9999"};
        bool handled = false;
        for (int i = 0; i < 5; ++i) {
            const std::string suf = kSuffix[i];
            if (name.size() > suf.size() && name.compare(name.size() - suf.size(), suf.size(), suf) == 0) {
                double v;
                if (kv.second.var->get_number(&v)) {
                    std::string base = name.substr(0, name.size() - suf.size()) + "_latency";
                    char line[512];
                    snprintf(line, sizeof(line), "%s{quantile=\"%s\"} %.6g\n", base.c_str(), kQuant[i], v);
                    out += line;
                }
                handled = true;
                break;
            }
        }
        if (handled) continue;
        std::string labeled;
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
        char line[512];
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
