#include <dlfcn.h>
// Builtin HTTP pages installed on every server (role of the reference's
// src/brpc/builtin/*: index, status, vars, flags, connections, rpcz,
// health, version, list, threads, vlog, bthreads, ids, sockets, protobufs,
// hotspots, pprof, dir, prometheus metrics; server.cpp:459-555 adds them).
// Pages answer in plain text (or HTML for /index); every one is a pb
// service with an empty request/response whose body is the attachment, so
// they are reachable over http on the same port as RPC traffic.
#include <dirent.h>
#include <malloc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <ctime>
#include <fstream>
#include <sstream>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"
#include "builtin/cpu_profiler.h"
#include "fiber/call_id.h"
#include "fiber/fiber.h"
#include "fiber/sync.h"
#include "gpu/gpu.h"
#include "rdma/rdma.h"
#include "http/http_header.h"
#include "mrpc/proto/builtin_service.pb.h"
#include "net/socket.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/health_reporter.h"
#include "rpc/method_status.h"
#include "rpc/server.h"
#include "rpc/span.h"
#include "rpc/span_db.h"
#include "var/var.h"

DEFINE_bool(enable_dir_service, false, "enable /dir (browse the file system)");
DEFINE_bool(enable_threads_service, false, "enable /threads (per-thread states)");
DECLARE_bool(enable_rpcz);

namespace mrpc {
namespace builtin {

namespace {

const char* kText = "text/plain; charset=utf-8";

Controller* C(RpcController* c) { return static_cast<Controller*>(c); }

void text(Controller* cntl, const std::string& s) {
    cntl->http_response().set_content_type(kText);
    cntl->response_attachment().append(s);
}

const std::string& unresolved(Controller* cntl) { return cntl->http_request().unresolved_path(); }

const std::string* query(Controller* cntl, const char* k) { return cntl->http_request().uri().GetQuery(k); }

std::string fmt_time(int64_t real_us) {
    time_t t = (time_t)(real_us / 1000000);
    struct tm tm;
    localtime_r(&t, &tm);
    char buf[64];
    strftime(buf, sizeof(buf), "%Y/%m/%d-%H:%M:%S", &tm);
    return buf;
}

std::string html_escape(const std::string& in) {
    std::string out;
    out.reserve(in.size());
    for (char c : in) {
        switch (c) {
        case '<': out += "&lt;"; break;
        case '>': out += "&gt;"; break;
        case '&': out += "&amp;"; break;
        case '"': out += "&quot;"; break;
        default: out += c;
        }
    }
    return out;
}

// Values of a series_json() array ("[[i,v],[i,v],...]"), in order.
std::vector<double> series_values(const std::string& json) {
    std::vector<double> v;
    const char* p = json.c_str();
    while ((p = strchr(p, '[')) != nullptr) {
        ++p;
        if (*p == '[') continue;  // the outer bracket
        const char* comma = strchr(p, ',');
        if (!comma) break;
        char* end = nullptr;
        const double x = strtod(comma + 1, &end);
        if (end == comma + 1) break;
        v.push_back(x);
        p = end;
    }
    return v;
}

// The series as an inline SVG line chart (no scripts, no downloads: the
// role of the reference's flot views, builtin/vars_service.cpp:40-75 and
// flot_min_js.cpp): the newest sample on the right, min/max/last labelled.
std::string svg_chart(const std::vector<double>& v, int w, int h, bool labels) {
    std::ostringstream os;
    os << "<svg xmlns=\"http://www.w3.org/2000/svg\" width=\"" << w << "\" height=\"" << h << "\" viewBox=\"0 0 "
       << w << " " << h << "\"><rect width=\"" << w << "\" height=\"" << h << "\" fill=\"#f8f8f8\" stroke=\"#ccc\"/>";
    if (v.size() >= 2) {
        double lo = v[0], hi = v[0];
        for (double x : v) {
            lo = std::min(lo, x);
            hi = std::max(hi, x);
        }
        const double span = hi > lo ? hi - lo : 1.0;
        const int pad = labels ? 16 : 2;
        os << "<polyline fill=\"none\" stroke=\"#1f77b4\" stroke-width=\"1.5\" points=\"";
        for (size_t i = 0; i < v.size(); ++i) {
            const double x = pad + (double)(w - 2 * pad) * i / (v.size() - 1);
            const double y = (h - pad) - (double)(h - 2 * pad) * (v[i] - lo) / span;
            os << (i ? " " : "") << (int)x << "," << (int)y;
        }
        os << "\"/>";
        if (labels) {
            os << "<text x=\"2\" y=\"12\" font-size=\"11\">max " << hi << "</text>"
               << "<text x=\"2\" y=\"" << h - 3 << "\" font-size=\"11\">min " << lo << "</text>"
               << "<text x=\"" << w - 120 << "\" y=\"12\" font-size=\"11\">last " << v.back() << "</text>";
        }
    } else {
        os << "<text x=\"4\" y=\"" << h / 2 << "\" font-size=\"11\">no samples yet</text>";
    }
    os << "</svg>";
    return os.str();
}

void html(Controller* cntl, const std::string& title, const std::string& body) {
    cntl->http_response().set_content_type("text/html; charset=utf-8");
    cntl->response_attachment().append("<!DOCTYPE html><html><head><meta charset=\"utf-8\"><title>" + html_escape(title) +
                                       "</title><style>body{font-family:monospace} td{padding:2px 8px;"
                                       "vertical-align:top} tr:nth-child(even){background:#f4f4f4}</style></head>"
                                       "<body>" + body + "</body></html>\n");
}

// ------------------------------------------------------------------ pages
class IndexImpl : public index {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        const Server* s = cntl->server();
        std::ostringstream os;
        os << "<html><head><title>mrpc server</title></head><body><pre>\n";
        os << "mrpc server on " << s->listen_address() << " (version: " << s->version() << ")\n\n";
        static const char* pages[][2] = {
            {"status", "per-method statistics"}, {"vars", "exposed metrics"},       {"flags", "runtime flags"},
            {"connections", "live connections"}, {"rpcz", "recent RPC spans"},     {"health", "health check"},
            {"version", "server version"},       {"list", "services and methods"}, {"threads", "thread states"},
            {"vlog", "verbose log level"},       {"fibers", "fiber runtime"},      {"ids", "call ids"},
            {"sockets", "socket details"},       {"protobufs", "message types"},   {"hotspots/cpu", "cpu profile"},
            {"hotspots/contention", "lock contention"}, {"pprof/profile", "pprof cpu profile"},
            {"brpc_metrics", "prometheus metrics"}, {"memory", "memory usage"},   {"gpu", "MI355X devices"},
            {"rdma", "RDMA provider and block pool"}, {"dir", "file browser (opt-in)"}};
        for (auto& p : pages) os << "<a href=\"/" << p[0] << "\">/" << p[0] << "</a>  " << p[1] << "\n";
        os << "\nservices:\n";
        std::vector<const Server::MethodProperty*> mps;
        s->ListMethodProperties(&mps);
        for (auto* mp : mps) {
            if (mp->is_builtin_service) continue;
            os << "  " << mp->method->full_name << "\n";
        }
        os << "</pre></body></html>\n";
        cntl->http_response().set_content_type("text/html; charset=utf-8");
        cntl->response_attachment().append(os.str());
    }
};

class StatusImpl : public status {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        const Server* s = cntl->server();
        std::ostringstream os;
        os << "version: " << s->version() << "\n";
        os << "listen: " << s->listen_address() << "\n";
        os << "start_time: " << fmt_time(s->start_time_us()) << "\n";
        os << "uptime_s: " << (realtime_us() - s->start_time_us()) / 1000000 << "\n";
        os << "concurrency: " << s->concurrency() << " (max " << s->max_concurrency() << ")\n\n";
        std::vector<const Server::MethodProperty*> mps;
        s->ListMethodProperties(&mps);
        if (query(cntl, "html")) {
            // the same, as a page: server facts, then one row per method
            std::ostringstream h;
            h << "<h3>" << html_escape(s->listen_address().to_string()) << "</h3><pre>" << html_escape(os.str()) << "</pre>"
              << "<table><tr><th>method</th><th>status</th></tr>";
            for (auto* mp : mps) {
                if (mp->is_builtin_service) continue;
                h << "<tr><td>" << html_escape(mp->method->full_name) << "</td><td><pre>"
                  << html_escape(mp->status ? mp->status->Describe() : std::string()) << "</pre></td></tr>";
            }
            h << "</table><p><a href=\"/vars?html\">/vars</a> <a href=\"/\">index</a></p>";
            html(cntl, "status", h.str());
            return;
        }
        for (auto* mp : mps) {
            if (mp->is_builtin_service) continue;
            os << mp->method->full_name << "\n";
            if (mp->status) os << mp->status->Describe() << "\n";
        }
        text(cntl, os.str());
    }
};

class VarsImpl : public vars {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        const std::string& name = unresolved(cntl);
        std::ostringstream os;
        if (!name.empty() && name.find_first_of("*?;") == std::string::npos && query(cntl, "chart")) {
            // one variable's series as a chart page
            if (var::Variable::describe_exposed(name, os) != 0) {
                cntl->SetFailed(ENOMETHOD, "no variable named `%s'", name.c_str());
                return;
            }
            const std::vector<double> v = series_values(var::Variable::series_exposed(name));
            html(cntl, name,
                 "<h3>" + html_escape(name) + " = " + html_escape(os.str()) + "</h3>" + svg_chart(v, 720, 240, true) +
                     "<p>" + std::to_string(v.size()) + " samples, oldest on the left. <a href=\"/vars/" +
                     html_escape(name) + "?series\">raw series</a> <a href=\"/vars?html\">all vars</a></p>");
            return;
        }
        if (query(cntl, "html")) {
            // every variable; those with a series get a sparkline linking to
            // their chart page
            std::vector<std::pair<std::string, std::string>> out;
            var::Variable::dump_exposed(&out, name);
            std::ostringstream h;
            h << "<table><tr><th>name</th><th>value</th><th>trend</th></tr>";
            for (auto& kv : out) {
                const std::vector<double> v = series_values(var::Variable::series_exposed(kv.first));
                h << "<tr><td>" << html_escape(kv.first) << "</td><td>" << html_escape(kv.second) << "</td><td>";
                if (!v.empty()) {
                    h << "<a href=\"/vars/" << html_escape(kv.first) << "?chart\">" << svg_chart(v, 160, 28, false)
                      << "</a>";
                }
                h << "</td></tr>";
            }
            h << "</table>";
            html(cntl, "vars", h.str());
            return;
        }
        if (!name.empty() && name.find_first_of("*?;") == std::string::npos) {
            if (query(cntl, "series")) {
                os << var::Variable::series_exposed(name);
            } else if (var::Variable::describe_exposed(name, os) != 0) {
                cntl->SetFailed(ENOMETHOD, "no variable named `%s'", name.c_str());
                return;
            }
            os << "\n";
        } else {
            std::vector<std::pair<std::string, std::string>> out;
            var::Variable::dump_exposed(&out, name);
            for (auto& kv : out) os << kv.first << " : " << kv.second << "\n";
        }
        text(cntl, os.str());
    }
};

class FlagsImpl : public flags {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        const std::string& name = unresolved(cntl);
        if (const std::string* v = query(cntl, "setvalue")) {
            if (name.empty()) {
                cntl->SetFailed(EREQUEST, "/flags/<name>?setvalue=<value>");
                return;
            }
            std::string err;
            if (!SetFlag(name, *v, /*require_reloadable=*/true, &err)) {
                cntl->SetFailed(EPERM, "fail to set %s=%s: %s", name.c_str(), v->c_str(), err.c_str());
                return;
            }
            text(cntl, "Set `" + name + "' to " + *v + "\n");
            return;
        }
        std::ostringstream os;
        for (const FlagInfo& f : ListFlags()) {
            if (!name.empty() && !wildcard_match(name, f.name)) continue;
            os << f.name << " = " << f.current_value;
            if (f.current_value != f.default_value) os << " (default: " << f.default_value << ")";
            if (f.reloadable) os << " [R]";
            os << "  # " << f.description << "\n";
        }
        text(cntl, os.str());
    }
    static bool wildcard_match(const std::string& pat, const std::string& s) {
        for (const std::string& p : split_string(pat, ';')) {
            if (p == s || fnmatch_simple(p.c_str(), s.c_str())) return true;
        }
        return false;
    }
    static bool fnmatch_simple(const char* p, const char* s) {
        if (!*p) return !*s;
        if (*p == '*') return fnmatch_simple(p + 1, s) || (*s && fnmatch_simple(p, s + 1));
        if (*s && (*p == '?' || *p == *s)) return fnmatch_simple(p + 1, s + 1);
        return false;
    }
};

class ConnectionsImpl : public connections {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        text(C(c), DescribeAllSockets());
    }
};

class RpczImpl : public rpcz {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        if (query(cntl, "enable")) {
            SetFlag("enable_rpcz", "true");
            text(cntl, "rpcz enabled\n");
            return;
        }
        if (query(cntl, "disable")) {
            SetFlag("enable_rpcz", "false");
            text(cntl, "rpcz disabled\n");
            return;
        }
        uint64_t trace = 0;
        if (const std::string* t = query(cntl, "trace_id")) trace = strtoull(t->c_str(), nullptr, 16);
        if (const std::string* t = query(cntl, "trace")) trace = strtoull(t->c_str(), nullptr, 16);
        size_t max = 100;
        if (const std::string* m = query(cntl, "max")) max = (size_t)atoi(m->c_str());
        const std::string* tq = query(cntl, "time");
        // time=<epoch us> or time=YYYY/MM/DD-HH:MM:SS (local time): spans
        // that ended at or before it, from the on-disk store
        int64_t before_us = 0;
        if (tq) {
            struct tm tmv = {};
            if (strptime(tq->c_str(), "%Y/%m/%d-%H:%M:%S", &tmv)) {
                tmv.tm_isdst = -1;
                before_us = (int64_t)mktime(&tmv) * 1000000 + 999999;
            } else {
                before_us = strtoll(tq->c_str(), nullptr, 10);
            }
        }
        const span_db::Stats st = span_db::GetStats();
        if (!IsRpczEnabled() && st.indexed == 0) {
            text(cntl, "rpcz is disabled; visit /rpcz?enable to turn it on\n");
            return;
        }
        std::ostringstream os;
        if (query(cntl, "stats")) {
            os << "dir: " << st.dir << "\nwritten: " << st.written << "\ndropped: " << st.dropped
               << "\nindexed: " << st.indexed << "\nfiles: " << st.files << "\nbytes: " << st.bytes
               << "\nreloaded: " << st.reloaded << "\n";
        } else if (trace) {
            // whole trace from disk (includes spans evicted from memory and,
            // with -rpcz_keep_span_db, spans of the previous run)
            std::vector<std::string> v = span_db::FindTrace(trace, max);
            if (v.empty()) v = ListRecentSpans(max, trace);
            for (const std::string& x : v) os << x << "\n";
        } else if (tq) {
            for (const std::string& x : span_db::ListBefore(before_us, max)) os << x << "\n";
        } else {
            for (const std::string& x : ListRecentSpans(max, 0)) os << x << "\n";
        }
        text(cntl, os.str());
    }
};

class HealthImpl : public health {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        Controller* cntl = C(c);
        HealthReporter* r = cntl->server()->options().health_reporter;
        if (r) {
            r->GenerateReport(cntl, done);
            return;
        }
        ClosureGuard g(done);
        text(cntl, "OK\n");
    }
};

class VersionImpl : public version {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        text(cntl, (cntl->server()->version().empty() ? std::string("unknown") : cntl->server()->version()) + "\n");
    }
};

class ListImpl : public list {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        std::vector<Service*> svcs;
        cntl->server()->ListServices(&svcs);
        std::ostringstream os;
        for (Service* s : svcs) {
            const pb::ServiceDescriptor* sd = s->GetDescriptor();
            os << "service " << sd->full_name << " {\n";
            for (int i = 0; i < sd->method_count(); ++i) {
                const pb::MethodDescriptor* m = sd->method(i);
                os << "  rpc " << m->name << "(" << (m->input_type ? m->input_type->full_name : m->input_type_name)
                   << ") returns (" << (m->output_type ? m->output_type->full_name : m->output_type_name) << ");\n";
            }
            os << "}\n";
        }
        text(cntl, os.str());
    }
};

class ThreadsImpl : public threads {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        if (!FLAGS_enable_threads_service) {
            cntl->SetFailed(EPERM, "/threads is disabled, set -enable_threads_service");
            return;
        }
        std::ostringstream os;
        DIR* d = opendir("/proc/self/task");
        if (d) {
            while (dirent* e = readdir(d)) {
                if (e->d_name[0] == '.') continue;
                std::ifstream comm(std::string("/proc/self/task/") + e->d_name + "/comm");
                std::ifstream stat(std::string("/proc/self/task/") + e->d_name + "/stat");
                std::string name, st;
                std::getline(comm, name);
                std::getline(stat, st);
                const size_t rp = st.rfind(')');
                const char state = rp != std::string::npos && rp + 2 < st.size() ? st[rp + 2] : '?';
                os << e->d_name << "\t" << state << "\t" << name << "\n";
            }
            closedir(d);
        }
        text(cntl, os.str());
    }
};

class VlogImpl : public vlog {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        if (const std::string* v = query(cntl, "setlevel")) SetVerboseLevel(atoi(v->c_str()));
        text(cntl, "verbose level: " + std::to_string(GetVerboseLevel()) + " (set with /vlog?setlevel=N)\n");
    }
};

class FibersImpl : public fibers {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        std::ostringstream os;
        os << "workers: " << fiber::get_concurrency() << "\n";
        os << "live fibers: " << fiber::fiber_count() << "\n";
        os << "context switches: " << fiber::switch_count() << "\n";
        os << "steals: " << fiber::steal_count() << "\n";
        os << "worker usage: " << fiber::worker_usage() << "\n\n";
        os << fiber::DescribeFibers(200);
        text(C(c), os.str());
    }
};

class IdsImpl : public ids {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        const std::string& id = unresolved(cntl);
        if (id.empty()) {
            text(cntl, "usage: /ids/<call id in decimal>\n");
            return;
        }
        const fiber::CallId cid{strtoull(id.c_str(), nullptr, 10)};
        text(cntl, std::string("call id ") + id + (fiber::call_id_exists(cid) ? " is alive\n" : " does not exist\n"));
    }
};

class SocketsImpl : public sockets {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        const std::string& id = unresolved(cntl);
        if (id.empty()) {
            text(cntl, DescribeAllSockets());
            return;
        }
        SocketUniquePtr s;
        if (Socket::AddressFailedAsWell(strtoull(id.c_str(), nullptr, 10), &s) != 0) {
            cntl->SetFailed(ENOMETHOD, "no socket %s", id.c_str());
            return;
        }
        text(cntl, s->description() + "\n");
    }
};

static void print_message(std::ostream& os, const pb::Descriptor* d) {
    os << "message " << d->full_name << " {\n";
    for (int i = 0; i < d->field_count(); ++i) {
        const pb::FieldDescriptor* f = d->field(i);
        const char* label = f->is_repeated() ? "repeated " : (f->is_required() ? "required " : "optional ");
        std::string type = f->message_type ? f->message_type->full_name
                                           : (f->enum_type ? f->enum_type->full_name : pb::FieldTypeName(f->type));
        os << "  " << label << type << " " << f->name << " = " << f->number;
        if (f->has_default) os << " [default = " << f->default_str << "]";
        os << ";\n";
    }
    os << "}\n";
}

class ProtobufsImpl : public protobufs {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        std::vector<Service*> svcs;
        cntl->server()->ListServices(&svcs);
        std::map<std::string, const pb::Descriptor*> types;
        std::function<void(const pb::Descriptor*)> add = [&](const pb::Descriptor* d) {
            if (!d || types.count(d->full_name)) return;
            types[d->full_name] = d;
            for (int i = 0; i < d->field_count(); ++i) add(d->field(i)->message_type);
        };
        for (Service* s : svcs) {
            const pb::ServiceDescriptor* sd = s->GetDescriptor();
            for (int i = 0; i < sd->method_count(); ++i) {
                add(sd->method(i)->input_type);
                add(sd->method(i)->output_type);
            }
        }
        const std::string& name = unresolved(cntl);
        std::ostringstream os;
        if (name.empty()) {
            for (auto& kv : types) os << kv.first << "\n";
        } else {
            auto it = types.find(name);
            if (it == types.end()) {
                cntl->SetFailed(ENOMETHOD, "no message type %s", name.c_str());
                return;
            }
            print_message(os, it->second);
        }
        text(cntl, os.str());
    }
};

static double seconds_param(Controller* cntl, double def) {
    const std::string* s = query(cntl, "seconds");
    double v = s ? atof(s->c_str()) : def;
    if (v <= 0) v = def;
    return std::min(v, 60.0);
}

// Heap profiles come from heapprof/heapprof.cc when it is linked into the
// executable (or LD_PRELOADed): found at run time, like the reference finds
// tcmalloc's MallocExtension (details/tcmalloc_extension.cpp).
std::string HeapProfileRaw(bool growth, bool* linked) {
    typedef char* (*Fn)(int);
    static Fn fn = reinterpret_cast<Fn>(dlsym(RTLD_DEFAULT, "mrpc_heap_profile_text"));
    *linked = fn != nullptr;
    if (!fn) return std::string();
    char* p = fn(growth ? 1 : 0);
    std::string out = p ? p : "";
    free(p);
    return out;
}

// Human view of a raw profile: stacks sorted by bytes, symbolized.
std::string HeapProfileReport(const std::string& raw, bool growth) {
    struct Row {
        long long bytes, count;
        std::string stack;
    };
    std::vector<Row> rows;
    std::istringstream is(raw);
    std::string line, header;
    std::getline(is, header);
    while (std::getline(is, line)) {
        if (line.empty() || line[0] == 'M') break;
        const size_t at = line.find('@');
        if (at == std::string::npos) continue;
        Row r;
        r.count = atoll(line.c_str());
        r.bytes = atoll(line.c_str() + line.find(':') + 1);
        std::istringstream fs(line.substr(at + 1));
        std::string a;
        bool first = true;
        while (fs >> a) {
            const std::string sym = profiler::Symbolize((uintptr_t)strtoull(a.c_str(), nullptr, 16));
            if (sym.find("mrpc_heap") != std::string::npos) continue;
            r.stack += (first ? "" : " <- ") + sym;
            first = false;
        }
        rows.push_back(r);
    }
    std::sort(rows.begin(), rows.end(), [](const Row& x, const Row& y) { return x.bytes > y.bytes; });
    std::ostringstream os;
    os << (growth ? "# cumulative sampled allocations (growth)\n" : "# in-use sampled allocations\n") << header
       << "\n# bytes count stack\n";
    for (const Row& r : rows) os << r.bytes << " " << r.count << " " << r.stack << "\n";
    return os.str();
}

class HotspotsImpl : public hotspots {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        const std::string& kind = unresolved(cntl);
        if (kind == "cpu" || kind.empty()) {
            std::string folded;
            int64_t n = 0;
            const int hz = query(cntl, "frequency") ? atoi(query(cntl, "frequency")->c_str()) : 100;
            if (!profiler::ProfileCpu(seconds_param(cntl, 10), hz, &folded, nullptr, &n)) {
                cntl->SetFailed(EAGAIN, "another cpu profile is running");
                return;
            }
            text(cntl, "# " + std::to_string(n) + " samples, folded stacks (flamegraph.pl input)\n" + folded);
        } else if (kind == "contention") {
            const double secs = seconds_param(cntl, 10);
            if (!fiber::ContentionProfilerStart(nullptr)) {
                cntl->SetFailed(EAGAIN, "another contention profile is running");
                return;
            }
            fiber::usleep((int64_t)(secs * 1e6));
            fiber::ContentionProfilerStop();
            std::string dump = fiber::ContentionProfilerDump();
            std::istringstream is(dump);
            std::ostringstream os;
            os << "# caller count total_wait_ns\n";
            std::string line;
            while (std::getline(is, line)) {
                unsigned long long addr = strtoull(line.c_str(), nullptr, 16);
                os << profiler::Symbolize((uintptr_t)addr) << " " << line.substr(line.find(' ') + 1) << "\n";
            }
            text(cntl, os.str());
        } else if (kind == "heap" || kind == "growth") {
            bool linked = false;
            const std::string raw = HeapProfileRaw(kind == "growth", &linked);
            if (linked) {
                text(cntl, HeapProfileReport(raw, kind == "growth"));
                return;
            }
            struct mallinfo2 mi = mallinfo2();
            std::ostringstream os;
            os << "heap profiling needs the sampling allocator (link heapprof/heapprof.cc or LD_PRELOAD "
                  "libmrpc_heapprof.so); glibc arena summary:\n";
            os << "arena " << mi.arena << "\nin_use " << mi.uordblks << "\nfree " << mi.fordblks << "\nmmap "
               << mi.hblkhd << "\n";
            text(cntl, os.str());
        } else {
            cntl->SetFailed(ENOMETHOD, "unknown hotspot kind `%s' (cpu|contention|heap|growth)", kind.c_str());
        }
    }
};

class PprofImpl : public pprof {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        const std::string& kind = unresolved(cntl);
        if (kind == "profile") {
            std::string bin;
            if (!profiler::ProfileCpu(seconds_param(cntl, 10), 100, nullptr, &bin, nullptr)) {
                cntl->SetFailed(EAGAIN, "another cpu profile is running");
                return;
            }
            cntl->http_response().set_content_type("application/octet-stream");
            cntl->response_attachment().append(bin);
        } else if (kind == "symbol") {
            // GET: report that symbols are available; POST: "0xaddr+0xaddr..."
            if (cntl->http_request().method() == HTTP_METHOD_GET) {
                text(cntl, "num_symbols: 1\n");
                return;
            }
            std::string body = cntl->request_attachment().to_string();
            std::ostringstream os;
            for (const std::string& a : split_string_any(body, "+ \n")) {
                const uintptr_t addr = (uintptr_t)strtoull(a.c_str(), nullptr, 16);
                if (addr) os << a << "\t" << profiler::Symbolize(addr) << "\n";
            }
            text(cntl, os.str());
        } else if (kind == "cmdline") {
            std::ifstream f("/proc/self/cmdline");
            std::string s((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
            std::replace(s.begin(), s.end(), '\0', '\n');
            text(cntl, s);
        } else if (kind == "heap" || kind == "growth") {
            bool linked = false;
            const std::string raw = HeapProfileRaw(kind == "growth", &linked);
            if (!linked) {
                cntl->SetFailed(ENOMETHOD, "heap profiles need heapprof/heapprof.cc linked or preloaded");
                return;
            }
            cntl->http_response().set_content_type("text/plain");
            cntl->response_attachment().append(raw);  // pprof reads the legacy text format
        } else {
            cntl->SetFailed(ENOMETHOD, "unknown pprof endpoint `%s' (profile|symbol|cmdline)", kind.c_str());
        }
    }
};

class DirImpl : public dir {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        if (!FLAGS_enable_dir_service) {
            cntl->SetFailed(EPERM, "/dir is disabled, set -enable_dir_service");
            return;
        }
        const std::string path = "/" + unresolved(cntl);
        struct stat st;
        if (stat(path.c_str(), &st) != 0) {
            cntl->SetFailed(ENOMETHOD, "no such path %s", path.c_str());
            return;
        }
        if (S_ISDIR(st.st_mode)) {
            std::ostringstream os;
            DIR* d = opendir(path.c_str());
            std::vector<std::string> names;
            while (d && (true)) {
                dirent* e = readdir(d);
                if (!e) break;
                names.push_back(e->d_name);
            }
            if (d) closedir(d);
            std::sort(names.begin(), names.end());
            for (auto& n : names) os << n << "\n";
            text(cntl, os.str());
        } else {
            std::ifstream f(path, std::ios::binary);
            std::string s((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
            text(cntl, s);
        }
    }
};

class MetricsImpl : public brpc_metrics {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = C(c);
        cntl->http_response().set_content_type("text/plain; version=0.0.4");
        cntl->response_attachment().append(var::Variable::dump_prometheus());
    }
};

class MemoryImpl : public memory {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        struct mallinfo2 mi = mallinfo2();
        std::ostringstream os;
        os << "buf_blocks " << Buf::block_count() << "\nbuf_block_memory " << Buf::block_memory()
           << "\nmalloc_arena " << mi.arena << "\nmalloc_in_use " << mi.uordblks << "\nmalloc_free " << mi.fordblks
           << "\nmalloc_mmap " << mi.hblkhd << "\n";
        text(C(c), os.str());
    }
};

class GpuImpl : public gpu {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        std::ostringstream os;
        const int n = mrpc::gpu::DeviceCount();
        os << "devices: " << n << "\n";
        for (int i = 0; i < n; ++i) {
            os << "  [" << i << "] " << mrpc::gpu::DeviceName(i) << " (" << mrpc::gpu::DeviceArch(i) << ")\n";
        }
        os << "completion events polled: " << mrpc::gpu::PolledEvents() << "\n";
        text(C(c), os.str());
    }
};

class RdmaImpl : public rdma {
public:
    void default_method(RpcController* c, const BuiltinRequest*, BuiltinResponse*, Closure* done) override {
        ClosureGuard g(done);
        text(C(c), mrpc::rdma::DescribeRdma());
    }
};

int AddBuiltinServices(Server* server) {
    Service* svcs[] = {new IndexImpl,   new StatusImpl,   new VarsImpl,     new FlagsImpl,   new ConnectionsImpl,
                       new RpczImpl,    new HealthImpl,   new VersionImpl,  new ListImpl,    new ThreadsImpl,
                       new VlogImpl,    new FibersImpl,   new IdsImpl,      new SocketsImpl, new ProtobufsImpl,
                       new HotspotsImpl, new PprofImpl,   new DirImpl,      new MetricsImpl, new MemoryImpl,
                       new GpuImpl,     new RdmaImpl};
    for (Service* s : svcs) {
        if (server->AddBuiltinService(s) != 0) {
            LOG(ERROR) << "Fail to add builtin service " << s->GetDescriptor()->full_name;
            return -1;
        }
    }
    return 0;
}

struct Installer {
    Installer() { SetAddBuiltinServicesHook(AddBuiltinServices); }
} g_installer;

}  // namespace
}  // namespace builtin
}  // namespace mrpc
