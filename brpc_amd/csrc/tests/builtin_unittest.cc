// Builtin pages (builtin/builtin_services.cc), in the spirit of the
// reference's test/brpc_builtin_service_unittest.cpp: every page answers over
// plain HTTP on the server's own port, with the content the page promises,
// its switches (/flags setvalue, /vlog setlevel, /rpcz enable) and its
// refusals (non-reloadable flags, disabled pages, unknown names).
#include <cstdlib>
#include <string>

#include "base/flags.h"
#include "http/http_header.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/health_reporter.h"
#include "rpc/server.h"
#include "rpc/span.h"
#include "services/echo_service.h"
#include "tests/test.h"
#include "var/var.h"
#include <unistd.h>

using namespace mrpc;

namespace {

struct Reporter : public HealthReporter {
    void GenerateReport(Controller* cntl, Closure* done) override {
        cntl->http_response().set_status_code(503);
        cntl->response_attachment().append("draining\n");
        done->Run();
    }
};

struct Site {
    Server server;
    EchoServiceImpl echo;
    Reporter reporter;
    Channel ch;
    int port = 0;
    explicit Site(bool with_reporter = false) {
        server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        server.set_version("builtin-test-7");
        ServerOptions o;
        if (with_reporter) o.health_reporter = &reporter;
        if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
        ChannelOptions co;
        co.protocol = "http";
        co.timeout_ms = 5000;
        ch.Init(("http://127.0.0.1:" + std::to_string(port)).c_str(), &co);
    }
    // GET path (with an optional query); returns the body, *code the
    // controller error (0 ok) and *status the http status
    std::string get(const std::string& url, int* code = nullptr, int* status = nullptr) {
        Controller cntl;
        cntl.http_request().uri().SetHttpURL(url);
        ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        if (code) *code = cntl.ErrorCode();
        if (status) *status = cntl.http_response().status_code();
        return cntl.response_attachment().to_string();
    }
};

bool has(const std::string& hay, const std::string& needle) { return hay.find(needle) != std::string::npos; }

}  // namespace

TEST(BuiltinPages, index_links_every_page) {
    Site s;
    ASSERT_GT(s.port, 0);
    int code = -1;
    const std::string body = s.get("/", &code);
    EXPECT_EQ(code, 0);
    for (const char* p : {"/status", "/vars", "/flags", "/connections", "/rpcz", "/health", "/version", "/list",
                          "/fibers", "/sockets", "/protobufs", "/brpc_metrics", "/gpu"}) {
        EXPECT_TRUE_M(has(body, std::string("href=\"") + p + "\""), std::string(p));
    }
    EXPECT_TRUE(has(body, "builtin-test-7"));
}

TEST(BuiltinPages, version_and_default_health) {
    Site s;
    int code = -1, status = 0;
    EXPECT_EQ(s.get("/version", &code), "builtin-test-7\n");
    EXPECT_EQ(code, 0);
    EXPECT_EQ(s.get("/health", &code, &status), "OK\n");
    EXPECT_EQ(status, 200);
}

TEST(BuiltinPages, customized_health_reporter) {
    Site s(/*with_reporter=*/true);
    int code = -1, status = 0;
    const std::string body = s.get("/health", &code, &status);
    EXPECT_EQ(status, 503);
    EXPECT_TRUE_M(has(body, "draining"), body);
}

TEST(BuiltinPages, status_lists_user_methods_with_their_counters) {
    Site s;
    // one echo over http+json first, so the method has a counted call
    {
        Controller cntl;
        cntl.http_request().uri().SetHttpURL("/example.EchoService/Echo");
        cntl.http_request().set_method(HTTP_METHOD_POST);
        cntl.http_request().set_content_type("application/json");
        cntl.request_attachment().append("{\"message\":\"hi\"}");
        s.ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        EXPECT_FALSE(cntl.Failed());
    }
    const std::string body = s.get("/status");
    EXPECT_TRUE_M(has(body, "example.EchoService.Echo"), body);
    EXPECT_TRUE_M(has(body, "version: builtin-test-7"), body);
    EXPECT_FALSE_M(has(body, "mrpc.BuiltinService") && has(body, "status.default_method"), body);
}

TEST(BuiltinPages, list_and_protobufs_describe_the_services) {
    Site s;
    const std::string list = s.get("/list");
    EXPECT_TRUE_M(has(list, "service example.EchoService {"), list);
    EXPECT_TRUE_M(has(list, "rpc Echo(example.EchoRequest) returns (example.EchoResponse);"), list);
    const std::string types = s.get("/protobufs");
    EXPECT_TRUE_M(has(types, "example.EchoRequest"), types);
    int code = -1;
    const std::string one = s.get("/protobufs/example.EchoRequest", &code);
    EXPECT_EQ(code, 0);
    EXPECT_TRUE_M(has(one, "message example.EchoRequest {"), one);
    EXPECT_TRUE_M(has(one, "message = 1;"), one);
    s.get("/protobufs/no.Such", &code);
    EXPECT_EQ(code, ENOMETHOD);
}

TEST(BuiltinPages, flags_list_filter_and_set) {
    Site s;
    const std::string all = s.get("/flags");
    EXPECT_TRUE(has(all, "max_body_size = "));
    // wildcard filter: only matching names
    const std::string some = s.get("/flags/health_check_*");
    EXPECT_TRUE_M(has(some, "health_check_interval"), some);
    EXPECT_FALSE(has(some, "max_body_size"));
    // reloadable flag set through the page, shown with its default
    int code = -1;
    s.get("/flags/max_body_size?setvalue=7654321", &code);
    EXPECT_EQ(code, 0);
    const std::string one = s.get("/flags/max_body_size");
    EXPECT_TRUE_M(has(one, "max_body_size = 7654321 (default: "), one);
    EXPECT_TRUE_M(has(one, "[R]"), one);
    SetFlag("max_body_size", "67108864");
    // a bad value and a setvalue without a name are refused
    s.get("/flags/max_body_size?setvalue=notanumber", &code);
    EXPECT_EQ(code, EPERM);
    s.get("/flags?setvalue=1", &code);
    EXPECT_EQ(code, EREQUEST);
}

TEST(BuiltinPages, flags_refuse_non_reloadable_ones) {
    Site s;
    std::string before;
    ASSERT_TRUE(GetFlag("enable_dir_service", &before));
    int code = -1;
    // a flag not declared reloadable refuses writes through the page
    s.get("/flags/enable_dir_service?setvalue=true", &code);
    EXPECT_EQ(code, EPERM);
    std::string after;
    GetFlag("enable_dir_service", &after);
    EXPECT_EQ(after, before);
}

TEST(BuiltinPages, vars_all_one_wildcard_and_unknown) {
    Site s;
    const std::string all = s.get("/vars");
    EXPECT_TRUE(has(all, "fiber_count : "));
    int code = -1;
    const std::string one = s.get("/vars/fiber_count", &code);
    EXPECT_EQ(code, 0);
    EXPECT_GT(atoi(one.c_str()), 0);
    const std::string wild = s.get("/vars/fiber_*");
    EXPECT_TRUE(has(wild, "fiber_count : "));
    EXPECT_FALSE(has(wild, "process_"));
    s.get("/vars/definitely_not_a_var", &code);
    EXPECT_EQ(code, ENOMETHOD);
}

TEST(BuiltinPages, vlog_reads_and_sets_the_level) {
    Site s;
    EXPECT_TRUE(has(s.get("/vlog?setlevel=3"), "verbose level: 3"));
    EXPECT_TRUE(has(s.get("/vlog"), "verbose level: 3"));
    s.get("/vlog?setlevel=0");
}

TEST(BuiltinPages, connections_and_sockets_show_the_caller) {
    Site s;
    const std::string conns = s.get("/connections");
    EXPECT_TRUE_M(has(conns, "127.0.0.1"), conns);
    const std::string socks = s.get("/sockets");
    EXPECT_FALSE(socks.empty());
    int code = -1;
    s.get("/sockets/999999999999", &code);
    EXPECT_EQ(code, ENOMETHOD);
}

TEST(BuiltinPages, fibers_and_ids) {
    Site s;
    const std::string f = s.get("/fibers");
    EXPECT_TRUE_M(has(f, "workers: "), f);
    EXPECT_TRUE(has(f, "live fibers: "));
    EXPECT_TRUE(has(s.get("/ids"), "usage: /ids/"));
    EXPECT_TRUE(has(s.get("/ids/12345"), "does not exist"));
}

TEST(BuiltinPages, threads_page_is_opt_in) {
    Site s;
    int code = -1;
    s.get("/threads", &code);
    EXPECT_EQ(code, EPERM);
    SetFlag("enable_threads_service", "true");
    const std::string t = s.get("/threads", &code);
    EXPECT_EQ(code, 0);
    EXPECT_FALSE(t.empty());
    SetFlag("enable_threads_service", "false");
}

TEST(BuiltinPages, dir_page_is_opt_in) {
    Site s;
    int code = -1;
    s.get("/dir/tmp", &code);
    EXPECT_EQ(code, EPERM);
    SetFlag("enable_dir_service", "true");
    s.get("/dir/proc/self/status", &code);
    EXPECT_EQ(code, 0);
    s.get("/dir/no/such/path/at/all", &code);
    EXPECT_EQ(code, ENOMETHOD);
    SetFlag("enable_dir_service", "false");
}

TEST(BuiltinPages, rpcz_enable_and_disable) {
    Site s;
    const bool was = IsRpczEnabled();
    EXPECT_TRUE(has(s.get("/rpcz?enable"), "rpcz enabled"));
    EXPECT_TRUE(IsRpczEnabled());
    int code = -1;
    s.get("/rpcz?stats", &code);
    EXPECT_EQ(code, 0);
    EXPECT_TRUE(has(s.get("/rpcz?disable"), "rpcz disabled"));
    EXPECT_FALSE(IsRpczEnabled());
    if (was) SetFlag("enable_rpcz", "true");
}

TEST(BuiltinPages, prometheus_metrics_format) {
    Site s;
    const std::string m = s.get("/brpc_metrics");
    EXPECT_TRUE_M(has(m, "# TYPE "), m.substr(0, 200));
    // every sample line is "<name> <number>" with a metric-safe name
    size_t lines = 0, bad = 0;
    size_t pos = 0;
    while (pos < m.size()) {
        size_t e = m.find('\n', pos);
        if (e == std::string::npos) e = m.size();
        const std::string line = m.substr(pos, e - pos);
        pos = e + 1;
        if (line.empty() || line[0] == '#') continue;
        ++lines;
        const size_t sp = line.rfind(' ');
        if (sp == std::string::npos) {
            ++bad;
            continue;
        }
        for (size_t i = 0; i < line.find_first_of(" {"); ++i) {
            const char c = line[i];
            if (!(isalnum((unsigned char)c) || c == '_' || c == ':')) {
                ++bad;
                break;
            }
        }
    }
    EXPECT_GT(lines, 10u);
    EXPECT_EQ(bad, 0u);
}

TEST(BuiltinPages, unknown_pages_and_kinds_are_404) {
    Site s;
    int code = -1, status = 0;
    s.get("/no_such_page", &code, &status);
    EXPECT_EQ(code, ENOMETHOD);
    EXPECT_EQ(status, 404);
    s.get("/hotspots/nonsense", &code);
    EXPECT_EQ(code, ENOMETHOD);
    s.get("/pprof/nonsense", &code);
    EXPECT_EQ(code, ENOMETHOD);
}

TEST(BuiltinPages, pprof_cmdline_and_symbol) {
    Site s;
    int code = -1;
    const std::string cmd = s.get("/pprof/cmdline", &code);
    EXPECT_EQ(code, 0);
    EXPECT_FALSE(cmd.empty());
    EXPECT_TRUE(has(s.get("/pprof/symbol"), "num_symbols"));
}

TEST(BuiltinPages, memory_and_gpu_pages_answer) {
    Site s;
    int code = -1;
    EXPECT_FALSE(s.get("/memory", &code).empty());
    EXPECT_EQ(code, 0);
    s.get("/gpu", &code);  // no device here: the page still answers
    EXPECT_EQ(code, 0);
}

// Chart views (role of the reference's flot pages, builtin/vars_service.cpp
// :40-75): a windowed variable's series as an inline SVG line, sparklines
// on the HTML variable list, and an HTML /status.
TEST(BuiltinPages, vars_series_chart_and_html_views) {
    Site s;
    var::Adder<int64_t> a;
    var::PerSecond<var::Adder<int64_t>> ps("builtin_chart_per_second", &a, 10);
    for (int i = 0; i < 3; ++i) {
        a << (i + 1) * 100;
        usleep(1100 * 1000);  // the sampler takes one point a second
    }
    int code = -1, status = 0;
    const std::string page = s.get("/vars/builtin_chart_per_second?chart", &code, &status);
    EXPECT_EQ(code, 0);
    EXPECT_TRUE(has(page, "<svg"));
    EXPECT_TRUE(has(page, "<polyline"));
    EXPECT_TRUE(has(page, "builtin_chart_per_second"));
    const std::string list = s.get("/vars/builtin_chart_*?html");
    EXPECT_TRUE(has(list, "<table>"));
    EXPECT_TRUE(has(list, "href=\"/vars/builtin_chart_per_second?chart\""));
    s.get("/vars/not_a_var_at_all?chart", &code);
    EXPECT_EQ(code, ENOMETHOD);
    const std::string st = s.get("/status?html", &code);
    EXPECT_EQ(code, 0);
    EXPECT_TRUE(has(st, "<table>"));
    EXPECT_TRUE(has(st, "example.EchoService.Echo"));
    // the plain views are unchanged
    EXPECT_FALSE(has(s.get("/status"), "<table>"));
}
