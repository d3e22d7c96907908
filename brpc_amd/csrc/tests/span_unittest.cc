// rpcz span store suite (spirit of the reference's span database,
// src/brpc/span.cpp:306-560 and builtin/rpcz_service.cpp: spans found by
// trace id and by time, kept across restarts with -rpcz_keep_span_db).
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>

#include "base/flags.h"
#include "base/time.h"
#include "base/util.h"
#include "mrpc/proto/echo.pb.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/server.h"
#include "rpc/span.h"
#include "rpc/span_db.h"
#include "services/echo_service.h"
#include "tests/test.h"

DECLARE_bool(enable_rpcz);
DECLARE_string(rpcz_database_dir);
DECLARE_bool(rpcz_keep_span_db);

extern char** environ;

using namespace mrpc;

namespace {

std::string make_tmpdir() {
    char tmpl[] = "/tmp/mrpc_rpcz_XXXXXX";
    const char* d = mkdtemp(tmpl);
    return d ? d : "";
}

struct EchoServer {
    Server server;
    EchoServiceImpl echo;
    int port = 0;
    EchoServer() {
        server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        ServerOptions o;
        o.has_builtin_services = false;
        if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
    }
};

// One echo; returns the trace id of the call.
uint64_t echo_once(Channel* ch, const std::string& msg) {
    example::EchoService_Stub stub(ch);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message(msg);
    stub.Echo(&cntl, &req, &res, nullptr);
    return cntl.Failed() ? 0 : cntl.trace_id();
}

// Spans are submitted by the server after its write returns: poll.
std::vector<std::string> wait_trace(uint64_t trace, size_t want) {
    std::vector<std::string> v;
    for (int i = 0; i < 200; ++i) {
        span_db::Flush();
        v = span_db::FindTrace(trace, 10);
        if (v.size() >= want) break;
        usleep(10000);
    }
    return v;
}

}  // namespace

TEST(Rpcz, spans_on_disk_by_trace_and_time) {
    const std::string dir = make_tmpdir();
    ASSERT_FALSE(dir.empty());
    FLAGS_rpcz_database_dir = dir;
    FLAGS_enable_rpcz = true;
    EchoServer s;
    ASSERT_GT(s.port, 0);
    Channel ch;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(s.port)).c_str(), nullptr), 0);

    const uint64_t t1 = echo_once(&ch, "first");
    ASSERT_TRUE(t1 != 0);
    // both sides of the call, server (S) and client (C), under one trace
    std::vector<std::string> v = wait_trace(t1, 2);
    ASSERT_EQ(v.size(), 2u);
    int servers = 0, clients = 0;
    for (const std::string& x : v) {
        EXPECT_TRUE(x.find("example.EchoService.Echo") != std::string::npos);
        EXPECT_TRUE(x.find(string_printf("trace=%016llx", (unsigned long long)t1)) != std::string::npos);
        servers += x[0] == 'S';
        clients += x[0] == 'C';
    }
    EXPECT_EQ(servers, 1);
    EXPECT_EQ(clients, 1);

    usleep(30000);
    const int64_t mid = realtime_us();
    usleep(30000);
    const uint64_t t2 = echo_once(&ch, "second");
    ASSERT_TRUE(t2 != 0 && t2 != t1);
    ASSERT_EQ(wait_trace(t2, 2).size(), 2u);

    // time query: before `mid` only the first call's spans exist
    std::vector<std::string> before = span_db::ListBefore(mid, 100);
    EXPECT_EQ(before.size(), 2u);
    for (const std::string& x : before) {
        EXPECT_TRUE(x.find(string_printf("trace=%016llx", (unsigned long long)t1)) != std::string::npos);
    }
    // now: newest first
    std::vector<std::string> all = span_db::ListBefore(0, 100);
    ASSERT_EQ(all.size(), 4u);
    EXPECT_TRUE(all[0].find(string_printf("trace=%016llx", (unsigned long long)t2)) != std::string::npos);
    EXPECT_TRUE(span_db::FindTrace(12345, 10).empty());

    span_db::Stats st = span_db::GetStats();
    EXPECT_EQ(st.written, 4);
    EXPECT_EQ(st.indexed, 4);
    EXPECT_EQ(st.dropped, 0);
    EXPECT_GE(st.files, 1);
    EXPECT_GT(st.bytes, 0);
    FLAGS_enable_rpcz = false;
}

// The writer half of the restart test: runs only in the child spawned by
// RpczRestart.reload_previous_run (a no-op when the driver runs it alone).
TEST(RpczWriter, write_spans_then_exit) {
    const char* out = getenv("MRPC_RPCZ_CHILD_OUT");
    if (!out) return;
    FLAGS_enable_rpcz = true;
    EchoServer s;
    ASSERT_GT(s.port, 0);
    Channel ch;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(s.port)).c_str(), nullptr), 0);
    std::ofstream f(out);
    for (int i = 0; i < 3; ++i) {
        const uint64_t t = echo_once(&ch, "child " + std::to_string(i));
        ASSERT_TRUE(t != 0);
        ASSERT_EQ(wait_trace(t, 2).size(), 2u);
        f << t << "\n";
    }
}

TEST(RpczRestart, reload_previous_run) {
    const std::string dir = make_tmpdir();
    ASSERT_FALSE(dir.empty());
    const std::string ids = dir + "/../" + dir.substr(dir.rfind('/') + 1) + ".ids";
    // previous "run": another process writes spans into `dir`
    char self[4096];
    const ssize_t n = readlink("/proc/self/exe", self, sizeof(self) - 1);
    ASSERT_GT(n, 0);
    self[n] = 0;
    std::string a0 = self, a1 = "--filter=RpczWriter.write_spans_then_exit", a2 = "--rpcz_database_dir=" + dir;
    char* argv[] = {&a0[0], &a1[0], &a2[0], nullptr};
    std::string env_out = "MRPC_RPCZ_CHILD_OUT=" + ids;
    std::vector<char*> envp;
    for (char** e = environ; *e; ++e) envp.push_back(*e);
    envp.push_back(&env_out[0]);
    envp.push_back(nullptr);
    pid_t pid = 0;
    ASSERT_EQ(posix_spawn(&pid, self, nullptr, nullptr, argv, envp.data()), 0);
    int status = 0;
    ASSERT_EQ(waitpid(pid, &status, 0), pid);
    ASSERT_TRUE(WIFEXITED(status) && WEXITSTATUS(status) == 0);
    std::vector<uint64_t> traces;
    {
        std::ifstream f(ids);
        uint64_t t;
        while (f >> t) traces.push_back(t);
    }
    unlink(ids.c_str());
    ASSERT_EQ(traces.size(), 3u);

    // this process opens the same directory keeping the old files
    FLAGS_rpcz_database_dir = dir;
    FLAGS_rpcz_keep_span_db = true;
    span_db::Stats st = span_db::GetStats();
    EXPECT_EQ(st.reloaded, 6);
    EXPECT_EQ(st.indexed, 6);
    for (uint64_t t : traces) EXPECT_EQ(span_db::FindTrace(t, 10).size(), 2u);
    EXPECT_EQ(span_db::ListBefore(0, 100).size(), 6u);

    // new spans append after the reloaded ones, in a new file
    FLAGS_enable_rpcz = true;
    EchoServer s;
    Channel ch;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(s.port)).c_str(), nullptr), 0);
    const uint64_t t = echo_once(&ch, "after restart");
    ASSERT_EQ(wait_trace(t, 2).size(), 2u);
    st = span_db::GetStats();
    EXPECT_EQ(st.indexed, 8);
    EXPECT_GE(st.files, 2);
    FLAGS_enable_rpcz = false;
}

// Device work done for a call shows up in its span (Span::AnnotateDevice).
TEST(Rpcz, device_annotation_recorded) {
    Span* s = Span::CreateServerSpan(0, 0, 0, "x.Y", realtime_us());
    if (!s) {
        FLAGS_enable_rpcz = true;
        s = Span::CreateServerSpan(0, 0, 0, "x.Y", realtime_us());
    }
    ASSERT_TRUE(s != nullptr);
    s->AnnotateDevice("copy+crc32c 4 segs 262144 B dev0", 0.042f);
    const std::string d = s->Describe();
    EXPECT_TRUE(d.find("[gpu] copy+crc32c 4 segs 262144 B dev0 0.042 ms") != std::string::npos);
    delete s;
    FLAGS_enable_rpcz = false;
}

namespace {
// Server A answers by calling server B from inside its handler: the nested
// client call must join the caller's trace (reference: Span::tls_parent,
// span.cpp CreateClientSpan with a parent server span).
class CascadeEcho : public example::EchoService {
public:
    Channel* downstream = nullptr;
    void Echo(RpcController* c, const example::EchoRequest* req, example::EchoResponse* res, Closure* done) override {
        ClosureGuard g(done);
        TRACEPRINTF("cascade hop for %s", req->message().c_str());
        example::EchoService_Stub stub(downstream);
        Controller sub;
        example::EchoRequest r2;
        example::EchoResponse s2;
        r2.set_message(req->message() + ">B");
        stub.Echo(&sub, &r2, &s2, nullptr);
        if (sub.Failed()) {
            static_cast<Controller*>(c)->SetFailed(sub.ErrorCode(), "%s", sub.ErrorText().c_str());
            return;
        }
        res->set_message(s2.message());
    }
};
}  // namespace

TEST(Rpcz, cascade_calls_share_one_trace) {
    const std::string dir = make_tmpdir();
    ASSERT_FALSE(dir.empty());
    FLAGS_rpcz_database_dir = dir;
    FLAGS_enable_rpcz = true;
    EchoServer b;
    ASSERT_GT(b.port, 0);
    Channel to_b;
    ASSERT_EQ(to_b.Init(("127.0.0.1:" + std::to_string(b.port)).c_str(), nullptr), 0);
    Server a;
    CascadeEcho cascade;
    cascade.downstream = &to_b;
    a.AddService(&cascade, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions o;
    o.has_builtin_services = false;
    ASSERT_EQ(a.Start("127.0.0.1:0", &o), 0);
    Channel to_a;
    ASSERT_EQ(to_a.Init(("127.0.0.1:" + std::to_string(a.listen_port())).c_str(), nullptr), 0);

    const uint64_t t = echo_once(&to_a, "hop");
    ASSERT_TRUE(t != 0);
    // Records: client->A (C), A's server span (S) and B's server span (S).
    // As in the reference, a server span shares its span id with the client
    // span that called it, and the nested A->B client span is kept inside
    // A's server span (local parent) rather than stored on its own.
    std::vector<std::string> v = wait_trace(t, 3);
    ASSERT_EQ(v.size(), 3u);
    auto field = [](const std::string& x, const char* key) {
        const size_t at = x.find(key);
        return at == std::string::npos ? std::string() : x.substr(at + strlen(key), 16);
    };
    std::string client_span, a_span, b_parent;
    int annotated = 0;
    for (const std::string& x : v) {
        EXPECT_TRUE(x.find(string_printf("trace=%016llx", (unsigned long long)t)) != std::string::npos);
        annotated += x.find("cascade hop for hop") != std::string::npos;
        if (x[0] == 'C') client_span = field(x, "span=");
        if (x[0] == 'S' && field(x, "parent=") == "0000000000000000") a_span = field(x, "span=");
        if (x[0] == 'S' && field(x, "parent=") != "0000000000000000") b_parent = field(x, "parent=");
    }
    EXPECT_FALSE(client_span.empty());
    EXPECT_EQ(a_span, client_span);  // the call's two halves share one id
    EXPECT_EQ(b_parent, a_span);     // B was called from inside A
    EXPECT_EQ(annotated, 1);         // TRACEPRINTF lands in A's server span only
    // an unrelated call starts a new trace
    const uint64_t t2 = echo_once(&to_a, "again");
    EXPECT_TRUE(t2 != 0 && t2 != t);
    EXPECT_EQ(wait_trace(t2, 3).size(), 3u);
    FLAGS_enable_rpcz = false;
    a.Stop(0);
    a.Join();
}
