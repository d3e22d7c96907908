// Server lifecycle and options (rpc/server.h), in the spirit of the
// reference's test/brpc_server_unittest.cpp: start/stop/join and restart,
// enabled_protocols (valid, empty, unknown, enforced), service registration
// (duplicates, removal, restful mappings and their conflicts, URI forms),
// missing required fields, builtin services on/off and the internal port,
// idle connection closing, port ranges, the pid file, max body size,
// server-wide and per-method max_concurrency, and stopping under load.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "base/flags.h"
#include "base/time.h"
#include "http/http_header.h"
#include "mrpc/proto/echo.pb.h"
#include "mrpc/proto/test_services.pb.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

class RawImpl : public test::HttpTest {
public:
    void Push(RpcController*, const test::Empty*, test::Empty*, Closure* done) override { done->Run(); }
    void Raw(RpcController* c, const test::Empty*, test::Empty*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = static_cast<Controller*>(c);
        cntl->response_attachment().append("raw:" + cntl->http_request().unresolved_path());
    }
    void Rich(RpcController*, const test::Rich* req, test::Rich* res, Closure* done) override {
        ClosureGuard g(done);
        *res = *req;
    }
};

std::unique_ptr<Channel> channel(int port, const char* proto = "baidu_std", int timeout_ms = 2000) {
    std::unique_ptr<Channel> ch(new Channel);
    ChannelOptions opt;
    opt.protocol = proto;
    opt.timeout_ms = timeout_ms;
    opt.max_retry = 0;
    if (ch->Init(("127.0.0.1:" + std::to_string(port)).c_str(), &opt) != 0) ch.reset();
    return ch;
}

int echo(Channel* ch, const std::string& msg, int sleep_us = 0, std::string* out = nullptr) {
    example::EchoService_Stub stub(ch);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message(msg);
    if (sleep_us) req.set_sleep_us(sleep_us);
    stub.Echo(&cntl, &req, &res, nullptr);
    if (out) *out = res.message();
    return cntl.ErrorCode();
}

int http_get(int port, const std::string& path, std::string* body = nullptr, int* status = nullptr) {
    auto ch = channel(port, "http");
    if (!ch) return -1;
    Controller cntl;
    cntl.http_request().uri().set_path(path);
    ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    if (body) *body = cntl.response_attachment().to_string();
    if (status) *status = cntl.http_response().status_code();
    return cntl.ErrorCode();
}

int free_port() {
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    bind(fd, (sockaddr*)&a, sizeof(a));
    socklen_t len = sizeof(a);
    getsockname(fd, (sockaddr*)&a, &len);
    close(fd);
    return ntohs(a.sin_port);
}

}  // namespace

TEST(Server, sanity_start_stop_join_restart) {
    Server s;
    EchoServiceImpl echo_svc;
    ASSERT_EQ(s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE), 0);
    EXPECT_FALSE(s.IsRunning());
    ASSERT_EQ(s.Start("127.0.0.1:0", nullptr), 0);
    EXPECT_TRUE(s.IsRunning());
    const int port = s.listen_port();
    EXPECT_GT(port, 0);
    EXPECT_NE(s.Start("127.0.0.1:0", nullptr), 0);  // already running
    auto ch = channel(port);
    std::string got;
    EXPECT_EQ(echo(ch.get(), "one", 0, &got), 0);
    EXPECT_EQ(got, "one");
    EXPECT_EQ(s.Stop(0), 0);
    EXPECT_EQ(s.Stop(0), 0);  // idempotent
    EXPECT_EQ(s.Join(), 0);
    EXPECT_FALSE(s.IsRunning());
    EXPECT_NE(echo(ch.get(), "after stop"), 0);
    // the same object serves again
    ASSERT_EQ(s.Start("127.0.0.1:0", nullptr), 0);
    auto ch2 = channel(s.listen_port());
    EXPECT_EQ(echo(ch2.get(), "two", 0, &got), 0);
    EXPECT_EQ(got, "two");
}

TEST(Server, unknown_protocol_in_enabled_protocols_fails_start) {
    Server s;
    EchoServiceImpl echo_svc;
    s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions o;
    o.enabled_protocols = "baidu_std no_such_protocol";
    EXPECT_NE(s.Start("127.0.0.1:0", &o), 0);
    EXPECT_FALSE(s.IsRunning());
    o.enabled_protocols = "baidu_std http";  // fixed: now it starts
    EXPECT_EQ(s.Start("127.0.0.1:0", &o), 0);
}

TEST(Server, empty_enabled_protocols_serves_every_protocol) {
    Server s;
    EchoServiceImpl echo_svc;
    s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions o;
    o.enabled_protocols = "";
    ASSERT_EQ(s.Start("127.0.0.1:0", &o), 0);
    for (const char* proto : {"baidu_std", "http", "h2", "h2:grpc", "hulu_pbrpc", "sofa_pbrpc"}) {
        auto ch = channel(s.listen_port(), proto);
        ASSERT_TRUE(ch != nullptr);
        std::string got;
        EXPECT_EQ(echo(ch.get(), proto, 0, &got), 0);
        EXPECT_EQ(got, proto);
    }
}

TEST(Server, only_enabled_protocols_are_served) {
    Server s;
    EchoServiceImpl echo_svc;
    s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions o;
    o.enabled_protocols = "http";
    ASSERT_EQ(s.Start("127.0.0.1:0", &o), 0);
    auto http = channel(s.listen_port(), "http");
    EXPECT_EQ(echo(http.get(), "http ok"), 0);
    auto baidu = channel(s.listen_port(), "baidu_std", 500);
    EXPECT_NE(echo(baidu.get(), "not served"), 0);
}

TEST(Server, uri_forms_reach_the_method) {
    Server s;
    EchoServiceImpl echo_svc;
    RawImpl raw;
    s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE);
    s.AddService(&raw, SERVER_DOESNT_OWN_SERVICE);
    ASSERT_EQ(s.Start("127.0.0.1:0", nullptr), 0);
    std::string body;
    for (const char* path : {"/HttpTest/Raw", "/mrpc.test.HttpTest/Raw", "//HttpTest//Raw", "/HttpTest/Raw/"}) {
        EXPECT_EQ(http_get(s.listen_port(), path, &body), 0);
        EXPECT_EQ(body, "raw:");
    }
    EXPECT_EQ(http_get(s.listen_port(), "/HttpTest/Raw/a/b", &body), 0);
    EXPECT_EQ(body, "raw:a/b");  // the rest of the path is the unresolved part
    int status = 0;
    EXPECT_EQ(http_get(s.listen_port(), "/HttpTest/NoSuch", &body, &status), ENOMETHOD);
    EXPECT_EQ(status, 404);
    EXPECT_EQ(http_get(s.listen_port(), "/NoSuchService/Raw", &body, &status), ENOMETHOD);
}

TEST(Server, missing_required_fields_are_rejected) {
    Server s;
    EchoServiceImpl echo_svc;
    s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE);
    ASSERT_EQ(s.Start("127.0.0.1:0", nullptr), 0);
    // the client refuses to send an uninitialized request
    auto ch = channel(s.listen_port());
    example::EchoService_Stub stub(ch.get());
    Controller cntl;
    example::EchoRequest req;  // no message
    example::EchoResponse res;
    stub.Echo(&cntl, &req, &res, nullptr);
    EXPECT_EQ(cntl.ErrorCode(), EREQUEST);
    // over http the server checks: empty json object
    auto http = channel(s.listen_port(), "http");
    Controller c2;
    c2.http_request().uri().set_path("/EchoService/Echo");
    c2.http_request().set_method(HTTP_METHOD_POST);
    c2.request_attachment().append("{}");
    http->CallMethod(nullptr, &c2, nullptr, nullptr, nullptr);
    EXPECT_EQ(c2.ErrorCode(), EREQUEST);
    EXPECT_EQ(c2.http_response().status_code(), 400);
}

TEST(Server, restful_mappings_route_and_conflicts_fail_cleanly) {
    Server s;
    RawImpl raw;
    EchoServiceImpl echo_svc;
    ASSERT_EQ(s.AddService(&raw, SERVER_DOESNT_OWN_SERVICE, "/v1/things/* => Raw, /v1/rich => Rich"), 0);
    // a path mapped twice, a bad target, a relative path: refused, and the
    // service is not half-registered
    EXPECT_NE(s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE, "/v1/rich => Echo"), 0);
    EXPECT_TRUE(s.FindServiceByName("EchoService") == nullptr);
    EXPECT_NE(s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE, "/x => NoSuchMethod"), 0);
    EXPECT_NE(s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE, "relative => Echo"), 0);
    EXPECT_TRUE(s.FindServiceByName("EchoService") == nullptr);
    ASSERT_EQ(s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE, "/v2/echo => Echo"), 0);
    ASSERT_EQ(s.Start("127.0.0.1:0", nullptr), 0);
    std::string body;
    EXPECT_EQ(http_get(s.listen_port(), "/v1/things/a/b/c", &body), 0);
    EXPECT_EQ(body, "raw:a/b/c");
    // the default URL keeps working next to the mapping
    EXPECT_EQ(http_get(s.listen_port(), "/HttpTest/Raw", &body), 0);
    auto http = channel(s.listen_port(), "http");
    Controller cntl;
    cntl.http_request().uri().set_path("/v2/echo");
    cntl.http_request().set_method(HTTP_METHOD_POST);
    cntl.request_attachment().append("{\"message\":\"restful\"}");
    http->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    ASSERT_EQ(cntl.ErrorCode(), 0);
    EXPECT_TRUE(cntl.response_attachment().to_string().find("restful") != std::string::npos);
}

TEST(Server, builtin_pages_win_over_a_master_service_path) {
    Server s;
    RawImpl raw;
    ServerOptions o;
    ASSERT_EQ(s.AddService(&raw, SERVER_DOESNT_OWN_SERVICE, "/anything/* => Raw"), 0);
    ASSERT_EQ(s.Start("127.0.0.1:0", &o), 0);
    std::string body;
    EXPECT_EQ(http_get(s.listen_port(), "/status", &body), 0);  // builtin
    EXPECT_TRUE(body.find("raw:") == std::string::npos);
    EXPECT_EQ(http_get(s.listen_port(), "/anything/else", &body), 0);
    EXPECT_EQ(body, "raw:else");
}

TEST(Server, add_and_remove_services) {
    Server s;
    EchoServiceImpl echo_svc;
    RawImpl raw;
    EXPECT_EQ(s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE), 0);
    EXPECT_NE(s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE), 0);  // twice
    EXPECT_NE(s.AddService(nullptr, SERVER_DOESNT_OWN_SERVICE), 0);
    EXPECT_EQ(s.AddService(&raw, SERVER_DOESNT_OWN_SERVICE), 0);
    EXPECT_EQ(s.service_count(), 2u);
    EXPECT_TRUE(s.FindServiceByName("EchoService") == &echo_svc);
    EXPECT_TRUE(s.FindServiceByFullName("example.EchoService") == &echo_svc);
    EXPECT_TRUE(s.FindServiceByFullName("EchoService") == nullptr);
    EXPECT_EQ(s.RemoveService(&raw), 0);
    EXPECT_NE(s.RemoveService(&raw), 0);  // not there any more
    EXPECT_EQ(s.service_count(), 1u);
    ASSERT_EQ(s.Start("127.0.0.1:0", nullptr), 0);
    // no registration changes while running
    EXPECT_NE(s.AddService(&raw, SERVER_DOESNT_OWN_SERVICE), 0);
    EXPECT_NE(s.RemoveService(&echo_svc), 0);
    std::string body;
    int status = 0;
    EXPECT_EQ(http_get(s.listen_port(), "/HttpTest/Raw", &body, &status), ENOMETHOD);
    s.Stop(0);
    s.Join();
    EXPECT_EQ(s.AddService(&raw, SERVER_DOESNT_OWN_SERVICE), 0);  // allowed again once stopped
}

TEST(Server, server_owned_services_are_deleted_with_it) {
    static std::atomic<int> alive{0};
    struct Counted : public EchoServiceImpl {
        Counted() { alive.fetch_add(1); }
        ~Counted() override { alive.fetch_sub(1); }
    };
    {
        Server s;
        ASSERT_EQ(s.AddService(new Counted, SERVER_OWNS_SERVICE), 0);
        EXPECT_EQ(alive.load(), 1);
    }
    EXPECT_EQ(alive.load(), 0);
}

TEST(Server, idle_connections_are_closed) {
    Server s;
    EchoServiceImpl echo_svc;
    s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions o;
    o.idle_timeout_sec = 1;
    ASSERT_EQ(s.Start("127.0.0.1:0", &o), 0);
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)s.listen_port());
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    ASSERT_EQ(connect(fd, (sockaddr*)&a, sizeof(a)), 0);
    // say nothing: the server closes the connection after ~1-2 s
    pollfd p{fd, POLLIN, 0};
    const int64_t t0 = monotonic_us();
    int closed = 0;
    while (monotonic_us() - t0 < 5000000) {
        if (poll(&p, 1, 100) > 0) {
            char c;
            if (read(fd, &c, 1) <= 0) {
                closed = 1;
                break;
            }
        }
    }
    close(fd);
    EXPECT_EQ(closed, 1);
    EXPECT_GT(monotonic_us() - t0, 500000);
}

TEST(Server, start_on_a_port_range_skips_taken_ports) {
    const int busy = free_port();
    Server first;
    EchoServiceImpl e1, e2;
    first.AddService(&e1, SERVER_DOESNT_OWN_SERVICE);
    if (first.Start(busy, nullptr) != 0) return;  // raced for the port: nothing to test
    Server second;
    second.AddService(&e2, SERVER_DOESNT_OWN_SERVICE);
    ASSERT_EQ(second.Start(busy, busy + 20, nullptr), 0);
    EXPECT_NE(second.listen_port(), busy);
    EXPECT_GT(second.listen_port(), busy);
    EXPECT_LE(second.listen_port(), busy + 20);
    Server third;
    EchoServiceImpl e3;
    third.AddService(&e3, SERVER_DOESNT_OWN_SERVICE);
    EXPECT_NE(third.Start(busy, busy, nullptr), 0);  // the only port is taken
}

TEST(Server, pid_file_is_written_with_its_directories_and_removed) {
    char tmpl[] = "/tmp/mrpc_pid_XXXXXX";
    ASSERT_TRUE(mkdtemp(tmpl) != nullptr);
    const std::string path = std::string(tmpl) + "/a/b/server.pid";
    {
        Server s;
        EchoServiceImpl echo_svc;
        s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE);
        ServerOptions o;
        o.pid_file = path;
        ASSERT_EQ(s.Start("127.0.0.1:0", &o), 0);
        std::ifstream in(path);
        long pid = 0;
        in >> pid;
        EXPECT_EQ(pid, (long)getpid());
    }
    struct stat st;
    EXPECT_NE(stat(path.c_str(), &st), 0);  // gone with the server
    rmdir((std::string(tmpl) + "/a/b").c_str());
    rmdir((std::string(tmpl) + "/a").c_str());
    rmdir(tmpl);
}

TEST(Server, builtin_services_can_be_turned_off) {
    Server on, off;
    EchoServiceImpl e1, e2;
    on.AddService(&e1, SERVER_DOESNT_OWN_SERVICE);
    off.AddService(&e2, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions o;
    ASSERT_EQ(on.Start("127.0.0.1:0", &o), 0);
    o.has_builtin_services = false;
    ASSERT_EQ(off.Start("127.0.0.1:0", &o), 0);
    std::string body;
    EXPECT_EQ(http_get(on.listen_port(), "/health", &body), 0);
    EXPECT_EQ(http_get(off.listen_port(), "/health", &body), ENOMETHOD);
    EXPECT_EQ(off.service_count(), 1u);
    auto ch = channel(off.listen_port());
    EXPECT_EQ(echo(ch.get(), "still serves"), 0);
}

TEST(Server, internal_port_keeps_builtin_pages_off_the_public_one) {
    Server s;
    EchoServiceImpl echo_svc;
    s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions o;
    o.internal_port = free_port();
    ASSERT_EQ(s.Start("127.0.0.1:0", &o), 0);
    std::string body;
    EXPECT_NE(http_get(s.listen_port(), "/status", &body), 0);   // public port: refused
    EXPECT_EQ(http_get(o.internal_port, "/status", &body), 0);   // internal port: served
    auto ch = channel(s.listen_port());
    EXPECT_EQ(echo(ch.get(), "public rpc"), 0);                  // user services stay public
}

TEST(Server, too_big_message_is_refused) {
    std::string prev;
    GetFlag("max_body_size", &prev);
    Server s;
    EchoServiceImpl echo_svc;
    s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE);
    ASSERT_EQ(s.Start("127.0.0.1:0", nullptr), 0);
    auto ch = channel(s.listen_port());
    EXPECT_EQ(echo(ch.get(), std::string(100000, 'a')), 0);
    SetFlag("max_body_size", "50000");
    EXPECT_NE(echo(ch.get(), std::string(100000, 'b')), 0);
    SetFlag("max_body_size", prev);
    // the refused connection was closed; the endpoint's connection revives
    // through the health check, then the same size goes through again
    int rc = -1;
    for (int i = 0; i < 60 && rc != 0; ++i) {
        auto ch2 = channel(s.listen_port());
        rc = echo(ch2.get(), std::string(100000, 'c'));
        if (rc != 0) usleep(100000);
    }
    EXPECT_EQ(rc, 0);
}

TEST(Server, server_wide_max_concurrency_rejects_the_excess) {
    Server s;
    EchoServiceImpl echo_svc;
    s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions o;
    o.max_concurrency = 2;
    ASSERT_EQ(s.Start("127.0.0.1:0", &o), 0);
    EXPECT_EQ(s.max_concurrency(), 2);
    std::atomic<int> ok{0}, limited{0};
    std::vector<std::thread> ths;
    for (int i = 0; i < 6; ++i) {
        ths.emplace_back([&] {
            auto ch = channel(s.listen_port(), "baidu_std", 3000);
            const int rc = echo(ch.get(), "slow", 200000);
            if (rc == 0) ok.fetch_add(1);
            else if (rc == ELIMIT) limited.fetch_add(1);
        });
    }
    for (auto& th : ths) th.join();
    EXPECT_GE(ok.load(), 2);
    EXPECT_GE(limited.load(), 1);
    EXPECT_EQ(ok.load() + limited.load(), 6);
}

TEST(Server, per_method_max_concurrency) {
    Server s;
    EchoServiceImpl echo_svc;
    s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE);
    EXPECT_EQ(s.SetMaxConcurrencyOf("example.EchoService.Echo", 1), 0);
    EXPECT_NE(s.SetMaxConcurrencyOf("example.EchoService.NoSuch", 1), 0);
    EXPECT_TRUE(s.MaxConcurrencyOf("example.EchoService.Echo") == AdaptiveMaxConcurrency(1));
    ASSERT_EQ(s.Start("127.0.0.1:0", nullptr), 0);
    std::atomic<int> ok{0}, limited{0};
    std::vector<std::thread> ths;
    for (int i = 0; i < 4; ++i) {
        ths.emplace_back([&] {
            auto ch = channel(s.listen_port(), "baidu_std", 3000);
            const int rc = echo(ch.get(), "slow", 200000);
            if (rc == 0) ok.fetch_add(1);
            else if (rc == ELIMIT) limited.fetch_add(1);
        });
    }
    for (auto& th : ths) th.join();
    EXPECT_GE(ok.load(), 1);
    EXPECT_GE(limited.load(), 1);
}

TEST(Server, stop_under_load_then_join_returns) {
    Server s;
    EchoServiceImpl echo_svc;
    s.AddService(&echo_svc, SERVER_DOESNT_OWN_SERVICE);
    ASSERT_EQ(s.Start("127.0.0.1:0", nullptr), 0);
    std::atomic<bool> stop{false};
    std::atomic<int> done{0}, ok{0};
    std::vector<std::thread> ths;
    for (int t = 0; t < 4; ++t) {
        ths.emplace_back([&] {
            auto ch = channel(s.listen_port(), "baidu_std", 1000);
            while (!stop.load()) {
                if (echo(ch.get(), "load", 1000) == 0) ok.fetch_add(1);
                done.fetch_add(1);
            }
        });
    }
    while (ok.load() < 50) usleep(1000);
    const int64_t t0 = monotonic_us();
    s.Stop(0);
    s.Join();
    EXPECT_LT(monotonic_us() - t0, 3000000);
    stop = true;
    for (auto& th : ths) th.join();
    EXPECT_GT(done.load(), ok.load() - 1);
    EXPECT_FALSE(s.IsRunning());
}

TEST(Server, start_with_a_port_number_or_a_string) {
    Server a, b;
    EchoServiceImpl e1, e2;
    a.AddService(&e1, SERVER_DOESNT_OWN_SERVICE);
    b.AddService(&e2, SERVER_DOESNT_OWN_SERVICE);
    const int p = free_port();
    if (a.Start(std::to_string(p).c_str(), nullptr) == 0) {  // "port" alone
        EXPECT_EQ(a.listen_port(), p);
    }
    EXPECT_NE(b.Start("not an address at all", nullptr), 0);
    EXPECT_EQ(b.Start("localhost:0", nullptr), 0);
    EXPECT_GT(b.listen_port(), 0);
}
