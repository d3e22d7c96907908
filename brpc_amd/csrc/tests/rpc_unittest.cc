// End-to-end RPC tests over loopback (spirit of reference
// test/brpc_channel_unittest.cpp, brpc_server_unittest.cpp,
// brpc_streaming_rpc_unittest.cpp): sync/async calls, attachments,
// timeouts, retries, backup requests, server errors, streams, naming
// services + load balancers.
#include <unistd.h>

#include <atomic>
#include <fstream>
#include <thread>
#include <vector>

#include "base/time.h"
#include "cluster/circuit_breaker.h"
#include "fiber/fiber.h"
#include "fiber/sync.h"
#include "cluster/naming_service.h"
#include "rpc/channel.h"
#include "rpc/errno.h"
#include "rpc/server.h"
#include "rpc/stream.h"
#include "services/echo_service.h"
#include "tests/test.h"

using namespace mrpc;

namespace {
struct TestServer {
    Server server;
    EchoServiceImpl echo;
    int port = 0;
    explicit TestServer(const ServerOptions* opt = nullptr) {
        server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        ServerOptions o = opt ? *opt : ServerOptions();
        o.has_builtin_services = false;
        if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
    }
    std::string addr() const { return "127.0.0.1:" + std::to_string(port); }
};
}  // namespace

TEST(Rpc, sync_echo_and_attachment) {
    TestServer ts;
    ASSERT_GT(ts.port, 0);
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 2000;
    ASSERT_EQ(ch.Init(ts.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    for (int i = 0; i < 100; ++i) {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("hello " + std::to_string(i));
        cntl.request_attachment().append("attach-" + std::to_string(i));
        stub.Echo(&cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        EXPECT_EQ(res.message(), "hello " + std::to_string(i));
        EXPECT_EQ(cntl.response_attachment().to_string(), "attach-" + std::to_string(i));
        EXPECT_GT(cntl.latency_us(), 0);
    }
    // large attachment (multi-block, > 64KB)
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("big");
    std::string big(1 << 20, 'x');
    for (size_t i = 0; i < big.size(); ++i) big[i] = (char)(i * 7);
    cntl.request_attachment().append(big);
    stub.Echo(&cntl, &req, &res, nullptr);
    ASSERT_FALSE(cntl.Failed());
    EXPECT_TRUE(cntl.response_attachment().equals(big));
    EXPECT_EQ(ts.echo.ncalls(), 101);
}

TEST(Rpc, async_many_concurrent) {
    TestServer ts;
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 5000;
    ASSERT_EQ(ch.Init(ts.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    const int N = 2000;
    std::atomic<int> ok{0}, done_count{0};
    fiber::CountdownEvent all(N);
    struct Call {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
    };
    std::vector<Call*> calls;
    for (int i = 0; i < N; ++i) {
        Call* c = new Call;
        c->req.set_message(std::to_string(i));
        calls.push_back(c);
        stub.Echo(&c->cntl, &c->req, &c->res, NewCallback([c, i, &ok, &all] {
            if (!c->cntl.Failed() && c->res.message() == std::to_string(i)) ok.fetch_add(1);
            all.signal();
        }));
    }
    all.wait();
    EXPECT_EQ(ok.load(), N);
    for (auto* c : calls) delete c;
}

TEST(Rpc, timeout_and_server_errors) {
    TestServer ts;
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 50;
    opt.max_retry = 0;
    ASSERT_EQ(ch.Init(ts.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("slow");
        req.set_sleep_us(300000);
        const int64_t t0 = monotonic_us();
        stub.Echo(&cntl, &req, &res, nullptr);
        EXPECT_TRUE(cntl.Failed());
        EXPECT_EQ(cntl.ErrorCode(), ERPCTIMEDOUT);
        EXPECT_LT(monotonic_us() - t0, 250000);
    }
    {
        Controller cntl;
        cntl.set_timeout_ms(2000);
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("fail");
        req.set_server_fail(true);
        req.set_code(EREQUEST);
        stub.Echo(&cntl, &req, &res, nullptr);
        EXPECT_EQ(cntl.ErrorCode(), EREQUEST);
        EXPECT_TRUE(cntl.ErrorText().find("server_fail") != std::string::npos);
    }
    {
        // missing required field -> client-side EREQUEST, never sent
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        stub.Echo(&cntl, &req, &res, nullptr);
        EXPECT_EQ(cntl.ErrorCode(), EREQUEST);
    }
}

TEST(Rpc, connection_refused_and_retry) {
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 1000;
    opt.max_retry = 2;
    ASSERT_EQ(ch.Init("127.0.0.1:1", &opt), 0);  // nothing listens on port 1
    example::EchoService_Stub stub(&ch);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("x");
    stub.Echo(&cntl, &req, &res, nullptr);
    EXPECT_TRUE(cntl.Failed());
    EXPECT_TRUE(cntl.ErrorCode() == ECONNREFUSED || cntl.ErrorCode() == EHOSTDOWN || cntl.ErrorCode() == EFAILEDSOCKET);
}

TEST(Rpc, naming_service_lb_and_retry_on_close) {
    TestServer s1, s2, s3;
    std::string list = "list://" + s1.addr() + "," + s2.addr() + "," + s3.addr();
    for (const char* lb : {"rr", "random", "wrr", "wr", "la", "c_murmurhash", "c_md5", "c_ketama"}) {
        Channel ch;
        ChannelOptions opt;
        opt.timeout_ms = 2000;
        ASSERT_EQ(ch.Init(list.c_str(), lb, &opt), 0);
        example::EchoService_Stub stub(&ch);
        int ok = 0;
        for (int i = 0; i < 60; ++i) {
            Controller cntl;
            cntl.set_request_code((uint64_t)i * 2654435761u);
            example::EchoRequest req;
            example::EchoResponse res;
            req.set_message("lb");
            stub.Echo(&cntl, &req, &res, nullptr);
            if (!cntl.Failed()) ++ok;
        }
        EXPECT_EQ(ok, 60);
    }
    // all three servers got traffic from rr
    EXPECT_GT(s1.echo.ncalls(), 0);
    EXPECT_GT(s2.echo.ncalls(), 0);
    EXPECT_GT(s3.echo.ncalls(), 0);
    // file:// naming service
    std::string path = "/tmp/mrpc_ns_test_" + std::to_string(getpid());
    {
        std::ofstream f(path);
        f << s1.addr() << "\n" << s2.addr() << " 2\n";
    }
    Channel fch;
    ChannelOptions fopt;
    fopt.timeout_ms = 2000;
    ASSERT_EQ(fch.Init(("file://" + path).c_str(), "rr", &fopt), 0);
    example::EchoService_Stub fstub(&fch);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("file");
    fstub.Echo(&cntl, &req, &res, nullptr);
    EXPECT_FALSE(cntl.Failed());
    unlink(path.c_str());
}

TEST(Rpc, retry_when_server_closes_connection) {
    TestServer s1;
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 2000;
    opt.max_retry = 3;
    ASSERT_EQ(ch.Init(s1.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("close");
    req.set_close_fd(true);
    stub.Echo(&cntl, &req, &res, nullptr);
    // every retry also closes: fails with a connection error after retries
    EXPECT_TRUE(cntl.Failed());
    EXPECT_GE(cntl.retried_count(), 1);
}

TEST(Rpc, backup_request) {
    TestServer s1;
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 3000;
    opt.backup_request_ms = 20;
    ASSERT_EQ(ch.Init(s1.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("slow");
    req.set_sleep_us(100000);
    stub.Echo(&cntl, &req, &res, nullptr);
    EXPECT_FALSE(cntl.Failed());
    EXPECT_TRUE(cntl.has_backup_request());
    EXPECT_EQ(res.message(), "slow");
}

TEST(Rpc, server_max_concurrency) {
    ServerOptions so;
    so.max_concurrency = 1;
    TestServer ts(&so);
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 3000;
    opt.max_retry = 0;
    ASSERT_EQ(ch.Init(ts.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    std::atomic<int> limited{0}, ok{0};
    fiber::CountdownEvent ev(8);
    for (int i = 0; i < 8; ++i) {
        fiber::start([&] {
            Controller cntl;
            example::EchoRequest req;
            example::EchoResponse res;
            req.set_message("x");
            req.set_sleep_us(50000);
            stub.Echo(&cntl, &req, &res, nullptr);
            if (cntl.ErrorCode() == ELIMIT) limited++;
            else if (!cntl.Failed()) ok++;
            ev.signal();
        });
    }
    ev.wait();
    EXPECT_GT(limited.load(), 0);
    EXPECT_GT(ok.load(), 0);
}

namespace {
class StreamReceiver : public StreamInputHandler {
public:
    int on_received_messages(StreamId, Buf* const messages[], size_t size) override {
        std::lock_guard<std::mutex> g(mu);
        for (size_t i = 0; i < size; ++i) got.push_back(messages[i]->to_string());
        return 0;
    }
    void on_closed(StreamId) override { closed = true; }
    std::mutex mu;
    std::vector<std::string> got;
    std::atomic<bool> closed{false};
};

class StreamEchoService : public example::EchoService {
public:
    void Echo(RpcController* cb, const example::EchoRequest* req, example::EchoResponse* res, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = static_cast<Controller*>(cb);
        StreamOptions so;
        so.handler = &receiver;
        StreamId sid;
        if (StreamAccept(&sid, *cntl, &so) != 0) {
            cntl->SetFailed("fail to accept stream");
            return;
        }
        res->set_message(req->message());
    }
    StreamReceiver receiver;
};
}  // namespace

TEST(Rpc, streaming_in_order_with_flow_control) {
    Server server;
    StreamEchoService svc;
    server.AddService(&svc, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions so;
    so.has_builtin_services = false;
    ASSERT_EQ(server.Start("127.0.0.1:0", &so), 0);
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 3000;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    Controller cntl;
    StreamId sid;
    StreamOptions copt;
    copt.max_buf_size = 64 * 1024;
    copt.min_buf_size = 16 * 1024;
    ASSERT_EQ(StreamCreate(&sid, cntl, &copt), 0);
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("stream");
    stub.Echo(&cntl, &req, &res, nullptr);
    ASSERT_FALSE(cntl.Failed());
    EXPECT_TRUE(StreamIsConnected(sid));
    const int N = 500;
    for (int i = 0; i < N; ++i) {
        Buf b;
        b.append("msg-" + std::to_string(i) + std::string(1000, 'p'));
        for (;;) {
            int rc = StreamWrite(sid, b);
            if (rc == 0) break;
            ASSERT_EQ(rc, EAGAIN);
            timespec ts = realtime_after_us(1000000);
            ASSERT_EQ(StreamWait(sid, &ts), 0);
        }
    }
    auto received = [&] {
        std::lock_guard<std::mutex> g(svc.receiver.mu);
        return (int)svc.receiver.got.size();
    };
    for (int i = 0; i < 300 && received() < N; ++i) fiber::usleep(10000);
    ASSERT_EQ(received(), N);
    std::vector<std::string> got;
    {
        std::lock_guard<std::mutex> g(svc.receiver.mu);
        got = svc.receiver.got;
    }
    for (int i = 0; i < N; ++i) EXPECT_EQ(got[i].substr(0, 4 + std::to_string(i).size()), "msg-" + std::to_string(i));
    StreamClose(sid);
    for (int i = 0; i < 200 && !svc.receiver.closed; ++i) fiber::usleep(5000);
    EXPECT_TRUE(svc.receiver.closed.load());
}

TEST(Rpc, circuit_breaker_isolates) {
    const SocketId fake = 0x7777000000000001ull;
    for (int i = 0; i < 4000 && !IsIsolatedByCircuitBreaker(fake); ++i) FeedCircuitBreaker(fake, EINTERNAL, 1000);
    EXPECT_TRUE(IsIsolatedByCircuitBreaker(fake));
}

TEST(Rpc, domain_list_https_and_redis_naming_services) {
    for (const char* scheme : {"dns", "https", "redis", "dlist"}) {
        std::unique_ptr<NamingService> ns(CreateNamingService(scheme));
        ASSERT_TRUE(ns != nullptr);
    }
    auto* dl = static_cast<PeriodicNamingService*>(CreateNamingService("dlist"));
    std::vector<ServerNode> servers;
    EXPECT_EQ(dl->GetServers("localhost:8001, 127.0.0.1:8002,localhost:8001", &servers), 0);
    EXPECT_EQ(servers.size(), 2u);  // localhost:8001 deduplicated
    delete dl;
    auto* https = static_cast<PeriodicNamingService*>(CreateNamingService("https"));
    servers.clear();
    EXPECT_EQ(https->GetServers("localhost", &servers), 0);
    ASSERT_FALSE(servers.empty());
    EXPECT_EQ(servers[0].addr.port, 443);
    delete https;
    auto* redis = static_cast<PeriodicNamingService*>(CreateNamingService("redis"));
    servers.clear();
    EXPECT_EQ(redis->GetServers("127.0.0.1", &servers), 0);
    ASSERT_FALSE(servers.empty());
    EXPECT_EQ(servers[0].addr.port, 6379);
    delete redis;
}

// IPv6 endpoints (reference: butil/details/extended_endpoint.hpp:155-311):
// parse/print round trips, ordering/hash distinctness, and a server on
// [::1] answering baidu_std and http clients, with the remote side seen
// as an IPv6 endpoint.
TEST(Rpc, ipv6_endpoints_and_loopback_echo) {
    EndPoint ep;
    ASSERT_EQ(str2endpoint("[::1]:8000", &ep), 0);
    EXPECT_TRUE(ep.is_ipv6());
    EXPECT_EQ(ep.port, 8000);
    EXPECT_EQ(ep.to_string(), "[::1]:8000");
    ASSERT_EQ(str2endpoint("[2001:db8::a:1]:65535", &ep), 0);
    EXPECT_EQ(ep.to_string(), "[2001:db8::a:1]:65535");
    EXPECT_EQ(ep.ip_string(), "2001:db8::a:1");
    EXPECT_NE(str2endpoint("::1:80", &ep), 0);      // bare v6 needs brackets
    EXPECT_NE(str2endpoint("[::1]80", &ep), 0);
    EXPECT_NE(str2endpoint("[::g]:80", &ep), 0);
    EXPECT_NE(str2endpoint("[::1]:70000", &ep), 0);
    ASSERT_EQ(str2endpoint("::", 81, &ep), 0);
    EXPECT_EQ(ep.to_string(), "[::]:81");
    ASSERT_EQ(str2endpoint("[::1]", 82, &ep), 0);
    EXPECT_EQ(ep.to_string(), "[::1]:82");
    EndPoint a, b, c;
    ASSERT_EQ(str2endpoint("[::1]:1", &a), 0);
    ASSERT_EQ(str2endpoint("[::2]:1", &b), 0);
    ASSERT_EQ(str2endpoint("0.0.0.1:1", &c), 0);
    EXPECT_TRUE(a != b && a != c && (a < b) != (b < a) && (a < c) != (c < a));
    EXPECT_NE(EndPointHash()(a), EndPointHash()(b));
    // IPv4 parsing is unchanged
    ASSERT_EQ(str2endpoint("127.0.0.1:80", &ep), 0);
    EXPECT_FALSE(ep.is_ipv6());
    EXPECT_EQ(ep.to_string(), "127.0.0.1:80");

    Server server;
    EchoServiceImpl echo;
    server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions so;
    so.has_builtin_services = false;
    ASSERT_EQ(server.Start("[::1]:0", &so), 0);
    ASSERT_TRUE(server.listen_address().is_ipv6());
    const std::string addr = server.listen_address().to_string();
    EXPECT_EQ(addr.compare(0, 5, "[::1]"), 0);
    for (const char* proto : {"baidu_std", "http"}) {
        Channel ch;
        ChannelOptions opt;
        opt.timeout_ms = 2000;
        opt.protocol = proto;
        ASSERT_EQ(ch.Init(addr.c_str(), &opt), 0);
        example::EchoService_Stub stub(&ch);
        for (int i = 0; i < 20; ++i) {
            Controller cntl;
            example::EchoRequest req;
            example::EchoResponse res;
            req.set_message("v6 " + std::to_string(i));
            stub.Echo(&cntl, &req, &res, nullptr);
            ASSERT_FALSE(cntl.Failed());
            EXPECT_EQ(res.message(), "v6 " + std::to_string(i));
            EXPECT_TRUE(cntl.remote_side().is_ipv6());
            EXPECT_EQ(cntl.remote_side(), server.listen_address());
        }
    }
    // a naming-service list of v6 servers through a load balancer
    Channel lbch;
    ChannelOptions lo;
    lo.timeout_ms = 2000;
    ASSERT_EQ(lbch.Init(("list://" + addr + "," + addr).c_str(), "rr", &lo), 0);
    example::EchoService_Stub lstub(&lbch);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("lb");
    lstub.Echo(&cntl, &req, &res, nullptr);
    ASSERT_FALSE(cntl.Failed());
    EXPECT_EQ(res.message(), "lb");
    server.Stop(0);
    server.Join();
}
