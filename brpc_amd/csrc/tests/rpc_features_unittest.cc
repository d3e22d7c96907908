// Focused RPC-core behaviours (spirit of the reference's
// test/brpc_channel_unittest.cpp and brpc_server_unittest.cpp: one feature
// per case — per-call options, retry accounting, cancel, compression,
// authentication, connection types, server-side controller fields, method
// limits, shutdown).
#include <unistd.h>

#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "base/time.h"
#include "fiber/fiber.h"
#include "fiber/sync.h"
#include "mrpc/proto/echo.pb.h"
#include "rpc/authenticator.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/retry_policy.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

// Echo that reports what the server-side controller saw.
class InspectEcho : public example::EchoService {
public:
    void Echo(RpcController* c, const example::EchoRequest* req, example::EchoResponse* res, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = static_cast<Controller*>(c);
        ++calls;
        {
            std::lock_guard<std::mutex> lk(mu);  // concurrent calls land here together
            last_log_id = cntl->log_id();
            last_remote = cntl->remote_side().to_string();
            last_local = cntl->local_side().to_string();
            last_req_compress = (int)cntl->request_compress_type();
            server_side = cntl->is_server_side();
        }
        if (req->sleep_us() > 0) fiber::usleep((uint64_t)req->sleep_us());
        if (req->server_fail()) {
            cntl->SetFailed(req->code() ? req->code() : EINTERNAL, "asked to fail");
            return;
        }
        res->set_message(req->message());
        cntl->response_attachment().append(cntl->request_attachment());
        if (req->code() > 0) cntl->set_response_compress_type((CompressType)req->code());
    }
    std::atomic<int> calls{0};
    std::mutex mu;
    uint64_t last_log_id = 0;
    std::string last_remote, last_local;
    int last_req_compress = -1;
    bool server_side = false;
};

struct Fixture {
    InspectEcho echo;  // outlives the server
    Server server;
    int port = 0;
    explicit Fixture(ServerOptions o = ServerOptions()) {
        server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        o.has_builtin_services = false;
        if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
    }
    ~Fixture() {
        server.Stop(0);
        server.Join();
    }
    std::string addr() const { return "127.0.0.1:" + std::to_string(port); }
};

bool Call(Channel* ch, Controller* cntl, const std::string& msg, example::EchoResponse* res,
          const example::EchoRequest* tmpl = nullptr) {
    example::EchoService_Stub stub(ch);
    example::EchoRequest req;
    if (tmpl) req = *tmpl;
    req.set_message(msg);
    stub.Echo(cntl, &req, res, nullptr);
    return !cntl->Failed();
}

class TokenAuth : public Authenticator {
public:
    explicit TokenAuth(std::string t) : _token(std::move(t)) {}
    int GenerateCredential(std::string* out) const override {
        *out = _token;
        return 0;
    }
    int VerifyCredential(const std::string& in, const EndPoint&, AuthContext* ctx) const override {
        if (in != "secret") return -1;
        ctx->set_user("tester");
        return 0;
    }

private:
    std::string _token;
};

}  // namespace

TEST(RpcFeatures, per_call_timeout_overrides_channel) {
    Fixture f;
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 5000;
    opt.max_retry = 0;
    ASSERT_EQ(ch.Init(f.addr().c_str(), &opt), 0);
    example::EchoRequest slow;
    slow.set_sleep_us(300000);
    Controller c1;
    c1.set_timeout_ms(50);
    example::EchoResponse r1;
    const int64_t t0 = monotonic_us();
    EXPECT_FALSE(Call(&ch, &c1, "x", &r1, &slow));
    EXPECT_EQ(c1.ErrorCode(), ERPCTIMEDOUT);
    EXPECT_LT(monotonic_us() - t0, 250000);
    Controller c2;  // channel default (5 s) lets it finish
    example::EchoResponse r2;
    EXPECT_TRUE(Call(&ch, &c2, "y", &r2, &slow));
}

TEST(RpcFeatures, log_id_and_sides_reach_the_server) {
    Fixture f;
    Channel ch;
    ASSERT_EQ(ch.Init(f.addr().c_str(), nullptr), 0);
    Controller c;
    c.set_log_id(0x1234567890ULL);
    example::EchoResponse r;
    ASSERT_TRUE(Call(&ch, &c, "hi", &r));
    EXPECT_EQ(f.echo.last_log_id, 0x1234567890ULL);
    EXPECT_TRUE(f.echo.server_side);
    EXPECT_EQ(f.echo.last_local, f.addr());
    EXPECT_EQ(f.echo.last_remote, c.local_side().to_string());  // the client's end
    EXPECT_EQ(c.remote_side().to_string(), f.addr());
    EXPECT_FALSE(c.is_server_side());
    EXPECT_GT(c.latency_us(), 0);
}

TEST(RpcFeatures, server_errors_are_not_retried) {
    Fixture f;
    Channel ch;
    ChannelOptions opt;
    opt.max_retry = 5;
    ASSERT_EQ(ch.Init(f.addr().c_str(), &opt), 0);
    example::EchoRequest fail;
    fail.set_server_fail(true);
    fail.set_code(4242);
    Controller c;
    example::EchoResponse r;
    EXPECT_FALSE(Call(&ch, &c, "x", &r, &fail));
    EXPECT_EQ(c.ErrorCode(), 4242);
    EXPECT_EQ(c.retried_count(), 0);
    EXPECT_EQ(f.echo.calls.load(), 1);  // the default policy retries connection errors only
}

TEST(RpcFeatures, custom_retry_policy_retries_application_errors) {
    class RetryEverything : public RetryPolicy {
    public:
        bool DoRetry(const Controller* c) const override { return c->ErrorCode() == 4242; }
    } policy;
    Fixture f;
    Channel ch;
    ChannelOptions opt;
    opt.max_retry = 3;
    opt.retry_policy = &policy;
    ASSERT_EQ(ch.Init(f.addr().c_str(), &opt), 0);
    example::EchoRequest fail;
    fail.set_server_fail(true);
    fail.set_code(4242);
    Controller c;
    example::EchoResponse r;
    EXPECT_FALSE(Call(&ch, &c, "x", &r, &fail));
    EXPECT_EQ(c.retried_count(), 3);
    EXPECT_EQ(f.echo.calls.load(), 4);
    Controller c2;  // per-call max_retry wins over the channel's
    c2.set_max_retry(1);
    EXPECT_FALSE(Call(&ch, &c2, "x", &r, &fail));
    EXPECT_EQ(c2.retried_count(), 1);
}

TEST(RpcFeatures, cancel_ends_a_pending_call) {
    Fixture f;
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 10000;
    ASSERT_EQ(ch.Init(f.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    Controller c;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("slow");
    req.set_sleep_us(2000000);
    std::atomic<bool> done{false};
    stub.Echo(&c, &req, &res, NewCallback([&done] { done = true; }));
    usleep(20000);
    const int64_t t0 = monotonic_us();
    c.StartCancel();
    c.Join();
    EXPECT_LT(monotonic_us() - t0, 500000);
    EXPECT_TRUE(c.Failed());
    EXPECT_EQ(c.ErrorCode(), ECANCELED);
    for (int i = 0; i < 200 && !done; ++i) usleep(1000);
    EXPECT_TRUE(done.load());
}

TEST(RpcFeatures, request_and_response_compression) {
    Fixture f;
    Channel ch;
    ASSERT_EQ(ch.Init(f.addr().c_str(), nullptr), 0);
    const std::string big(100000, 'c');
    for (int t : {COMPRESS_TYPE_SNAPPY, COMPRESS_TYPE_GZIP, COMPRESS_TYPE_ZLIB}) {
        Controller c;
        c.set_request_compress_type((CompressType)t);
        example::EchoRequest req;
        req.set_code(t);  // the server answers with the same codec
        example::EchoResponse r;
        ASSERT_TRUE(Call(&ch, &c, big, &r, &req));
        EXPECT_EQ(r.message(), big);
        EXPECT_EQ(f.echo.last_req_compress, t);
        EXPECT_EQ((int)c.response_compress_type(), t);
    }
}

TEST(RpcFeatures, authentication_accepts_and_rejects) {
    TokenAuth server_auth("unused");
    ServerOptions so;
    so.auth = &server_auth;
    Fixture f(so);
    TokenAuth good("secret"), bad("wrong");
    Channel ok_ch, bad_ch, none_ch;
    ChannelOptions o1, o2;
    o1.auth = &good;
    o2.auth = &bad;
    o2.max_retry = 0;
    ASSERT_EQ(ok_ch.Init(f.addr().c_str(), &o1), 0);
    ASSERT_EQ(bad_ch.Init(f.addr().c_str(), &o2), 0);
    ChannelOptions o3;
    o3.max_retry = 0;
    ASSERT_EQ(none_ch.Init(f.addr().c_str(), &o3), 0);
    for (int i = 0; i < 5; ++i) {  // every call on the authenticated connection
        Controller c;
        example::EchoResponse r;
        EXPECT_TRUE(Call(&ok_ch, &c, "in", &r));
    }
    Controller c2, c3;
    example::EchoResponse r2, r3;
    EXPECT_FALSE(Call(&bad_ch, &c2, "out", &r2));
    EXPECT_FALSE(Call(&none_ch, &c3, "out", &r3));
    EXPECT_EQ(f.echo.calls.load(), 5);
}

TEST(RpcFeatures, connection_types_single_pooled_short) {
    Fixture f;
    for (const char* type : {"single", "pooled", "short"}) {
        Channel ch;
        ChannelOptions opt;
        opt.connection_type = type;
        ASSERT_EQ(ch.Init(f.addr().c_str(), &opt), 0);
        std::vector<std::thread> th;
        std::atomic<int> ok{0};
        for (int t = 0; t < 4; ++t) {
            th.emplace_back([&] {
                for (int i = 0; i < 25; ++i) {
                    Controller c;
                    example::EchoResponse r;
                    if (Call(&ch, &c, std::string(type) + std::to_string(i), &r)) ++ok;
                }
            });
        }
        for (auto& t : th) t.join();
        EXPECT_EQ(ok.load(), 100);
    }
    EXPECT_EQ(f.echo.calls.load(), 300);
}

TEST(RpcFeatures, per_method_limit_returns_elimit) {
    Fixture f;
    ASSERT_EQ(f.server.SetMaxConcurrencyOf("example.EchoService.Echo", 1), 0);
    Channel ch;
    ChannelOptions opt;
    opt.max_retry = 0;
    ASSERT_EQ(ch.Init(f.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    const int N = 8;
    std::vector<Controller> cntls(N);
    std::vector<example::EchoRequest> reqs(N);
    std::vector<example::EchoResponse> ress(N);
    for (int i = 0; i < N; ++i) {
        reqs[i].set_message("m");
        reqs[i].set_sleep_us(100000);
        stub.Echo(&cntls[i], &reqs[i], &ress[i], NewCallback([] {}));
    }
    int limited = 0, ok = 0;
    for (int i = 0; i < N; ++i) {
        cntls[i].Join();
        if (!cntls[i].Failed()) ++ok;
        else if (cntls[i].ErrorCode() == ELIMIT) ++limited;
    }
    EXPECT_GE(ok, 1);
    EXPECT_GE(limited, 1);
    EXPECT_EQ(ok + limited, N);
}

TEST(RpcFeatures, stopped_server_fails_calls_cleanly) {
    Fixture* f = new Fixture;
    const std::string addr = f->addr();
    Channel ch;
    ChannelOptions opt;
    opt.max_retry = 0;
    opt.timeout_ms = 2000;
    ASSERT_EQ(ch.Init(addr.c_str(), &opt), 0);
    Controller c1;
    example::EchoResponse r1;
    ASSERT_TRUE(Call(&ch, &c1, "before", &r1));
    f->server.Stop(0);
    f->server.Join();
    delete f;
    Controller c2;
    example::EchoResponse r2;
    const int64_t t0 = monotonic_us();
    EXPECT_FALSE(Call(&ch, &c2, "after", &r2));
    EXPECT_LT(monotonic_us() - t0, 1500000);  // not a timeout: the connection is gone
    EXPECT_NE(c2.ErrorCode(), 0);
}

TEST(RpcFeatures, channel_init_rejects_bad_arguments) {
    Channel a, b, c, d;
    EXPECT_NE(a.Init("not-an-address", nullptr), 0);
    ChannelOptions bad_proto;
    bad_proto.protocol = "no_such_protocol";
    EXPECT_NE(b.Init("127.0.0.1:8000", &bad_proto), 0);
    EXPECT_NE(c.Init("list://127.0.0.1:8000", "no_such_lb", nullptr), 0);
    EXPECT_NE(d.Init("nosuchscheme://x", "rr", nullptr), 0);
}

TEST(RpcFeatures, connect_to_closed_port_fails_fast) {
    // grab a port and close it again
    Fixture* f = new Fixture;
    const std::string addr = f->addr();
    f->server.Stop(0);
    f->server.Join();
    delete f;
    Channel ch;
    ChannelOptions opt;
    opt.max_retry = 0;
    opt.timeout_ms = 3000;
    ASSERT_EQ(ch.Init(addr.c_str(), &opt), 0);
    Controller c;
    example::EchoResponse r;
    const int64_t t0 = monotonic_us();
    EXPECT_FALSE(Call(&ch, &c, "x", &r));
    EXPECT_LT(monotonic_us() - t0, 1000000);
    EXPECT_TRUE(c.ErrorCode() == ECONNREFUSED || c.ErrorCode() == EHOSTDOWN || c.ErrorCode() == EFAILEDSOCKET);
}

TEST(RpcFeatures, large_and_empty_attachments) {
    Fixture f;
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 10000;
    ASSERT_EQ(ch.Init(f.addr().c_str(), &opt), 0);
    for (size_t n : {(size_t)0, (size_t)1, (size_t)65536, (size_t)(8 << 20)}) {
        Controller c;
        std::string att(n, '\0');
        for (size_t i = 0; i < n; ++i) att[i] = (char)(i * 31 + 7);
        c.request_attachment().append(att);
        example::EchoResponse r;
        ASSERT_TRUE(Call(&ch, &c, "att", &r));
        EXPECT_EQ(c.response_attachment().size(), n);
        EXPECT_TRUE(c.response_attachment().equals(att));
    }
}

TEST(RpcFeatures, fiber_callers_share_one_connection) {
    Fixture f;
    Channel ch;
    ASSERT_EQ(ch.Init(f.addr().c_str(), nullptr), 0);
    const int N = 200;
    std::atomic<int> ok{0};
    fiber::CountdownEvent all(N);
    struct Arg {
        Channel* ch;
        std::atomic<int>* ok;
        fiber::CountdownEvent* all;
        int i;
    };
    std::vector<Arg> args(N);
    for (int i = 0; i < N; ++i) {
        args[i] = Arg{&ch, &ok, &all, i};
        fiber::fiber_t tid;
        fiber::start_background(&tid, nullptr, [](void* p) -> void* {
            Arg* a = static_cast<Arg*>(p);
            Controller c;
            example::EchoResponse r;
            if (Call(a->ch, &c, "fiber" + std::to_string(a->i), &r) && r.message() == "fiber" + std::to_string(a->i)) {
                a->ok->fetch_add(1);
            }
            a->all->signal();
            return nullptr;
        }, &args[i]);
    }
    all.wait();
    EXPECT_EQ(ok.load(), N);
}
