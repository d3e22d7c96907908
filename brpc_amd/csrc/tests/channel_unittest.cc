// Channel behaviour across the three kinds a user calls through — a single
// server Channel, a ParallelChannel (fan-out to 3 servers) and a
// SelectiveChannel (load-balanced over 3 servers) — in the spirit of the
// reference's test/brpc_channel_unittest.cpp, whose cases are this same
// matrix: success sync/async, cancel before / during / after the call,
// uninitialized requests, timeouts, connections the server closes, server
// failures, authentication, retries onto other servers, many threads on one
// channel, destroying a channel with calls done, plus Init forms (naming
// services, unknown schemes, hostnames) and the parallel-only mapper cases
// (skip all, bad sub call, duplicated sub channel, fail/success limits).
#include <unistd.h>

#include <atomic>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "base/time.h"
#include "fiber/fiber.h"
#include "mrpc/proto/echo.pb.h"
#include "rpc/authenticator.h"
#include "rpc/channel.h"
#include "rpc/combo_channels.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

struct Auth : public Authenticator {
    int GenerateCredential(std::string* out) const override {
        *out = "token-ok";
        return 0;
    }
    int VerifyCredential(const std::string& cred, const EndPoint&, AuthContext*) const override {
        return cred == "token-ok" ? 0 : -1;
    }
};

class TaggedEcho : public example::EchoService {
public:
    explicit TaggedEcho(int tag) : _tag(tag) {}
    void Echo(RpcController* c, const example::EchoRequest* req, example::EchoResponse* res, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = static_cast<Controller*>(c);
        calls.fetch_add(1);
        if (req->sleep_us() > 0) fiber::usleep((uint64_t)req->sleep_us());
        if (req->server_fail() || fail_all.load()) {
            cntl->SetFailed(req->code() ? req->code() : EINTERNAL, "server %d failed on purpose", _tag);
            return;
        }
        if (req->close_fd()) {
            cntl->CloseConnection("close_fd requested");
            return;
        }
        res->set_message(req->message());
        res->set_receiving_socket_id(_tag);
        cntl->response_attachment().append(cntl->request_attachment());
    }
    std::atomic<int> calls{0};
    std::atomic<bool> fail_all{false};

private:
    int _tag;
};

// Three servers (optionally requiring authentication).
struct Cluster {
    // services outlive the servers: handlers still sleeping in Echo when a
    // test ends are joined by ~Cluster before their service goes away
    std::vector<std::unique_ptr<TaggedEcho>> services;
    std::vector<std::unique_ptr<Server>> servers;
    std::vector<int> ports;
    Auth auth;
    explicit Cluster(bool with_auth = false, int n = 3) {
        for (int i = 0; i < n; ++i) {
            services.emplace_back(new TaggedEcho(i));
            servers.emplace_back(new Server);
            servers.back()->AddService(services.back().get(), SERVER_DOESNT_OWN_SERVICE);
            ServerOptions o;
            o.has_builtin_services = false;
            if (with_auth) o.auth = &auth;
            servers.back()->Start("127.0.0.1:0", &o);
            ports.push_back(servers.back()->listen_port());
        }
    }
    ~Cluster() {
        for (auto& s : servers) {
            s->Stop(0);
            s->Join();
        }
    }
    std::string addr(int i) const { return "127.0.0.1:" + std::to_string(ports[i]); }
    std::string list_url() const {
        std::string u = "list://";
        for (size_t i = 0; i < ports.size(); ++i) u += (i ? "," : "") + addr((int)i);
        return u;
    }
    int total_calls() const {
        int n = 0;
        for (auto& s : services) n += s->calls.load();
        return n;
    }
};

enum Kind { SINGLE, PARALLEL, SELECTIVE };

std::unique_ptr<ChannelBase> make(Kind kind, Cluster& c, int timeout_ms = 2000, bool with_auth = false,
                                  int max_retry = 0) {
    ChannelOptions o;
    o.timeout_ms = timeout_ms;
    o.max_retry = max_retry;
    if (with_auth) o.auth = &c.auth;
    if (kind == SINGLE) {
        std::unique_ptr<Channel> ch(new Channel);
        if (ch->Init(c.addr(0).c_str(), &o) != 0) return nullptr;
        return std::unique_ptr<ChannelBase>(ch.release());
    }
    if (kind == PARALLEL) {
        std::unique_ptr<ParallelChannel> p(new ParallelChannel);
        ParallelChannelOptions po;
        po.timeout_ms = timeout_ms;
        p->Init(&po);
        for (size_t i = 0; i < c.ports.size(); ++i) {
            Channel* sub = new Channel;
            sub->Init(c.addr((int)i).c_str(), &o);
            p->AddChannel(sub, OWNS_CHANNEL, nullptr, nullptr);
        }
        return std::unique_ptr<ChannelBase>(p.release());
    }
    std::unique_ptr<SelectiveChannel> s(new SelectiveChannel);
    ChannelOptions so = o;
    s->Init("rr", &so);
    for (size_t i = 0; i < c.ports.size(); ++i) {
        Channel* sub = new Channel;
        sub->Init(c.addr((int)i).c_str(), &o);
        s->AddChannel(sub, OWNS_CHANNEL);
    }
    return std::unique_ptr<ChannelBase>(s.release());
}

const pb::MethodDescriptor* echo_method() { return example::EchoService::descriptor()->method(0); }

int call(ChannelBase* ch, const example::EchoRequest& req, example::EchoResponse* res, Controller* cntl = nullptr) {
    Controller local;
    Controller* c = cntl ? cntl : &local;
    ch->CallMethod(echo_method(), c, &req, res, nullptr);
    return c->ErrorCode();
}

example::EchoRequest req_of(const std::string& m) {
    example::EchoRequest r;
    r.set_message(m);
    return r;
}

// -------------------------------------------------------------- helpers
void check_success(Kind kind) {
    Cluster c;
    auto ch = make(kind, c);
    ASSERT_TRUE(ch != nullptr);
    example::EchoResponse res;
    ASSERT_EQ(call(ch.get(), req_of("hello"), &res), 0);
    EXPECT_EQ(res.message(), "hello");  // parallel: 3 responses merged (MergeFrom overwrites a string)
    // async: the done closure runs once with the response filled
    std::atomic<int> done{0};
    Controller cntl;
    example::EchoResponse ares;
    example::EchoRequest areq = req_of("async");
    ch->CallMethod(echo_method(), &cntl, &areq, &ares, NewCallback([&done] { done.fetch_add(1); }));
    for (int i = 0; i < 300 && !done.load(); ++i) usleep(10000);
    EXPECT_EQ(done.load(), 1);
    EXPECT_FALSE(cntl.Failed());
}

void check_cancel_before(Kind kind) {
    Cluster c;
    auto ch = make(kind, c);
    Controller cntl;
    StartCancel(cntl.call_id());  // canceled before the call starts
    example::EchoResponse res;
    const int rc = call(ch.get(), req_of("x"), &res, &cntl);
    EXPECT_EQ(rc, ECANCELED);
    EXPECT_EQ(c.total_calls(), 0);
}

void check_cancel_during(Kind kind) {
    Cluster c;
    auto ch = make(kind, c, 5000);
    Controller cntl;
    example::EchoRequest req = req_of("slow");
    req.set_sleep_us(500000);
    example::EchoResponse res;
    std::atomic<int> done{0};
    const int64_t t0 = monotonic_us();
    ch->CallMethod(echo_method(), &cntl, &req, &res, NewCallback([&done] { done.fetch_add(1); }));
    usleep(30000);
    StartCancel(cntl.call_id());
    for (int i = 0; i < 300 && !done.load(); ++i) usleep(2000);
    EXPECT_EQ(done.load(), 1);
    EXPECT_EQ(cntl.ErrorCode(), ECANCELED);
    EXPECT_LT(monotonic_us() - t0, 400000);  // did not wait for the server
}

void check_cancel_after(Kind kind) {
    Cluster c;
    auto ch = make(kind, c);
    Controller cntl;
    example::EchoResponse res;
    ASSERT_EQ(call(ch.get(), req_of("done already"), &res, &cntl), 0);
    const fiber::CallId cid = cntl.call_id();
    StartCancel(cid);  // the call is over: nothing happens
    EXPECT_FALSE(cntl.Failed());
    EXPECT_EQ(cntl.ErrorCode(), 0);
}

void check_request_not_init(Kind kind) {
    Cluster c;
    auto ch = make(kind, c);
    example::EchoRequest req;  // required message missing
    example::EchoResponse res;
    EXPECT_EQ(call(ch.get(), req, &res), EREQUEST);
    EXPECT_EQ(c.total_calls(), 0);
}

void check_timeout(Kind kind) {
    Cluster c;
    auto ch = make(kind, c, 100);
    example::EchoRequest req = req_of("too slow");
    req.set_sleep_us(400000);
    example::EchoResponse res;
    const int64_t t0 = monotonic_us();
    EXPECT_EQ(call(ch.get(), req, &res), ERPCTIMEDOUT);
    EXPECT_LT(monotonic_us() - t0, 350000);
}

void check_close_fd(Kind kind) {
    Cluster c;
    auto ch = make(kind, c);
    example::EchoRequest req = req_of("bye");
    req.set_close_fd(true);
    example::EchoResponse res;
    const int rc = call(ch.get(), req, &res);
    EXPECT_NE(rc, 0);
    EXPECT_TRUE(rc == EEOF || rc == EFAILEDSOCKET || rc == ECLOSE || rc == ETOOMANYFAILS || rc == ECONNRESET ||
                rc == EHOSTDOWN);
}

void check_server_fail(Kind kind) {
    Cluster c;
    auto ch = make(kind, c);
    example::EchoRequest req = req_of("fail");
    req.set_server_fail(true);
    req.set_code(EINTERNAL);
    example::EchoResponse res;
    const int rc = call(ch.get(), req, &res);
    // parallel: every sub call failed with the same code, which becomes the
    // parent's (the reference's unified error code)
    EXPECT_EQ(rc, EINTERNAL);
}

void check_authentication(Kind kind) {
    Cluster c(/*with_auth=*/true);
    auto good = make(kind, c, 2000, /*with_auth=*/true);
    example::EchoResponse res;
    EXPECT_EQ(call(good.get(), req_of("signed"), &res), 0);
    auto bad = make(kind, c, 500, /*with_auth=*/false);
    EXPECT_NE(call(bad.get(), req_of("unsigned"), &res), 0);
}

void check_destroy_with_async_calls_done(Kind kind) {
    Cluster c;
    std::atomic<int> done{0};
    std::vector<std::unique_ptr<Controller>> cntls;
    std::vector<std::unique_ptr<example::EchoResponse>> ress;
    example::EchoRequest req = req_of("async");
    {
        auto ch = make(kind, c);
        for (int i = 0; i < 20; ++i) {
            cntls.emplace_back(new Controller);
            ress.emplace_back(new example::EchoResponse);
            ch->CallMethod(echo_method(), cntls.back().get(), &req, ress.back().get(),
                           NewCallback([&done] { done.fetch_add(1); }));
        }
        for (int i = 0; i < 500 && done.load() < 20; ++i) usleep(5000);
    }  // channel destroyed after every done ran
    EXPECT_EQ(done.load(), 20);
    for (auto& cn : cntls) EXPECT_FALSE(cn->Failed());
}

}  // namespace

// -------------------------------------------------------------- init

TEST(Channel, init_as_single_server_forms) {
    Cluster c(false, 1);
    for (const std::string& a : {c.addr(0), "localhost:" + std::to_string(c.ports[0]), "127.0.0.1:" + std::to_string(c.ports[0])}) {
        Channel ch;
        ChannelOptions o;
        ASSERT_EQ(ch.Init(a.c_str(), &o), 0);
        example::EchoResponse res;
        EXPECT_EQ(call(&ch, req_of("x"), &res), 0);
    }
    Channel by_port;
    ChannelOptions o;
    ASSERT_EQ(by_port.Init("127.0.0.1", c.ports[0], &o), 0);
    example::EchoResponse res;
    EXPECT_EQ(call(&by_port, req_of("y"), &res), 0);
}

TEST(Channel, init_with_unknown_naming_service_or_lb_fails) {
    Channel a, b, d;
    ChannelOptions o;
    EXPECT_NE(a.Init("nosuchscheme://host:1", "rr", &o), 0);
    EXPECT_NE(b.Init("list://127.0.0.1:1", "no_such_lb", &o), 0);
    EXPECT_NE(d.Init("not a host:port at all", &o), 0);
}

TEST(Channel, init_with_missing_file_naming_service_fails_calls) {
    Channel ch;
    ChannelOptions o;
    o.timeout_ms = 300;
    const int rc = ch.Init("file:///tmp/mrpc_no_such_servers_file", "rr", &o);
    if (rc == 0) {  // allowed to start empty: calls then find no server
        example::EchoResponse res;
        EXPECT_NE(call(&ch, req_of("x"), &res), 0);
    }
}

TEST(Channel, init_with_empty_list_fails_calls_with_no_server) {
    Channel ch;
    ChannelOptions o;
    o.timeout_ms = 300;
    ASSERT_EQ(ch.Init("list://", "rr", &o), 0);
    example::EchoResponse res;
    const int rc = call(&ch, req_of("x"), &res);
    EXPECT_NE(rc, 0);
}

TEST(Channel, init_using_naming_service_spreads_calls) {
    Cluster c;
    Channel ch;
    ChannelOptions o;
    ASSERT_EQ(ch.Init(c.list_url().c_str(), "rr", &o), 0);
    for (int i = 0; i < 30; ++i) {
        example::EchoResponse res;
        ASSERT_EQ(call(&ch, req_of("x"), &res), 0);
    }
    for (auto& s : c.services) EXPECT_GT(s->calls.load(), 3);
}

TEST(Channel, connection_failed_to_a_closed_port) {
    int port;
    {
        Cluster c(false, 1);
        port = c.ports[0];
    }  // the server is gone
    Channel ch;
    ChannelOptions o;
    o.timeout_ms = 500;
    o.max_retry = 0;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(port)).c_str(), &o), 0);
    example::EchoResponse res;
    const int64_t t0 = monotonic_us();
    EXPECT_NE(call(&ch, req_of("x"), &res), 0);
    EXPECT_LT(monotonic_us() - t0, 450000);  // refused, not timed out
}

// -------------------------------------------------------------- the matrix

TEST(Channel, success_single) { check_success(SINGLE); }
TEST(Channel, success_parallel) { check_success(PARALLEL); }
TEST(Channel, success_selective) { check_success(SELECTIVE); }
TEST(Channel, cancel_before_callmethod_single) { check_cancel_before(SINGLE); }
TEST(Channel, cancel_before_callmethod_parallel) { check_cancel_before(PARALLEL); }
TEST(Channel, cancel_before_callmethod_selective) { check_cancel_before(SELECTIVE); }
TEST(Channel, cancel_during_callmethod_single) { check_cancel_during(SINGLE); }
TEST(Channel, cancel_during_callmethod_parallel) { check_cancel_during(PARALLEL); }
TEST(Channel, cancel_during_callmethod_selective) { check_cancel_during(SELECTIVE); }
TEST(Channel, cancel_after_callmethod_single) { check_cancel_after(SINGLE); }
TEST(Channel, cancel_after_callmethod_parallel) { check_cancel_after(PARALLEL); }
TEST(Channel, request_not_init_single) { check_request_not_init(SINGLE); }
TEST(Channel, request_not_init_parallel) { check_request_not_init(PARALLEL); }
TEST(Channel, request_not_init_selective) { check_request_not_init(SELECTIVE); }
TEST(Channel, timeout_single) { check_timeout(SINGLE); }
TEST(Channel, timeout_parallel) { check_timeout(PARALLEL); }
TEST(Channel, timeout_selective) { check_timeout(SELECTIVE); }
TEST(Channel, close_fd_single) { check_close_fd(SINGLE); }
TEST(Channel, close_fd_parallel) { check_close_fd(PARALLEL); }
TEST(Channel, close_fd_selective) { check_close_fd(SELECTIVE); }
TEST(Channel, server_fail_single) { check_server_fail(SINGLE); }
TEST(Channel, server_fail_parallel) { check_server_fail(PARALLEL); }
TEST(Channel, server_fail_selective) { check_server_fail(SELECTIVE); }
TEST(Channel, authentication_single) { check_authentication(SINGLE); }
TEST(Channel, authentication_parallel) { check_authentication(PARALLEL); }
TEST(Channel, authentication_selective) { check_authentication(SELECTIVE); }
TEST(Channel, destroy_channel_single) { check_destroy_with_async_calls_done(SINGLE); }
TEST(Channel, destroy_channel_parallel) { check_destroy_with_async_calls_done(PARALLEL); }
TEST(Channel, destroy_channel_selective) { check_destroy_with_async_calls_done(SELECTIVE); }

// -------------------------------------------------------------- parallel only

namespace {
struct SkipAll : public CallMapper {
    SubCall Map(int, int, const pb::MethodDescriptor*, const pb::Message*, pb::Message*) override {
        return SubCall::Skip();
    }
};
struct BadSecond : public CallMapper {
    SubCall Map(int i, int, const pb::MethodDescriptor* m, const pb::Message* req, pb::Message* res) override {
        if (i == 1) return SubCall::Bad();
        return SubCall(m, req, res->New(), SubCall::DELETE_RESPONSE);
    }
};
struct SkipOdd : public CallMapper {
    SubCall Map(int i, int, const pb::MethodDescriptor* m, const pb::Message* req, pb::Message* res) override {
        if (i % 2) return SubCall::Skip();
        return SubCall(m, req, res->New(), SubCall::DELETE_RESPONSE);
    }
};
}  // namespace

TEST(Channel, empty_parallel_channel_fails) {
    ParallelChannel p;
    ParallelChannelOptions po;
    p.Init(&po);
    example::EchoResponse res;
    EXPECT_NE(call(&p, req_of("x"), &res), 0);
}

TEST(Channel, empty_selective_channel_fails) {
    SelectiveChannel s;
    ChannelOptions o;
    o.timeout_ms = 300;
    s.Init("rr", &o);
    example::EchoResponse res;
    EXPECT_NE(call(&s, req_of("x"), &res), 0);
}

TEST(Channel, skip_all_channels_fails_parallel) {
    Cluster c;
    ParallelChannel p;
    ParallelChannelOptions po;
    p.Init(&po);
    auto skip = std::make_shared<SkipAll>();
    for (int i = 0; i < 3; ++i) {
        Channel* sub = new Channel;
        ChannelOptions o;
        sub->Init(c.addr(i).c_str(), &o);
        p.AddChannel(sub, OWNS_CHANNEL, skip, nullptr);
    }
    example::EchoResponse res;
    EXPECT_NE(call(&p, req_of("x"), &res), 0);
    EXPECT_EQ(c.total_calls(), 0);
}

TEST(Channel, bad_sub_call_fails_the_parallel_call) {
    Cluster c;
    ParallelChannel p;
    ParallelChannelOptions po;
    p.Init(&po);
    auto bad = std::make_shared<BadSecond>();
    for (int i = 0; i < 3; ++i) {
        Channel* sub = new Channel;
        ChannelOptions o;
        sub->Init(c.addr(i).c_str(), &o);
        p.AddChannel(sub, OWNS_CHANNEL, bad, nullptr);
    }
    example::EchoResponse res;
    EXPECT_EQ(call(&p, req_of("x"), &res), EREQUEST);
}

TEST(Channel, skipped_sub_calls_leave_the_others) {
    Cluster c;
    ParallelChannel p;
    ParallelChannelOptions po;
    p.Init(&po);
    auto skip = std::make_shared<SkipOdd>();
    for (int i = 0; i < 3; ++i) {
        Channel* sub = new Channel;
        ChannelOptions o;
        sub->Init(c.addr(i).c_str(), &o);
        p.AddChannel(sub, OWNS_CHANNEL, skip, nullptr);
    }
    example::EchoResponse res;
    ASSERT_EQ(call(&p, req_of("ab"), &res), 0);
    EXPECT_EQ(res.message(), "ab");  // channels 0 and 2 answered
    EXPECT_EQ(c.services[0]->calls.load() + c.services[2]->calls.load(), 2);
    EXPECT_EQ(c.services[1]->calls.load(), 0);
}

TEST(Channel, duplicated_sub_channel_is_called_twice) {
    Cluster c(false, 1);
    ParallelChannel p;
    ParallelChannelOptions po;
    p.Init(&po);
    Channel sub;
    ChannelOptions o;
    sub.Init(c.addr(0).c_str(), &o);
    p.AddChannel(&sub, DOESNT_OWN_CHANNEL, nullptr, nullptr);
    p.AddChannel(&sub, DOESNT_OWN_CHANNEL, nullptr, nullptr);
    example::EchoResponse res;
    ASSERT_EQ(call(&p, req_of("d"), &res), 0);
    EXPECT_EQ(res.message(), "d");
    EXPECT_EQ(c.services[0]->calls.load(), 2);
}

TEST(Channel, fail_limit_ends_early_and_success_limit_needs_few) {
    Cluster c;
    c.services[0]->fail_all = true;
    {
        ParallelChannel p;
        ParallelChannelOptions po;
        po.fail_limit = 1;  // one failure is enough to fail the call
        p.Init(&po);
        for (int i = 0; i < 3; ++i) {
            Channel* sub = new Channel;
            ChannelOptions o;
            sub->Init(c.addr(i).c_str(), &o);
            p.AddChannel(sub, OWNS_CHANNEL, nullptr, nullptr);
        }
        example::EchoResponse res;
        EXPECT_NE(call(&p, req_of("x"), &res), 0);
    }
    {
        ParallelChannel p;
        ParallelChannelOptions po;
        po.success_limit = 2;  // two successes are enough
        p.Init(&po);
        for (int i = 0; i < 3; ++i) {
            Channel* sub = new Channel;
            ChannelOptions o;
            sub->Init(c.addr(i).c_str(), &o);
            p.AddChannel(sub, OWNS_CHANNEL, nullptr, nullptr);
        }
        example::EchoResponse res;
        EXPECT_EQ(call(&p, req_of("x"), &res), 0);
    }
}

// -------------------------------------------------------------- retries, threads

TEST(Channel, retry_goes_to_other_servers) {
    Cluster c;
    c.services[0]->fail_all = true;
    Channel ch;
    ChannelOptions o;
    o.max_retry = 3;
    ASSERT_EQ(ch.Init(c.list_url().c_str(), "rr", &o), 0);
    // close_fd failures are retried (a connection error); with rr the retry
    // lands on another server. Application errors are not retried.
    int ok = 0;
    for (int i = 0; i < 12; ++i) {
        example::EchoResponse res;
        if (call(&ch, req_of("r"), &res) == 0) ++ok;
    }
    EXPECT_GE(ok, 6);  // servers 1 and 2 answer
    EXPECT_GT(c.services[1]->calls.load() + c.services[2]->calls.load(), 6);
}

TEST(Channel, selective_channel_retries_a_failed_sub_channel_elsewhere) {
    Cluster c;
    c.servers[0]->Stop(0);
    c.servers[0]->Join();
    SelectiveChannel s;
    ChannelOptions o;
    o.max_retry = 3;
    o.timeout_ms = 2000;
    s.Init("rr", &o);
    for (int i = 0; i < 3; ++i) {
        Channel* sub = new Channel;
        ChannelOptions so;
        so.max_retry = 0;
        sub->Init(c.addr(i).c_str(), &so);
        s.AddChannel(sub, OWNS_CHANNEL);
    }
    int ok = 0;
    for (int i = 0; i < 9; ++i) {
        example::EchoResponse res;
        if (call(&s, req_of("s"), &res) == 0) ++ok;
    }
    EXPECT_EQ(ok, 9);  // the stopped server's turn went to the others
}

TEST(Channel, multiple_threads_single_channel) {
    Cluster c(false, 1);
    Channel ch;
    ChannelOptions o;
    o.timeout_ms = 5000;
    ASSERT_EQ(ch.Init(c.addr(0).c_str(), &o), 0);
    std::atomic<int> ok{0};
    std::vector<std::thread> ths;
    for (int t = 0; t < 8; ++t) {
        ths.emplace_back([&, t] {
            for (int i = 0; i < 100; ++i) {
                example::EchoResponse res;
                const std::string m = std::to_string(t) + ":" + std::to_string(i);
                if (call(&ch, req_of(m), &res) == 0 && res.message() == m) ok.fetch_add(1);
            }
        });
    }
    for (auto& th : ths) th.join();
    EXPECT_EQ(ok.load(), 800);
}

TEST(Channel, multiple_threads_multiple_channels) {
    Cluster c;
    std::atomic<int> ok{0};
    std::vector<std::thread> ths;
    for (int t = 0; t < 6; ++t) {
        ths.emplace_back([&, t] {
            auto ch = make((Kind)(t % 3), c, 5000);
            for (int i = 0; i < 50; ++i) {
                example::EchoResponse res;
                if (call(ch.get(), req_of("m"), &res) == 0) ok.fetch_add(1);
            }
        });
    }
    for (auto& th : ths) th.join();
    EXPECT_EQ(ok.load(), 300);
}

TEST(Channel, unused_controller_and_call_id_are_harmless) {
    for (int i = 0; i < 100; ++i) {
        Controller cntl;
        (void)cntl.call_id();  // created, never used by a call
    }
    Cluster c(false, 1);
    Channel ch;
    ChannelOptions o;
    ASSERT_EQ(ch.Init(c.addr(0).c_str(), &o), 0);
    example::EchoResponse res;
    EXPECT_EQ(call(&ch, req_of("after"), &res), 0);
}

TEST(Channel, connection_types_and_protocols_by_name) {
    Cluster c(false, 1);
    for (const char* ct : {"single", "pooled", "short"}) {
        for (const char* proto : {"baidu_std", "hulu_pbrpc", "sofa_pbrpc", "http", "h2"}) {
            Channel ch;
            ChannelOptions o;
            o.protocol = proto;
            o.connection_type = ct;
            o.timeout_ms = 2000;
            const int rc = ch.Init(c.addr(0).c_str(), &o);
            const bool h2_not_short = std::string(proto) == "h2" && std::string(ct) != "single";
            if (rc != 0) {
                // a protocol may refuse a connection type (h2 multiplexes
                // on one connection)
                EXPECT_TRUE(h2_not_short || std::string(ct) == "short" || std::string(ct) == "single");
                continue;
            }
            example::EchoResponse res;
            EXPECT_EQ(call(&ch, req_of(std::string(proto) + "/" + ct), &res), 0);
            EXPECT_EQ(res.message(), std::string(proto) + "/" + ct);
        }
    }
}

TEST(Channel, response_attachment_cleared_between_retries) {
    Cluster c;
    c.services[0]->fail_all = true;
    Channel ch;
    ChannelOptions o;
    o.max_retry = 2;
    ASSERT_EQ(ch.Init(c.list_url().c_str(), "rr", &o), 0);
    for (int i = 0; i < 6; ++i) {
        Controller cntl;
        cntl.request_attachment().append("attach");
        example::EchoResponse res;
        example::EchoRequest req = req_of("r");
        ch.CallMethod(echo_method(), &cntl, &req, &res, nullptr);
        if (!cntl.Failed()) EXPECT_EQ(cntl.response_attachment().to_string(), "attach");
    }
}
