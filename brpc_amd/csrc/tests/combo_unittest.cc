// Combo channels: ParallelChannel, PartitionChannel, DynamicPartitionChannel,
// SelectiveChannel (spirit of the reference's
// test/brpc_channel_unittest.cpp parallel/selective/partition cases).
#include <unistd.h>

#include <set>
#include <thread>

#include "base/time.h"
#include "fiber/fiber.h"
#include "mrpc/proto/echo.pb.h"
#include "rpc/channel.h"
#include "rpc/combo_channels.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

class TaggedEcho : public example::EchoService {
public:
    explicit TaggedEcho(std::string tag) : _tag(std::move(tag)) {}
    void Echo(RpcController* c, const example::EchoRequest* req, example::EchoResponse* res, Closure* done) override {
        ClosureGuard g(done);
        if (req->sleep_us() > 0) fiber::usleep(req->sleep_us());
        if (delay_us > 0) fiber::usleep(delay_us);
        if (req->server_fail()) {
            static_cast<Controller*>(c)->SetFailed(EINTERNAL, "asked to fail by %s", _tag.c_str());
            return;
        }
        res->set_message(req->message() + "@" + _tag);
    }

    int64_t delay_us = 0;

private:
    std::string _tag;
};

struct TaggedServer {
    Server server;
    TaggedEcho echo;
    int port = 0;
    explicit TaggedServer(const std::string& tag) : echo(tag) {
        server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        ServerOptions o;
        o.has_builtin_services = false;
        if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
    }
    std::string addr() const { return "127.0.0.1:" + std::to_string(port); }
};

Channel* make_channel(const std::string& addr, int timeout_ms = 2000) {
    Channel* ch = new Channel;
    ChannelOptions o;
    o.timeout_ms = timeout_ms;
    o.max_retry = 0;
    if (ch->Init(addr.c_str(), &o) != 0) {
        delete ch;
        return nullptr;
    }
    return ch;
}

class ConcatMerger : public ResponseMerger {
public:
    Result Merge(pb::Message* response, const pb::Message* sub) override {
        auto* r = static_cast<example::EchoResponse*>(response);
        auto* s = static_cast<const example::EchoResponse*>(sub);
        r->set_message(r->message().empty() ? s->message() : r->message() + "|" + s->message());
        return MERGED;
    }
};

class SplitMapper : public CallMapper {
public:
    SubCall Map(int i, int n, const pb::MethodDescriptor* m, const pb::Message* req, pb::Message* res) override {
        auto* r = new example::EchoRequest(*static_cast<const example::EchoRequest*>(req));
        r->set_message(r->message() + "#" + std::to_string(i) + "/" + std::to_string(n));
        return SubCall(m, r, res->New(), SubCall::DELETE_REQUEST | SubCall::DELETE_RESPONSE);
    }
};

std::set<std::string> split(const std::string& s) {
    std::set<std::string> out;
    size_t b = 0;
    while (true) {
        size_t e = s.find('|', b);
        out.insert(s.substr(b, e == std::string::npos ? std::string::npos : e - b));
        if (e == std::string::npos) break;
        b = e + 1;
    }
    return out;
}

}  // namespace

TEST(ParallelChannel, broadcast_merge_map_and_limits) {
    TaggedServer a("a"), b("b"), c("c");
    ParallelChannel pc;
    ParallelChannelOptions po;
    po.timeout_ms = 2000;
    pc.Init(&po);
    auto merger = std::make_shared<ConcatMerger>();
    auto mapper = std::make_shared<SplitMapper>();
    for (TaggedServer* s : {&a, &b, &c}) pc.AddChannel(make_channel(s->addr()), OWNS_CHANNEL, mapper, merger);
    example::EchoService_Stub stub(&pc);
    for (int i = 0; i < 20; ++i) {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("m");
        stub.Echo(&cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        EXPECT_TRUE(split(res.message()) == (std::set<std::string>{"m#0/3@a", "m#1/3@b", "m#2/3@c"}));
    }
    // async
    {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("x");
        std::atomic<int> fired{0};
        stub.Echo(&cntl, &req, &res, NewCallback([&] { fired.store(1); }));
        cntl.Join();
        // Join() returns once the call id is gone; done may still be running
        for (int spin = 0; spin < 2000 && fired.load() == 0; ++spin) usleep(1000);
        EXPECT_EQ(fired.load(), 1);
        EXPECT_FALSE(cntl.Failed());
        EXPECT_EQ(split(res.message()).size(), 3u);
    }
    // one dead sub channel: default fail_limit tolerates it, fail_limit=1 does not
    ParallelChannel pc2;
    pc2.Init(&po);
    pc2.AddChannel(make_channel(a.addr()), OWNS_CHANNEL, nullptr, merger);
    pc2.AddChannel(make_channel("127.0.0.1:1", 300), OWNS_CHANNEL, nullptr, merger);
    example::EchoService_Stub stub2(&pc2);
    {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("y");
        stub2.Echo(&cntl, &req, &res, nullptr);
        EXPECT_FALSE(cntl.Failed());
        EXPECT_EQ(res.message(), "y@a");
    }
    ParallelChannelOptions strict = po;
    strict.fail_limit = 1;
    ParallelChannel pc3;
    pc3.Init(&strict);
    pc3.AddChannel(make_channel(a.addr()), OWNS_CHANNEL, nullptr, merger);
    pc3.AddChannel(make_channel("127.0.0.1:1", 300), OWNS_CHANNEL, nullptr, merger);
    example::EchoService_Stub stub3(&pc3);
    {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("z");
        stub3.Echo(&cntl, &req, &res, nullptr);
        EXPECT_TRUE(cntl.Failed());
    }
    // success_limit=1 returns on the first answer
    ParallelChannelOptions first = po;
    first.success_limit = 1;
    ParallelChannel pc4;
    pc4.Init(&first);
    pc4.AddChannel(make_channel(a.addr()), OWNS_CHANNEL, nullptr, merger);
    pc4.AddChannel(make_channel(b.addr()), OWNS_CHANNEL, nullptr, merger);
    example::EchoService_Stub stub4(&pc4);
    {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("f");
        stub4.Echo(&cntl, &req, &res, nullptr);
        EXPECT_FALSE(cntl.Failed());
        EXPECT_EQ(split(res.message()).size(), 1u);
    }
}

TEST(PartitionChannel, static_and_dynamic) {
    TaggedServer p0("p0"), p1("p1"), p2("p2"), q0("q0"), q1("q1");
    auto merger = std::make_shared<ConcatMerger>();
    PartitionParser parser;
    PartitionChannelOptions opt;
    opt.timeout_ms = 2000;
    opt.response_merger = merger;
    const std::string url = "list://" + p0.addr() + " 0/3," + p1.addr() + " 1/3," + p2.addr() + " 2/3," +
                            q0.addr() + " 0/2," + q1.addr() + " 1/2";
    PartitionChannel pch;
    ASSERT_EQ(pch.Init(3, &parser, url.c_str(), "rr", &opt), 0);
    EXPECT_EQ(pch.partition_count(), 3);
    example::EchoService_Stub stub(&pch);
    {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("k");
        stub.Echo(&cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        EXPECT_TRUE(split(res.message()) == (std::set<std::string>{"k@p0", "k@p1", "k@p2"}));
    }
    DynamicPartitionChannel dch;
    ASSERT_EQ(dch.Init(&parser, url.c_str(), "rr", &opt), 0);
    EXPECT_EQ(dch.scheme_count(), 2);
    example::EchoService_Stub dstub(&dch);
    int saw3 = 0, saw2 = 0;
    for (int i = 0; i < 60; ++i) {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("d");
        dstub.Echo(&cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        const size_t parts = split(res.message()).size();
        saw3 += parts == 3;
        saw2 += parts == 2;
    }
    EXPECT_GT(saw3, 0);
    EXPECT_GT(saw2, 0);
}

TEST(SelectiveChannel, failover_balance_backup) {
    TaggedServer a("a"), b("b");
    SelectiveChannel sc;
    SelectiveChannelOptions so;
    so.timeout_ms = 2000;
    so.max_retry = 2;
    sc.Init(&so);
    sc.AddChannel(make_channel(a.addr()));
    sc.AddChannel(make_channel("127.0.0.1:1", 300));
    sc.AddChannel(make_channel(b.addr()));
    example::EchoService_Stub stub(&sc);
    std::set<std::string> seen;
    for (int i = 0; i < 30; ++i) {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("s");
        stub.Echo(&cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        seen.insert(res.message());
    }
    EXPECT_TRUE(seen == (std::set<std::string>{"s@a", "s@b"}));
    // application errors are not retried
    {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("e");
        req.set_server_fail(true);
        stub.Echo(&cntl, &req, &res, nullptr);
        EXPECT_TRUE(cntl.Failed());
    }
    // backup request: a slow first choice is overtaken by the backup
    TaggedServer slow("slow"), fast("fast");
    SelectiveChannel bc;
    SelectiveChannelOptions bo;
    bo.timeout_ms = 3000;
    bo.backup_request_ms = 20;
    bc.Init(&bo);
    bc.AddChannel(make_channel(slow.addr(), 3000));
    bc.AddChannel(make_channel(fast.addr(), 3000));
    example::EchoService_Stub bstub(&bc);
    slow.echo.delay_us = 300000;
    int fast_wins = 0;
    for (int i = 0; i < 4; ++i) {
        Controller c2;
        example::EchoResponse r2;
        example::EchoRequest q2;
        q2.set_message("b");
        const int64_t t0 = monotonic_us();
        bstub.Echo(&c2, &q2, &r2, nullptr);
        ASSERT_FALSE(c2.Failed());
        EXPECT_LT(monotonic_us() - t0, 250000);  // never waits for the slow replica
        fast_wins += r2.message() == "b@fast";
    }
    EXPECT_EQ(fast_wins, 4);
}

// TP analog: the attachment is scattered in slices, echoed, gathered back.
TEST(ParallelChannel, scatter_attachment_slices_and_gather) {
    struct EchoNode {
        Server server;
        EchoServiceImpl echo;
        int port = 0;
        EchoNode() {
            server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
            ServerOptions o;
            o.has_builtin_services = false;
            if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
        }
    };
    EchoNode n[3];
    ParallelChannel pc;
    ParallelChannelOptions po;
    po.timeout_ms = 3000;
    po.gather_response_attachments = true;
    pc.Init(&po);
    auto mapper = std::make_shared<ScatterAttachmentMapper>();
    for (auto& x : n) pc.AddChannel(make_channel("127.0.0.1:" + std::to_string(x.port)), OWNS_CHANNEL, mapper, nullptr);
    example::EchoService_Stub stub(&pc);
    for (size_t len : {(size_t)0, (size_t)2, (size_t)10007, (size_t)(1 << 20)}) {
        std::string att(len, '\0');
        for (size_t i = 0; i < len; ++i) att[i] = (char)(i * 13 + len);
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("tp");
        cntl.request_attachment().append(att);
        stub.Echo(&cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        EXPECT_EQ(res.message(), "tp");
        EXPECT_EQ(cntl.response_attachment().size(), len);
        EXPECT_TRUE(cntl.response_attachment().equals(att));  // slices back in channel order
    }
    EXPECT_EQ(n[0].echo.ncalls(), 4);
    EXPECT_EQ(n[2].echo.ncalls(), 4);
    // without the opt-in the parent's response attachment stays untouched,
    // as in the reference (parallel_channel.cpp:683-684)
    {
        ParallelChannel plain;
        ParallelChannelOptions pp;
        pp.timeout_ms = 3000;
        plain.Init(&pp);
        for (auto& x : n) plain.AddChannel(make_channel("127.0.0.1:" + std::to_string(x.port)), OWNS_CHANNEL, mapper, nullptr);
        example::EchoService_Stub s2(&plain);
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("tp");
        cntl.request_attachment().append(std::string(999, 'q'));
        s2.Echo(&cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        EXPECT_EQ(cntl.response_attachment().size(), 0u);
    }
    // slice boundaries: near-equal, contiguous, covering everything
    ScatterAttachmentMapper m;
    Buf whole;
    whole.append(std::string(10, 'a') + std::string(10, 'b') + std::string(11, 'c'));
    size_t covered = 0;
    for (int i = 0; i < 3; ++i) {
        Buf part;
        m.MapAttachment(i, 3, whole, &part);
        EXPECT_TRUE(part.size() == 10 || part.size() == 11);
        covered += part.size();
    }
    EXPECT_EQ(covered, whole.size());
}

// ------------------------------------------------------------ more ParallelChannel semantics
// (reference test/brpc_channel_unittest.cpp: skip/bad sub calls, merger
// verdicts, success_limit, parent timeout, health)

namespace {

class OddSkipMapper : public CallMapper {
public:
    bool all = false, bad = false;
    SubCall Map(int i, int n, const pb::MethodDescriptor* m, const pb::Message* req, pb::Message* res) override {
        if (bad && i == 1) return SubCall::Bad();
        if (all || i % 2 == 1) return SubCall::Skip();
        return SubCall(m, req, res->New(), SubCall::DELETE_RESPONSE);
    }
};

class VerdictMerger : public ResponseMerger {
public:
    explicit VerdictMerger(Result r) : _r(r) {}
    Result Merge(pb::Message* response, const pb::Message* sub) override {
        if (_r == MERGED) response->MergeFrom(*sub);
        return _r;
    }

private:
    Result _r;
};

int call(ChannelBase* ch, const std::string& msg, std::string* out, int64_t sleep_us = 0, int timeout_ms = -1,
         int64_t* elapsed_us = nullptr) {
    example::EchoService_Stub stub(ch);
    Controller cntl;
    if (timeout_ms > 0) cntl.set_timeout_ms(timeout_ms);
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message(msg);
    if (sleep_us) req.set_sleep_us(sleep_us);
    const int64_t t0 = monotonic_us();
    stub.Echo(&cntl, &req, &res, nullptr);
    if (elapsed_us) *elapsed_us = monotonic_us() - t0;
    if (out) *out = res.message();
    return cntl.Failed() ? cntl.ErrorCode() : 0;
}

}  // namespace

TEST(ParallelChannel, skipped_and_bad_sub_calls) {
    TaggedServer a("a"), b("b"), c("c"), d("d");
    ParallelChannelOptions po;
    po.timeout_ms = 2000;
    ParallelChannel pc;
    pc.Init(&po);
    auto mapper = std::make_shared<OddSkipMapper>();
    auto merger = std::make_shared<ConcatMerger>();
    for (TaggedServer* s : {&a, &b, &c, &d}) pc.AddChannel(make_channel(s->addr()), OWNS_CHANNEL, mapper, merger);
    std::string out;
    ASSERT_EQ(call(&pc, "k", &out), 0);
    EXPECT_TRUE(split(out) == (std::set<std::string>{"k@a", "k@c"}));  // odd sub calls skipped
    mapper->all = true;
    EXPECT_EQ(call(&pc, "k", &out), EREQUEST);  // nothing left to call
    mapper->all = false;
    mapper->bad = true;
    EXPECT_EQ(call(&pc, "k", &out), EREQUEST);  // one Bad() fails the whole call before any I/O
}

TEST(ParallelChannel, merger_verdicts) {
    TaggedServer a("a"), b("b"), c("c");
    ParallelChannelOptions po;
    po.timeout_ms = 2000;
    {
        // one FAIL is one failed sub call: tolerated by the default limit
        ParallelChannel pc;
        pc.Init(&po);
        pc.AddChannel(make_channel(a.addr()), OWNS_CHANNEL, nullptr, std::make_shared<ConcatMerger>());
        pc.AddChannel(make_channel(b.addr()), OWNS_CHANNEL, nullptr,
                      std::make_shared<VerdictMerger>(ResponseMerger::FAIL));
        pc.AddChannel(make_channel(c.addr()), OWNS_CHANNEL, nullptr, std::make_shared<ConcatMerger>());
        std::string out;
        EXPECT_EQ(call(&pc, "v", &out), 0);
        EXPECT_TRUE(split(out) == (std::set<std::string>{"v@a", "v@c"}));
    }
    {
        ParallelChannelOptions strict = po;
        strict.fail_limit = 1;
        ParallelChannel pc;
        pc.Init(&strict);
        pc.AddChannel(make_channel(a.addr()), OWNS_CHANNEL, nullptr, std::make_shared<ConcatMerger>());
        pc.AddChannel(make_channel(b.addr()), OWNS_CHANNEL, nullptr,
                      std::make_shared<VerdictMerger>(ResponseMerger::FAIL));
        // the merger failed sub call 1 with ERESPONSE: the only failure, so
        // the unified code is ERESPONSE (ETOOMANYFAILS only when codes differ)
        EXPECT_EQ(call(&pc, "v", nullptr), ERESPONSE);
    }
    {
        ParallelChannel pc;
        pc.Init(&po);
        pc.AddChannel(make_channel(a.addr()), OWNS_CHANNEL, nullptr,
                      std::make_shared<VerdictMerger>(ResponseMerger::FAIL_ALL));
        pc.AddChannel(make_channel(b.addr()), OWNS_CHANNEL, nullptr, std::make_shared<ConcatMerger>());
        EXPECT_EQ(call(&pc, "v", nullptr), ERESPONSE);
    }
}

TEST(ParallelChannel, success_limit_returns_without_the_slow_sub_call) {
    TaggedServer fast("fast"), slow("slow");
    slow.echo.delay_us = 400000;
    ParallelChannelOptions po;
    po.timeout_ms = 3000;
    po.success_limit = 1;
    ParallelChannel pc;
    pc.Init(&po);
    pc.AddChannel(make_channel(fast.addr()), OWNS_CHANNEL, nullptr, std::make_shared<ConcatMerger>());
    pc.AddChannel(make_channel(slow.addr()), OWNS_CHANNEL, nullptr, std::make_shared<ConcatMerger>());
    std::string out;
    int64_t us = 0;
    ASSERT_EQ(call(&pc, "s", &out, 0, -1, &us), 0);
    EXPECT_EQ(out, "s@fast");
    EXPECT_LT(us, 300000);
    // without the limit the parent waits for both
    ParallelChannelOptions all = po;
    all.success_limit = -1;
    ParallelChannel pc2;
    pc2.Init(&all);
    pc2.AddChannel(make_channel(fast.addr()), OWNS_CHANNEL, nullptr, std::make_shared<ConcatMerger>());
    pc2.AddChannel(make_channel(slow.addr()), OWNS_CHANNEL, nullptr, std::make_shared<ConcatMerger>());
    ASSERT_EQ(call(&pc2, "s", &out, 0, -1, &us), 0);
    EXPECT_TRUE(split(out) == (std::set<std::string>{"s@fast", "s@slow"}));
    EXPECT_GE(us, 350000);
}

TEST(ParallelChannel, parent_timeout_cancels_sub_calls_and_health) {
    TaggedServer a("a"), b("b");
    ParallelChannelOptions po;
    po.timeout_ms = 5000;
    ParallelChannel pc;
    pc.Init(&po);
    pc.AddChannel(make_channel(a.addr(), 5000), OWNS_CHANNEL, nullptr, std::make_shared<ConcatMerger>());
    pc.AddChannel(make_channel(b.addr(), 5000), OWNS_CHANNEL, nullptr, std::make_shared<ConcatMerger>());
    int64_t us = 0;
    // the servers sleep 1 s; the parent's 150 ms deadline ends the call
    EXPECT_NE(call(&pc, "t", nullptr, 1000000, 150, &us), 0);
    EXPECT_LT(us, 800000);
    EXPECT_EQ(pc.CheckHealth(), 0);
    EXPECT_EQ(pc.channel_count(), 2);
    // a dead sub channel: healthy while fail_limit tolerates it
    ParallelChannelOptions lim = po;
    lim.fail_limit = 1;
    ParallelChannel pc2;
    pc2.Init(&lim);
    pc2.AddChannel(make_channel(a.addr()), OWNS_CHANNEL, nullptr, nullptr);
    pc2.AddChannel(make_channel("127.0.0.1:1", 200), OWNS_CHANNEL, nullptr, nullptr);
    EXPECT_NE(call(&pc2, "h", nullptr), 0);  // the dead one fails the call (fail_limit 1)
    ParallelChannel empty;
    EXPECT_EQ(empty.CheckHealth(), -1);
}

TEST(SelectiveChannel, remove_channel_moves_traffic) {
    TaggedServer a("a"), b("b");
    SelectiveChannelOptions so;
    so.timeout_ms = 2000;
    SelectiveChannel sc;
    ASSERT_EQ(sc.Init(&so), 0);
    const int ha = sc.AddChannel(make_channel(a.addr()));
    const int hb = sc.AddChannel(make_channel(b.addr()));
    ASSERT_GE(ha, 0);
    ASSERT_GE(hb, 0);
    std::set<std::string> seen;
    std::string out;
    for (int i = 0; i < 40; ++i) {
        ASSERT_EQ(call(&sc, "r", &out), 0);
        seen.insert(out);
    }
    EXPECT_EQ(seen.size(), 2u);  // balanced over both
    sc.RemoveAndDestroyChannel(ha);
    seen.clear();
    for (int i = 0; i < 20; ++i) {
        ASSERT_EQ(call(&sc, "r", &out), 0);
        seen.insert(out);
    }
    EXPECT_TRUE(seen == (std::set<std::string>{"r@b"}));
    sc.RemoveAndDestroyChannel(hb);
    EXPECT_EQ(call(&sc, "r", &out), EHOSTDOWN);
}

// A cancel that comes after enough sub calls succeeded: the call succeeds
// with what was merged (parallel_channel.cpp:375-381); with a fail_limit the
// canceled sub call reaches, it fails with ECANCELED.
TEST(ParallelChannel, cancel_after_partial_success) {
    TaggedServer fast("fast"), slow("slow");
    slow.echo.delay_us = 1000000;
    for (int limit : {2, 1}) {
        ParallelChannelOptions po;
        po.timeout_ms = 5000;
        po.fail_limit = limit;
        ParallelChannel pc;
        pc.Init(&po);
        pc.AddChannel(make_channel(fast.addr(), 5000), OWNS_CHANNEL, nullptr, std::make_shared<ConcatMerger>());
        pc.AddChannel(make_channel(slow.addr(), 5000), OWNS_CHANNEL, nullptr, std::make_shared<ConcatMerger>());
        example::EchoService_Stub stub(&pc);
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("c");
        std::atomic<int> done{0};
        const int64_t t0 = monotonic_us();
        stub.Echo(&cntl, &req, &res, NewCallback([&done] { done.fetch_add(1); }));
        usleep(150000);  // the fast sub call is back, the slow one sleeps
        StartCancel(cntl.call_id());
        for (int i = 0; i < 400 && !done.load(); ++i) usleep(2000);
        ASSERT_EQ(done.load(), 1);
        EXPECT_LT(monotonic_us() - t0, 800000);  // did not wait for the slow server
        if (limit == 2) {
            EXPECT_FALSE(cntl.Failed());
            EXPECT_EQ(res.message(), "c@fast");
        } else {
            EXPECT_EQ(cntl.ErrorCode(), ECANCELED);
        }
    }
}
