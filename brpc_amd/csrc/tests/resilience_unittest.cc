// Cluster recover policy and -usercode_in_pthread (spirit of the reference's
// cluster_recover_policy tests in brpc_load_balancer_unittest.cpp and the
// usercode_in_pthread runs of brpc_server_unittest.cpp).
#include <unistd.h>

#include <atomic>
#include <memory>
#include <vector>

#include "base/flags.h"
#include "base/time.h"
#include "cluster/cluster_recover_policy.h"
#include "mrpc/proto/echo.pb.h"
#include "rpc/channel.h"
#include "rpc/errno.h"
#include "rpc/server.h"
#include "rpc/usercode_backup_pool.h"
#include "tests/test.h"

using namespace mrpc;

TEST(ClusterRecover, params_parsing) {
    std::shared_ptr<ClusterRecoverPolicy> p;
    EXPECT_TRUE(GetRecoverPolicyByParams("", &p));
    EXPECT_TRUE(p == nullptr);
    EXPECT_TRUE(GetRecoverPolicyByParams("min_working_instances=4 hold_seconds=2", &p));
    EXPECT_TRUE(p != nullptr);
    EXPECT_FALSE(GetRecoverPolicyByParams("min_working_instances=x", &p));
    EXPECT_FALSE(GetRecoverPolicyByParams("hold_seconds=3", &p));
}

TEST(ClusterRecover, rejects_proportionally_then_recovers) {
    DefaultClusterRecoverPolicy p(10, 1);
    std::vector<ServerId> none;  // no usable server at all
    EXPECT_FALSE(p.StopRecoverIfNecessary());
    p.StartRecover();
    EXPECT_TRUE(p.StopRecoverIfNecessary());
    int rejected = 0;
    for (int i = 0; i < 1000; ++i) rejected += p.DoReject(none) ? 1 : 0;
    EXPECT_EQ(rejected, 1000);  // 0 usable of 10 wanted: reject everything
    // recovery only ends once some server came back and the usable count
    // then stayed stable for hold_seconds: with none usable it keeps going
    usleep(1200 * 1000);
    EXPECT_TRUE(p.StopRecoverIfNecessary());
    EXPECT_TRUE(p.DoReject(none));
}

TEST(ClusterRecover, lb_returns_ereject_while_recovering) {
    Server server;
    ServerOptions o;
    o.has_builtin_services = false;
    ASSERT_EQ(server.Start("127.0.0.1:0", &o), 0);
    const int live = server.listen_port();
    server.Stop(0);
    server.Join();
    // list with one dead server; rr with a recover policy
    Channel ch;
    ChannelOptions opt;
    opt.max_retry = 0;
    opt.timeout_ms = 500;
    const std::string url = "list://127.0.0.1:" + std::to_string(live);
    ASSERT_EQ(ch.Init(url.c_str(), "rr:min_working_instances=3 hold_seconds=10", &opt), 0);
    example::EchoService_Stub stub(&ch);
    int hostdown = 0, rejected = 0;
    for (int i = 0; i < 20; ++i) {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("x");
        stub.Echo(&cntl, &req, &res, nullptr);
        EXPECT_TRUE(cntl.Failed());
        if (cntl.ErrorCode() == EREJECT) ++rejected;
        else ++hostdown;
        usleep(20000);
    }
    // the first failures start recovery; afterwards calls are rejected up front
    EXPECT_GT(rejected, 0);
}

namespace {
// A service that blocks its pthread (sleeps) — the case usercode_in_pthread is for.
class BlockingEcho : public example::EchoService {
public:
    std::atomic<int> running{0}, max_running{0};
    void Echo(RpcController*, const example::EchoRequest* req, example::EchoResponse* res, Closure* done) override {
        ClosureGuard g(done);
        const int r = running.fetch_add(1) + 1;
        int m = max_running.load();
        while (r > m && !max_running.compare_exchange_weak(m, r)) {
        }
        usleep(20000);  // blocking syscall, not a fiber sleep
        running.fetch_sub(1);
        res->set_message(req->message());
    }
};
}  // namespace

TEST(UsercodeInPthread, blocking_handlers_do_not_starve_io) {
    SetFlag("usercode_in_pthread", "true");
    BlockingEcho svc;
    Server server;
    server.AddService(&svc, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions o;
    o.has_builtin_services = false;
    ASSERT_EQ(server.Start("127.0.0.1:0", &o), 0);
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 10000;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    const int N = 40;
    std::vector<std::unique_ptr<Controller>> cntls(N);
    std::vector<example::EchoRequest> reqs(N);
    std::vector<example::EchoResponse> ress(N);
    const int64_t t0 = monotonic_us();
    for (int i = 0; i < N; ++i) {
        cntls[i].reset(new Controller);
        reqs[i].set_message("b" + std::to_string(i));
        stub.Echo(cntls[i].get(), &reqs[i], &ress[i], NewCallback([] {}));
    }
    for (int i = 0; i < N; ++i) {
        cntls[i]->Join();
        ASSERT_FALSE(cntls[i]->Failed());
        EXPECT_EQ(ress[i].message(), reqs[i].message());
    }
    const int64_t elapsed = monotonic_us() - t0;
    SetFlag("usercode_in_pthread", "false");
    // in-place + backup pthreads ran handlers concurrently
    EXPECT_GE(svc.max_running.load(), 2);
    EXPECT_LT(elapsed, (int64_t)N * 20000);
}
