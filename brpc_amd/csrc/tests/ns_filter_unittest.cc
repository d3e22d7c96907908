// NamingServiceFilter (spirit of the reference's
// test/brpc_naming_service_filter_unittest.cpp): servers the filter
// rejects never receive calls; tags reach the filter; a filter that
// rejects everything leaves the channel without servers.
#include <memory>
#include <string>
#include <vector>

#include "cluster/naming_service.h"
#include "mrpc/proto/echo.pb.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

using namespace mrpc;

namespace {
struct Three {
    std::vector<std::unique_ptr<Server>> servers;
    std::vector<std::unique_ptr<EchoServiceImpl>> echos;
    std::string list;  // list:// url with tags a, b, c
    Three() {
        const char* tags[] = {"a", "b", "c"};
        for (int i = 0; i < 3; ++i) {
            echos.emplace_back(new EchoServiceImpl);
            servers.emplace_back(new Server);
            servers.back()->AddService(echos.back().get(), SERVER_DOESNT_OWN_SERVICE);
            ServerOptions so;
            so.has_builtin_services = false;
            servers.back()->Start("127.0.0.1:0", &so);
            list += std::string(i ? "," : "list://") + "127.0.0.1:" + std::to_string(servers.back()->listen_port()) +
                    " " + tags[i];
        }
    }
    ~Three() {
        for (auto& s : servers) {
            s->Stop(0);
            s->Join();
        }
    }
    std::vector<int64_t> calls(Channel* ch, int n, int* failed) {
        std::vector<int64_t> before;
        for (auto& e : echos) before.push_back(e->ncalls());
        example::EchoService_Stub stub(ch);
        for (int i = 0; i < n; ++i) {
            Controller cntl;
            example::EchoRequest req;
            example::EchoResponse res;
            req.set_message("f");
            stub.Echo(&cntl, &req, &res, nullptr);
            if (cntl.Failed()) ++*failed;
        }
        std::vector<int64_t> d;
        for (size_t i = 0; i < echos.size(); ++i) d.push_back(echos[i]->ncalls() - before[i]);
        return d;
    }
};

struct TagFilter : public NamingServiceFilter {
    std::string reject;
    mutable int seen = 0;
    bool Accept(const ServerNode& s) const override {
        ++seen;
        return s.tag != reject;
    }
};
struct NoneFilter : public NamingServiceFilter {
    bool Accept(const ServerNode&) const override { return false; }
};
}  // namespace

TEST(NsFilter, rejected_servers_get_no_calls) {
    Three t;
    TagFilter f;
    f.reject = "b";
    Channel ch;
    ChannelOptions o;
    o.timeout_ms = 2000;
    o.ns_filter = &f;
    ASSERT_EQ(ch.Init(t.list.c_str(), "rr", &o), 0);
    int failed = 0;
    const std::vector<int64_t> d = t.calls(&ch, 40, &failed);
    EXPECT_EQ(failed, 0);
    EXPECT_EQ(d[0], 20);
    EXPECT_EQ(d[1], 0);
    EXPECT_EQ(d[2], 20);
    EXPECT_GE(f.seen, 3);  // every resolved node went through the filter, tags included
}

TEST(NsFilter, without_a_filter_every_server_serves) {
    Three t;
    Channel ch;
    ChannelOptions o;
    o.timeout_ms = 2000;
    ASSERT_EQ(ch.Init(t.list.c_str(), "rr", &o), 0);
    int failed = 0;
    const std::vector<int64_t> d = t.calls(&ch, 30, &failed);
    EXPECT_EQ(failed, 0);
    EXPECT_EQ(d[0], 10);
    EXPECT_EQ(d[1], 10);
    EXPECT_EQ(d[2], 10);
}

TEST(NsFilter, rejecting_everything_leaves_no_server) {
    Three t;
    NoneFilter f;
    Channel ch;
    ChannelOptions o;
    o.timeout_ms = 500;
    o.max_retry = 0;
    o.ns_filter = &f;
    ch.Init(t.list.c_str(), "rr", &o);  // may fail or succeed with an empty server set
    int failed = 0;
    const std::vector<int64_t> d = t.calls(&ch, 5, &failed);
    EXPECT_EQ(failed, 5);
    EXPECT_EQ(d[0] + d[1] + d[2], 0);
}
