// More load balancer and naming cases, after the reference's
// test/brpc_load_balancer_unittest.cpp and brpc_naming_service_unittest.cpp:
// registry names and parameter parsing, duplicate/unknown membership
// changes, batch add/remove, empty LBs, the excluded-server fallbacks of
// each policy, wrr tags as weights, consistent hashing without a request
// code and with custom replicas, ExcludedServers eviction, and the
// address/tag parsing and list:// / dns:// / dlist:// / file:// naming
// services.
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <vector>

#include "base/time.h"
#include "cluster/load_balancer.h"
#include "cluster/naming_service.h"
#include "fiber/fiber.h"
#include "net/socket.h"
#include "rpc/errno.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

SocketId lazy_server(int port) {
    SocketOptions o;
    str2endpoint("127.0.0.1", port, &o.remote_side);
    o.connect_lazily = true;
    SocketId id = INVALID_SOCKET_ID;
    Socket::Create(o, &id);
    return id;
}

struct Servers {
    std::vector<SocketId> ids;
    Servers(int n, int base) {
        for (int i = 0; i < n; ++i) ids.push_back(lazy_server(base + i));
    }
    ~Servers() {
        for (SocketId id : ids) Socket::SetFailed(id);
    }
    int index_of(SocketId id) const {
        auto it = std::find(ids.begin(), ids.end(), id);
        return it == ids.end() ? -1 : (int)(it - ids.begin());
    }
};

int pick(LoadBalancer* lb, const Servers& s, const LoadBalancer::SelectIn& in, int* rc = nullptr) {
    SocketUniquePtr p;
    LoadBalancer::SelectOut out;
    out.ptr = &p;
    int r = lb->SelectServer(in, &out);
    if (rc) *rc = r;
    return r == 0 ? s.index_of(p->id()) : -1;
}

std::string describe(const LoadBalancer* lb) {
    std::ostringstream os;
    lb->Describe(os);
    return os.str();
}

struct Collect : NamingServiceActions {
    std::vector<std::vector<ServerNode>> resets;
    void ResetServers(const std::vector<ServerNode>& s) override { resets.push_back(s); }
};

}  // namespace

TEST(LbMore, every_builtin_is_listed_and_describes_itself) {
    std::vector<std::string> names = ListLoadBalancers();
    for (const char* n : {"rr", "random", "wrr", "wr", "la", "c_murmurhash", "c_md5", "c_ketama"}) {
        EXPECT_TRUE(std::find(names.begin(), names.end(), n) != names.end());
        std::unique_ptr<LoadBalancer> lb(CreateLoadBalancer(n));
        ASSERT_TRUE(lb != nullptr);
        if (std::string(n) != "la") EXPECT_EQ(describe(lb.get()), std::string(n));
        EXPECT_EQ(lb->ServerCount(), 0u);
    }
    EXPECT_TRUE(CreateLoadBalancer("no_such_lb") == nullptr);
    EXPECT_TRUE(CreateLoadBalancer("") == nullptr);
}

TEST(LbMore, malformed_recover_parameters_are_refused) {
    EXPECT_TRUE(CreateLoadBalancer("rr:min_working_instances=2") == nullptr);
    EXPECT_TRUE(CreateLoadBalancer("random:hold_seconds=x min_working_instances=2") == nullptr);
    std::unique_ptr<LoadBalancer> ok(CreateLoadBalancer("random:min_working_instances=2 hold_seconds=1"));
    EXPECT_TRUE(ok != nullptr);
}

TEST(LbMore, duplicate_and_unknown_membership_changes) {
    Servers s(3, 32100);
    for (const char* n : {"rr", "random", "wrr", "wr", "la", "c_md5"}) {
        std::unique_ptr<LoadBalancer> lb(CreateLoadBalancer(n));
        EXPECT_TRUE(lb->AddServer(ServerId(s.ids[0])));
        EXPECT_FALSE(lb->AddServer(ServerId(s.ids[0])));
        EXPECT_FALSE(lb->RemoveServer(ServerId(s.ids[1])));
        EXPECT_EQ(lb->ServerCount(), 1u);
        EXPECT_TRUE(lb->RemoveServer(ServerId(s.ids[0])));
        EXPECT_FALSE(lb->RemoveServer(ServerId(s.ids[0])));
        EXPECT_EQ(lb->ServerCount(), 0u);
    }
}

TEST(LbMore, batch_add_and_remove_count_what_changed) {
    Servers s(5, 32110);
    for (const char* n : {"rr", "wrr", "la", "c_murmurhash"}) {
        std::unique_ptr<LoadBalancer> lb(CreateLoadBalancer(n));
        std::vector<ServerId> v;
        for (SocketId id : s.ids) v.push_back(ServerId(id));
        v.push_back(ServerId(s.ids[0]));  // duplicate inside the batch
        EXPECT_EQ(lb->AddServersInBatch(v), 5u);
        EXPECT_EQ(lb->AddServersInBatch(v), 0u);
        std::vector<ServerId> rm = {ServerId(s.ids[1]), ServerId(s.ids[3]), ServerId(INVALID_SOCKET_ID - 1)};
        EXPECT_EQ(lb->RemoveServersInBatch(rm), 2u);
        EXPECT_EQ(lb->ServerCount(), 3u);
    }
}

TEST(LbMore, empty_balancers_say_host_down) {
    Servers s(1, 32120);
    LoadBalancer::SelectIn in;
    in.has_request_code = true;
    in.request_code = 42;
    for (const char* n : {"rr", "random", "wrr", "wr", "la", "c_murmurhash", "c_md5", "c_ketama"}) {
        std::unique_ptr<LoadBalancer> lb(CreateLoadBalancer(n));
        int rc = 0;
        EXPECT_EQ(pick(lb.get(), s, in, &rc), -1);
        EXPECT_EQ(rc, EHOSTDOWN);
    }
}

TEST(LbMore, consistent_hashing_needs_a_request_code) {
    Servers s(2, 32130);
    std::unique_ptr<LoadBalancer> lb(CreateLoadBalancer("c_murmurhash"));
    for (SocketId id : s.ids) lb->AddServer(ServerId(id));
    LoadBalancer::SelectIn in;
    int rc = 0;
    EXPECT_EQ(pick(lb.get(), s, in, &rc), -1);
    EXPECT_EQ(rc, EINVAL);
    in.has_request_code = true;
    in.request_code = 7;
    EXPECT_TRUE(pick(lb.get(), s, in, &rc) >= 0);
}

TEST(LbMore, same_code_same_server_across_instances_and_replica_counts) {
    Servers s(6, 32140);
    for (const char* spec : {"c_murmurhash", "c_md5", "c_ketama", "c_murmurhash:replicas=7", "c_md5:replicas=500"}) {
        std::unique_ptr<LoadBalancer> a(CreateLoadBalancer(spec)), b(CreateLoadBalancer(spec));
        ASSERT_TRUE(a && b);
        for (SocketId id : s.ids) a->AddServer(ServerId(id));
        for (auto it = s.ids.rbegin(); it != s.ids.rend(); ++it) b->AddServer(ServerId(*it));  // other order
        LoadBalancer::SelectIn in;
        in.has_request_code = true;
        std::set<int> used;
        for (uint64_t code = 0; code < 2000; ++code) {
            in.request_code = code * 2654435761u;
            int ka = pick(a.get(), s, in), kb = pick(b.get(), s, in);
            EXPECT_EQ(ka, kb);
            used.insert(ka);
        }
        EXPECT_EQ(used.size(), 6u);
    }
}

TEST(LbMore, consistent_hashing_walks_past_excluded_and_failed_nodes) {
    Servers s(4, 32150);
    std::unique_ptr<LoadBalancer> lb(CreateLoadBalancer("c_md5"));
    for (SocketId id : s.ids) lb->AddServer(ServerId(id));
    LoadBalancer::SelectIn in;
    in.has_request_code = true;
    in.request_code = 123456;
    const int home = pick(lb.get(), s, in);
    ASSERT_TRUE(home >= 0);
    ExcludedServers ex;
    ex.Add(s.ids[home]);
    in.excluded = &ex;
    const int next = pick(lb.get(), s, in);
    EXPECT_TRUE(next >= 0 && next != home);
    in.excluded = nullptr;
    Socket::SetFailed(s.ids[home]);
    EXPECT_EQ(pick(lb.get(), s, in), next);  // the ring's next live node
}

TEST(LbMore, rr_and_random_fall_back_to_excluded_servers) {
    Servers s(3, 32160);
    for (const char* n : {"rr", "random"}) {
        std::unique_ptr<LoadBalancer> lb(CreateLoadBalancer(n));
        for (SocketId id : s.ids) lb->AddServer(ServerId(id));
        ExcludedServers ex(3);
        for (SocketId id : s.ids) ex.Add(id);
        LoadBalancer::SelectIn in;
        in.excluded = &ex;
        int rc = -1;
        EXPECT_TRUE(pick(lb.get(), s, in, &rc) >= 0);  // better an excluded server than none
        EXPECT_EQ(rc, 0);
    }
}

TEST(LbMore, rr_cycles_through_live_servers_evenly) {
    Servers s(4, 32170);
    std::unique_ptr<LoadBalancer> lb(CreateLoadBalancer("rr"));
    for (SocketId id : s.ids) lb->AddServer(ServerId(id));
    Socket::SetFailed(s.ids[2]);
    LoadBalancer::SelectIn in;
    std::map<int, int> hits;
    for (int i = 0; i < 3000; ++i) ++hits[pick(lb.get(), s, in)];
    EXPECT_EQ(hits.count(2), 0u);
    EXPECT_EQ(hits.count(-1), 0u);
    // the failed server's turn goes to its successor
    EXPECT_NEAR(hits[0], 750, 2);
    EXPECT_NEAR(hits[1], 750, 2);
    EXPECT_NEAR(hits[3], 1500, 2);
}

TEST(LbMore, wrr_takes_weights_from_tags_and_ignores_bad_ones) {
    Servers s(3, 32180);
    std::unique_ptr<LoadBalancer> lb(CreateLoadBalancer("wrr"));
    lb->AddServer(ServerId(s.ids[0], "3"));
    lb->AddServer(ServerId(s.ids[1], "weight"));  // not a number: weight 1
    lb->AddServer(ServerId(s.ids[2], "-4"));      // not positive: weight 1
    LoadBalancer::SelectIn in;
    std::map<int, int> hits;
    for (int i = 0; i < 500; ++i) ++hits[pick(lb.get(), s, in)];
    EXPECT_EQ(hits[0], 300);
    EXPECT_EQ(hits[1], 100);
    EXPECT_EQ(hits[2], 100);
}

TEST(LbMore, wrr_schedule_follows_membership) {
    Servers s(3, 32190);
    std::unique_ptr<LoadBalancer> lb(CreateLoadBalancer("wrr"));
    lb->AddServer(ServerId(s.ids[0], "2"));
    lb->AddServer(ServerId(s.ids[1], "2"));
    LoadBalancer::SelectIn in;
    std::map<int, int> hits;
    for (int i = 0; i < 200; ++i) ++hits[pick(lb.get(), s, in)];
    EXPECT_EQ(hits[0], 100);
    EXPECT_EQ(hits[1], 100);
    lb->AddServer(ServerId(s.ids[2], "4"));
    lb->RemoveServer(ServerId(s.ids[0]));
    hits.clear();
    for (int i = 0; i < 600; ++i) ++hits[pick(lb.get(), s, in)];
    EXPECT_EQ(hits.count(0), 0u);
    EXPECT_EQ(hits[1], 200);
    EXPECT_EQ(hits[2], 400);
}

TEST(LbMore, wr_skips_the_excluded_unless_it_is_the_last) {
    Servers s(2, 32200);
    std::unique_ptr<LoadBalancer> lb(CreateLoadBalancer("wr"));
    lb->AddServer(ServerId(s.ids[0], "1"));
    lb->AddServer(ServerId(s.ids[1], "1"));
    ExcludedServers ex;
    ex.Add(s.ids[0]);
    LoadBalancer::SelectIn in;
    in.excluded = &ex;
    std::map<int, int> hits;
    for (int i = 0; i < 400; ++i) ++hits[pick(lb.get(), s, in)];
    // draws landing on 0 move to 1; draws landing on 1 with 0 as the only
    // fallback keep 1: in both cases the excluded server is avoided unless
    // it is the last candidate of the walk
    EXPECT_TRUE(hits[1] > 300);
}

TEST(LbMore, la_describes_its_weights) {
    Servers s(2, 32210);
    std::unique_ptr<LoadBalancer> lb(CreateLoadBalancer("la"));
    for (SocketId id : s.ids) lb->AddServer(ServerId(id));
    std::string d = describe(lb.get());
    EXPECT_TRUE(d.find("la") != std::string::npos);
    EXPECT_EQ(lb->ServerCount(), 2u);
}

TEST(LbMore, excluded_servers_keep_the_newest) {
    ExcludedServers ex(2);
    ex.Add(1);
    ex.Add(2);
    ex.Add(2);  // already there
    EXPECT_EQ(ex.size(), 2u);
    ex.Add(3);  // evicts 1
    EXPECT_FALSE(ex.IsExcluded(1));
    EXPECT_TRUE(ex.IsExcluded(2));
    EXPECT_TRUE(ex.IsExcluded(3));
    EXPECT_EQ(ex.size(), 2u);
}

TEST(LbMore, server_ids_order_by_socket_then_tag) {
    ServerId a(5, "x"), b(5, "y"), c(6, "");
    EXPECT_TRUE(a < b);
    EXPECT_TRUE(b < c);
    EXPECT_FALSE(c < a);
    EXPECT_TRUE(a == ServerId(5, "x"));
    EXPECT_FALSE(a == b);
}

TEST(NsMore, server_node_lines) {
    ServerNode n;
    EXPECT_TRUE(ParseServerNode("127.0.0.1:8000", &n));
    EXPECT_EQ(n.addr.port, 8000);
    EXPECT_TRUE(n.tag.empty());
    EXPECT_TRUE(ParseServerNode("  10.0.0.2:81   tag with spaces  ", &n));
    EXPECT_EQ(n.addr.port, 81);
    EXPECT_EQ(n.tag, "tag with spaces");
    EXPECT_TRUE(ParseServerNode("localhost:9000\t7", &n));
    EXPECT_EQ(n.addr.port, 9000);
    EXPECT_EQ(n.tag, "7");
    EXPECT_FALSE(ParseServerNode("", &n));
    EXPECT_FALSE(ParseServerNode("   ", &n));
    EXPECT_FALSE(ParseServerNode("# 127.0.0.1:80", &n));
    EXPECT_FALSE(ParseServerNode("127.0.0.1:99999", &n));
    EXPECT_FALSE(ParseServerNode("not an address at all", &n));
}

TEST(NsMore, server_nodes_compare_by_address_then_tag) {
    ServerNode a, b, c;
    ParseServerNode("127.0.0.1:80 a", &a);
    ParseServerNode("127.0.0.1:80 b", &b);
    ParseServerNode("127.0.0.1:81", &c);
    EXPECT_TRUE(a < b);
    EXPECT_TRUE(a < c && b < c);
    EXPECT_FALSE(a == b);
    ServerNode a2;
    ParseServerNode("127.0.0.1:80   a", &a2);
    EXPECT_TRUE(a == a2);
}

TEST(NsMore, list_service_keeps_good_entries_in_order) {
    std::unique_ptr<NamingService> ns(CreateNamingService("list"));
    ASSERT_TRUE(ns != nullptr);
    EXPECT_TRUE(ns->RunNamingServiceReturnsQuickly());
    Collect c;
    EXPECT_EQ(ns->RunNamingService("127.0.0.1:1 t1, bogus,,127.0.0.1:3,127.0.0.1:2 t2", &c), 0);
    ASSERT_EQ(c.resets.size(), 1u);
    ASSERT_EQ(c.resets[0].size(), 3u);
    EXPECT_EQ(c.resets[0][0].addr.port, 1);
    EXPECT_EQ(c.resets[0][0].tag, "t1");
    EXPECT_EQ(c.resets[0][1].addr.port, 3);
    EXPECT_EQ(c.resets[0][2].tag, "t2");
}

TEST(NsMore, unknown_scheme_has_no_service) {
    EXPECT_TRUE(CreateNamingService("gopher") == nullptr);
    for (const char* s : {"list", "file", "http", "https", "dns", "redis", "dlist", "remotefile", "consul",
                          "discovery", "nacos"}) {
        std::unique_ptr<NamingService> ns(CreateNamingService(s));
        EXPECT_TRUE(ns != nullptr);
    }
}

TEST(NsMore, dns_resolves_localhost_with_default_and_explicit_ports) {
    std::unique_ptr<NamingService> http(CreateNamingService("http"));
    auto* p = dynamic_cast<PeriodicNamingService*>(http.get());
    ASSERT_TRUE(p != nullptr);
    std::vector<ServerNode> v;
    ASSERT_EQ(p->GetServers("localhost", &v), 0);
    ASSERT_TRUE(!v.empty());
    EXPECT_EQ(v[0].addr.port, 80);
    v.clear();
    ASSERT_EQ(p->GetServers("localhost:8123/some/path", &v), 0);
    EXPECT_EQ(v[0].addr.port, 8123);
    std::unique_ptr<NamingService> https(CreateNamingService("https"));
    v.clear();
    ASSERT_EQ(dynamic_cast<PeriodicNamingService*>(https.get())->GetServers("localhost", &v), 0);
    EXPECT_EQ(v[0].addr.port, 443);
    v.clear();
    EXPECT_NE(p->GetServers("no-such-host.invalid", &v), 0);
}

TEST(NsMore, dlist_merges_domains_and_fails_only_if_none_resolve) {
    std::unique_ptr<NamingService> ns(CreateNamingService("dlist"));
    auto* p = dynamic_cast<PeriodicNamingService*>(ns.get());
    ASSERT_TRUE(p != nullptr);
    std::vector<ServerNode> v;
    EXPECT_EQ(p->GetServers("localhost:81, no-such-host.invalid:82 ,localhost:83", &v), 0);
    std::set<int> ports;
    for (auto& n : v) ports.insert(n.addr.port);
    EXPECT_EQ(ports.count(81), 1u);
    EXPECT_EQ(ports.count(83), 1u);
    EXPECT_EQ(ports.count(82), 0u);
    v.clear();
    EXPECT_NE(p->GetServers("no-such-host.invalid:1", &v), 0);
}

TEST(NsMore, access_interval_follows_the_flag_with_a_floor) {
    std::unique_ptr<NamingService> ns(CreateNamingService("dns"));
    auto* p = dynamic_cast<PeriodicNamingService*>(ns.get());
    ASSERT_TRUE(p != nullptr);
    EXPECT_TRUE(p->GetNamingServiceAccessIntervalMs() >= 1000);
}

TEST(NsMore, file_service_reloads_when_the_file_changes) {
    char path[] = "/tmp/mrpc_ns_more_XXXXXX";
    int fd = mkstemp(path);
    ASSERT_TRUE(fd >= 0);
    const char* first = "127.0.0.1:9001\n# comment\n\n127.0.0.1:9002 tagged\n";
    ASSERT_EQ(write(fd, first, strlen(first)), (ssize_t)strlen(first));
    close(fd);
    struct Shared : NamingServiceActions {
        std::mutex mu;
        std::vector<std::vector<ServerNode>> resets;
        void ResetServers(const std::vector<ServerNode>& s) override {
            std::lock_guard<std::mutex> g(mu);
            resets.push_back(s);
        }
        size_t count() {
            std::lock_guard<std::mutex> g(mu);
            return resets.size();
        }
    } acts;
    std::unique_ptr<NamingService> ns(CreateNamingService("file"));
    std::string p = path;
    fiber::fiber_t tid;
    ASSERT_EQ(fiber::start([&] { ns->RunNamingService(p.c_str(), &acts); }, false, nullptr, &tid), 0);
    for (int i = 0; i < 200 && acts.count() < 1; ++i) usleep(10000);
    ASSERT_EQ(acts.count(), 1u);
    {
        std::lock_guard<std::mutex> g(acts.mu);
        ASSERT_EQ(acts.resets[0].size(), 2u);
        EXPECT_EQ(acts.resets[0][1].tag, "tagged");
    }
    // rewrite with a later mtime
    sleep(1);
    FILE* f = fopen(path, "w");
    fputs("127.0.0.1:9003\n", f);
    fclose(f);
    for (int i = 0; i < 300 && acts.count() < 2; ++i) usleep(10000);
    EXPECT_EQ(acts.count(), 2u);
    {
        std::lock_guard<std::mutex> g(acts.mu);
        if (acts.resets.size() >= 2) {
            ASSERT_EQ(acts.resets[1].size(), 1u);
            EXPECT_EQ(acts.resets[1][0].addr.port, 9003);
        }
    }
    fiber::stop(tid);
    fiber::join(tid);
    unlink(path);
}
