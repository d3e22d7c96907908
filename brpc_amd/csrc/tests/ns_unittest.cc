// Naming services against mocked control planes (spirit of the reference's
// test/brpc_naming_service_unittest.cpp:199-265,404-440,557, which emulates
// consul/discovery/nacos with in-process brpc HTTP services): one HTTP
// server of this framework plays consul, discovery, nacos and a remotefile
// host; the naming services resolve through it, then a Channel load
// balances real echo calls across what they resolved — and follows a
// membership change.
#include <unistd.h>

#include <algorithm>
#include <mutex>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "base/flags.h"
#include "base/time.h"
#include "cluster/naming_service.h"
#include "http/http_client.h"
#include "http/http_header.h"
#include "mrpc/proto/echo.pb.h"
#include "mrpc/proto/test_services.pb.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

DECLARE_string(consul_agent_addr);
DECLARE_string(discovery_api_addr);
DECLARE_string(nacos_address);
DECLARE_int32(ns_access_interval);

using namespace mrpc;

namespace {

// The mocked control plane: every unmatched HTTP request lands in the first
// method of ServerOptions.http_master_service (Push) and is answered from
// `servers`.
class ControlPlane : public test::HttpTest {
public:
    void Raw(RpcController*, const test::Empty*, test::Empty*, Closure* done) override { done->Run(); }
    void Rich(RpcController*, const test::Rich*, test::Rich*, Closure* done) override { done->Run(); }
    void Push(RpcController* c, const test::Empty*, test::Empty*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = static_cast<Controller*>(c);
        const std::string path = cntl->http_request().uri().path();
        std::vector<std::pair<std::string, int>> s;
        {
            std::lock_guard<std::mutex> lk(mu);
            s = servers;
            ++hits;
        }
        std::ostringstream os;
        if (path == "/v1/health/service/echo") {  // consul
            os << "[";
            for (size_t i = 0; i < s.size(); ++i) {
                os << (i ? "," : "") << "{\"Node\":{\"Node\":\"n" << i << "\"},\"Service\":{\"ID\":\"echo" << i
                   << "\",\"Service\":\"echo\",\"Tags\":[\"t" << i << "\"],\"Address\":\"" << s[i].first
                   << "\",\"Port\":" << s[i].second << "}}";
            }
            os << "]";
        } else if (path == "/discovery/fetchs") {
            // only appid "echo" is registered
            os << "{\"code\":0,\"data\":{\"echo\":{\"instances\":[";
            for (size_t i = 0; i < s.size(); ++i) {
                os << (i ? "," : "") << "{\"hostname\":\"h" << i << "\",\"addrs\":[\"grpc://" << s[i].first << ":"
                   << s[i].second << "\"],\"status\":1}";
            }
            os << "]}}}";
        } else if (path == "/nacos/v1/ns/instance/list") {
            os << "{\"name\":\"echo\",\"hosts\":[";
            for (size_t i = 0; i < s.size(); ++i) {
                os << "{\"ip\":\"" << s[i].first << "\",\"port\":" << s[i].second << ",\"weight\":" << (i + 1)
                   << ".0,\"healthy\":true},";
            }
            os << "{\"ip\":\"127.0.0.1\",\"port\":1,\"weight\":1.0,\"healthy\":false}]}";  // filtered out
        } else if (path == "/servers.txt") {  // remotefile
            for (size_t i = 0; i < s.size(); ++i) os << s[i].first << ":" << s[i].second << " rf" << i << "\n";
            os << "# comment line\n\n";
        } else {
            cntl->http_response().set_status_code(404);
        }
        cntl->response_attachment().append(os.str());
    }
    void set(const std::vector<std::pair<std::string, int>>& s) {
        std::lock_guard<std::mutex> lk(mu);
        servers = s;
    }
    std::mutex mu;
    std::vector<std::pair<std::string, int>> servers;
    int hits = 0;
};

struct Env {
    ControlPlane plane;
    Server control;
    std::vector<std::unique_ptr<Server>> echo_servers;
    std::vector<std::unique_ptr<EchoServiceImpl>> echos;
    std::string control_addr;
    Env() {
        ServerOptions o;
        o.http_master_service = &plane;
        control.Start("127.0.0.1:0", &o);
        control_addr = "http://127.0.0.1:" + std::to_string(control.listen_port());
        FLAGS_consul_agent_addr = control_addr;
        FLAGS_discovery_api_addr = control_addr;
        FLAGS_nacos_address = control_addr;
        for (int i = 0; i < 3; ++i) {
            echos.emplace_back(new EchoServiceImpl);
            echo_servers.emplace_back(new Server);
            echo_servers.back()->AddService(echos.back().get(), SERVER_DOESNT_OWN_SERVICE);
            ServerOptions eo;
            echo_servers.back()->Start("127.0.0.1:0", &eo);
        }
        use(2);
    }
    void use(int n) {
        std::vector<std::pair<std::string, int>> s;
        for (int i = 0; i < n; ++i) s.emplace_back("127.0.0.1", echo_servers[i]->listen_port());
        plane.set(s);
    }
    std::set<int> ports(int n) const {
        std::set<int> p;
        for (int i = 0; i < n; ++i) p.insert(echo_servers[i]->listen_port());
        return p;
    }
};

Env& env() {
    static Env* e = new Env;
    return *e;
}

std::set<int> resolve(const std::string& scheme, const std::string& name, std::vector<ServerNode>* nodes = nullptr) {
    std::unique_ptr<NamingService> ns(CreateNamingService(scheme));
    std::set<int> ports;
    if (!ns) return ports;
    PeriodicNamingService* p = dynamic_cast<PeriodicNamingService*>(ns.get());
    if (!p) return ports;
    std::vector<ServerNode> out;
    if (p->GetServers(name.c_str(), &out) != 0) return ports;
    for (auto& n : out) ports.insert(n.addr.port);
    if (nodes) *nodes = out;
    return ports;
}

}  // namespace

TEST(NamingService, list_parses_tags_and_rejects_garbage) {
    ServerNode n;
    EXPECT_TRUE(ParseServerNode("127.0.0.1:8000", &n));
    EXPECT_EQ(n.addr.port, 8000);
    EXPECT_TRUE(ParseServerNode("127.0.0.1:8001 tagx", &n));
    EXPECT_EQ(n.tag, std::string("tagx"));
    EXPECT_FALSE(ParseServerNode("not an address", &n));
    std::vector<ServerNode> out;
    std::unique_ptr<NamingService> ns(CreateNamingService("list"));
    ASSERT_TRUE(ns != nullptr);
    EXPECT_TRUE(CreateNamingService("no_such_scheme") == nullptr);
}

TEST(NamingService, control_plane_answers_http) {
    Env& e = env();
    HttpSimpleResponse r;
    const int rc = HttpFetch("GET", e.control_addr + "/v1/health/service/echo?passing", "", &r, 2000);
    fprintf(stderr, "rc=%d status=%d body=%s\n", rc, r.status, r.body.substr(0, 200).c_str());
    EXPECT_EQ(rc, 0);
    EXPECT_EQ(r.status, 200);
}

TEST(NamingService, consul_mock) {
    Env& e = env();
    std::vector<ServerNode> nodes;
    EXPECT_TRUE(resolve("consul", "echo", &nodes) == e.ports(2));
    ASSERT_EQ(nodes.size(), 2u);
    EXPECT_EQ(nodes[0].tag, std::string("t0"));  // first consul tag
}

TEST(NamingService, discovery_mock) {
    Env& e = env();
    EXPECT_TRUE(resolve("discovery", "echo") == e.ports(2));
    // an unknown appid resolves to nothing (not an error)
    EXPECT_TRUE(resolve("discovery", "nobody").empty());
}

TEST(NamingService, nacos_mock_filters_unhealthy_and_keeps_weights) {
    Env& e = env();
    std::vector<ServerNode> nodes;
    EXPECT_TRUE(resolve("nacos", "echo", &nodes) == e.ports(2));  // the unhealthy port 1 is dropped
    ASSERT_EQ(nodes.size(), 2u);
    std::set<std::string> tags;
    for (auto& n : nodes) tags.insert(n.tag);
    EXPECT_TRUE(tags.count("1") && tags.count("2"));  // weights become wr/wrr tags
}

TEST(NamingService, remotefile_mock) {
    Env& e = env();
    const std::string host = e.control_addr.substr(strlen("http://"));
    std::vector<ServerNode> nodes;
    EXPECT_TRUE(resolve("remotefile", host + "/servers.txt", &nodes) == e.ports(2));
    ASSERT_EQ(nodes.size(), 2u);
    EXPECT_EQ(nodes[1].tag, std::string("rf1"));
}

TEST(NamingService, control_plane_down_is_an_error) {
    std::unique_ptr<NamingService> ns(CreateNamingService("consul"));
    PeriodicNamingService* p = dynamic_cast<PeriodicNamingService*>(ns.get());
    ASSERT_TRUE(p != nullptr);
    const std::string saved = FLAGS_consul_agent_addr;
    FLAGS_consul_agent_addr = "http://127.0.0.1:1";
    std::vector<ServerNode> out;
    EXPECT_NE(p->GetServers("echo", &out), 0);
    FLAGS_consul_agent_addr = saved;
}

TEST(NamingService, channels_follow_membership_changes) {
    // Channel over consul:// with rr: calls reach exactly the resolved
    // servers; after the control plane adds a third server the naming
    // service thread hands it to the LB within one access interval.
    Env& e = env();
    const int saved = FLAGS_ns_access_interval;
    FLAGS_ns_access_interval = 1;
    for (const char* url : {"consul://echo", "nacos://echo", "discovery://echo"}) {
        e.use(2);
        Channel ch;
        ChannelOptions o;
        o.timeout_ms = 2000;
        ASSERT_EQ(ch.Init(url, "rr", &o), 0);
        example::EchoService_Stub stub(&ch);
        auto calls_by_server = [&](int n) {
            std::vector<int64_t> before;
            for (auto& s : e.echos) before.push_back(s->ncalls());
            for (int i = 0; i < n; ++i) {
                Controller cntl;
                example::EchoRequest req;
                example::EchoResponse res;
                req.set_message("ns");
                stub.Echo(&cntl, &req, &res, nullptr);
                EXPECT_FALSE(cntl.Failed());
            }
            std::vector<int64_t> d;
            for (size_t i = 0; i < e.echos.size(); ++i) d.push_back(e.echos[i]->ncalls() - before[i]);
            return d;
        };
        std::vector<int64_t> d = calls_by_server(60);
        EXPECT_EQ(d[0], 30);
        EXPECT_EQ(d[1], 30);
        EXPECT_EQ(d[2], 0);
        e.use(3);
        usleep(2500 * 1000);
        d = calls_by_server(90);
        EXPECT_EQ(d[0], 30);
        EXPECT_EQ(d[1], 30);
        EXPECT_EQ(d[2], 30);
    }
    FLAGS_ns_access_interval = saved;
}
