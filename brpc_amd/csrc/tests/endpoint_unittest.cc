// EndPoint depth (base/endpoint.h), in the spirit of the reference's
// test/endpoint_unittest.cpp: IPv4, IPv6 (with zones) and unix-socket
// endpoints parsed, printed, compared, hashed, converted to and from
// sockaddrs through real sockets, and parsed concurrently.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <set>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "base/containers.h"
#include "base/endpoint.h"
#include "tests/test.h"

using namespace mrpc;

TEST(EndPointDepth, ipv4_bounds) {
    EndPoint ep;
    ASSERT_EQ(str2endpoint("0.0.0.0:0", &ep), 0);
    EXPECT_EQ(ep.ip, 0u);
    EXPECT_EQ(ep.port, 0);
    ASSERT_EQ(str2endpoint("255.255.255.255:65535", &ep), 0);
    EXPECT_EQ(ep.ip, 0xFFFFFFFFu);
    EXPECT_EQ(ep.port, 65535);
    EXPECT_EQ(ep.to_string(), "255.255.255.255:65535");
    const char* bad[] = {"256.0.0.1:80", "1.2.3.4:-1", "1.2.3.4:65536", "1.2.3.4:", ":80", "1.2.3.4:8o", "", "1.2.3.4.5:80"};
    for (const char* s : bad) EXPECT_TRUE_M(str2endpoint(s, &ep) != 0, std::string(s));
}

TEST(EndPointDepth, ip_strings_round_trip) {
    uint32_t ip = 0;
    ASSERT_EQ(str2ip("10.20.30.40", &ip), 0);
    EXPECT_EQ(ip2str(ip), "10.20.30.40");
    EXPECT_EQ(ntohl(ip), 0x0A141E28u);
    EXPECT_NE(str2ip("10.20.30", &ip), 0);
    EXPECT_NE(str2ip("a.b.c.d", &ip), 0);
    EndPoint ep;
    ASSERT_EQ(str2endpoint("192.168.1.7", 443, &ep), 0);
    EXPECT_EQ(ep.to_string(), "192.168.1.7:443");
    EXPECT_EQ(ep.ip_string(), "192.168.1.7");
}

TEST(EndPointDepth, ipv6_forms) {
    EndPoint ep;
    ASSERT_EQ(str2endpoint("[::1]:8080", &ep), 0);
    EXPECT_TRUE(ep.is_ipv6());
    EXPECT_EQ(ep.port, 8080);
    EXPECT_EQ(ep.ip6[15], 1);
    EXPECT_EQ(ep.to_string(), "[::1]:8080");
    ASSERT_EQ(str2endpoint("[2001:db8::ff00:42:8329]:1", &ep), 0);
    EXPECT_EQ(ep.ip6[0], 0x20);
    EXPECT_EQ(ep.ip6[1], 0x01);
    EXPECT_EQ(ep.ip6[15], 0x29);
    EXPECT_EQ(ep.to_string(), "[2001:db8::ff00:42:8329]:1");
    // the ip-and-port form
    ASSERT_EQ(str2endpoint("::1", 99, &ep), 0);
    EXPECT_TRUE(ep.is_ipv6());
    EXPECT_EQ(ep.port, 99);
    const char* bad[] = {"[::1]", "[::1]:", "[::g]:80", "[:::1]:80", "::1:80x"};
    for (const char* s : bad) EXPECT_TRUE_M(str2endpoint(s, &ep) != 0, std::string(s));
}

TEST(EndPointDepth, ipv6_zone_on_link_local) {
    EndPoint ep;
    ASSERT_EQ(str2endpoint("[fe80::1%1]:80", &ep), 0);
    EXPECT_TRUE(ep.is_ipv6());
    EXPECT_EQ(ep.scope_id, 1u);
    EndPoint other;
    ASSERT_EQ(str2endpoint("[fe80::1%2]:80", &other), 0);
    EXPECT_TRUE(ep != other);  // the zone is part of the address
    EXPECT_TRUE(ep < other || other < ep);
}

TEST(EndPointDepth, unix_socket_endpoints) {
    EndPoint ep;
    ASSERT_EQ(str2endpoint("unix:/tmp/some.sock", &ep), 0);
    EXPECT_TRUE(ep.is_unix());
    EXPECT_FALSE(ep.is_ipv6());
    EXPECT_EQ(ep.path, "/tmp/some.sock");
    EXPECT_EQ(ep.to_string(), "unix:/tmp/some.sock");
    EndPoint b;
    ASSERT_EQ(str2endpoint("unix:/tmp/other.sock", &b), 0);
    EXPECT_TRUE(ep != b);
    EXPECT_TRUE(b < ep);
}

TEST(EndPointDepth, ordering_is_total_across_families) {
    std::vector<std::string> specs = {"10.0.0.1:1", "10.0.0.1:2", "10.0.0.2:1", "[::1]:1", "[::2]:1", "unix:/a",
                                      "unix:/b", "0.0.0.0:0"};
    std::vector<EndPoint> eps;
    for (const std::string& s : specs) {
        EndPoint e;
        ASSERT_EQ(str2endpoint(s.c_str(), &e), 0);
        eps.push_back(e);
    }
    // irreflexive and asymmetric, and equal ones are exactly the same spec
    for (size_t i = 0; i < eps.size(); ++i) {
        EXPECT_FALSE(eps[i] < eps[i]);
        for (size_t j = 0; j < eps.size(); ++j) {
            if (i == j) continue;
            EXPECT_TRUE(eps[i] != eps[j]);
            EXPECT_TRUE((eps[i] < eps[j]) != (eps[j] < eps[i]));
        }
    }
    std::set<EndPoint> uniq(eps.begin(), eps.end());
    EXPECT_EQ(uniq.size(), eps.size());
}

TEST(EndPointDepth, hashing_in_tables) {
    std::unordered_set<EndPoint, EndPointHash> s;
    for (int port = 1; port <= 500; ++port) {
        EndPoint a(htonl(0x7F000001), port), b;
        ASSERT_EQ(str2endpoint("::1", port, &b), 0);
        s.insert(a);
        s.insert(b);
    }
    EXPECT_EQ(s.size(), 1000u);
    EndPoint probe;
    str2endpoint("[::1]:77", &probe);
    EXPECT_EQ(s.count(probe), 1u);
    str2endpoint("127.0.0.1:77", &probe);
    EXPECT_EQ(s.count(probe), 1u);
    str2endpoint("127.0.0.1:501", &probe);
    EXPECT_EQ(s.count(probe), 0u);
}

TEST(EndPointDepth, sockaddr_conversion_through_ipv4_sockets) {
    EndPoint any;
    ASSERT_EQ(str2endpoint("127.0.0.1:0", &any), 0);
    const int lfd = tcp_listen(any);
    ASSERT_GE(lfd, 0);
    EndPoint bound;
    ASSERT_EQ(get_local_side(lfd, &bound), 0);
    EXPECT_GT(bound.port, 0);
    EXPECT_EQ(bound.ip_string(), "127.0.0.1");
    const int cfd = tcp_connect(bound, 2000);
    ASSERT_GE(cfd, 0);
    EndPoint remote, local;
    ASSERT_EQ(get_remote_side(cfd, &remote), 0);
    ASSERT_EQ(get_local_side(cfd, &local), 0);
    EXPECT_TRUE(remote == bound);
    EXPECT_EQ(local.ip_string(), "127.0.0.1");
    close(cfd);
    close(lfd);
}

TEST(EndPointDepth, sockaddr_conversion_through_ipv6_sockets) {
    EndPoint any;
    ASSERT_EQ(str2endpoint("[::1]:0", &any), 0);
    const int lfd = tcp_listen(any);
    if (lfd < 0) return;  // host without an IPv6 loopback
    EndPoint bound;
    ASSERT_EQ(get_local_side(lfd, &bound), 0);
    EXPECT_TRUE(bound.is_ipv6());
    EXPECT_GT(bound.port, 0);
    const int cfd = tcp_connect(bound, 2000);
    ASSERT_GE(cfd, 0);
    EndPoint remote;
    ASSERT_EQ(get_remote_side(cfd, &remote), 0);
    EXPECT_TRUE(remote == bound);
    EXPECT_EQ(remote.to_string(), "[::1]:" + std::to_string(bound.port));
    close(cfd);
    close(lfd);
}

TEST(EndPointDepth, sockaddr_conversion_through_unix_sockets) {
    const std::string path = "/tmp/mrpc_ep_" + std::to_string(getpid()) + ".sock";
    unlink(path.c_str());
    EndPoint ep;
    ASSERT_EQ(str2endpoint(("unix:" + path).c_str(), &ep), 0);
    const int lfd = tcp_listen(ep);
    ASSERT_GE(lfd, 0);
    const int cfd = tcp_connect(ep, 2000);
    ASSERT_GE(cfd, 0);
    EndPoint remote;
    ASSERT_EQ(get_remote_side(cfd, &remote), 0);
    EXPECT_TRUE(remote.is_unix());
    EXPECT_EQ(remote.path, path);
    close(cfd);
    close(lfd);
    unlink(path.c_str());
}

TEST(EndPointDepth, hostnames_resolve) {
    EndPoint ep;
    ASSERT_EQ(hostname2endpoint("localhost:1234", &ep), 0);
    EXPECT_EQ(ep.port, 1234);
    EXPECT_TRUE(ep.ip_string() == "127.0.0.1" || ep.is_ipv6());
    EXPECT_NE(hostname2endpoint("no-such-host.invalid:80", &ep), 0);
    EXPECT_FALSE(my_hostname().empty());
}

TEST(EndPointDepth, concurrent_parsing_and_printing) {
    std::atomic<int> bad{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < 8; ++t) {
        ts.emplace_back([t, &bad] {
            for (int i = 0; i < 2000; ++i) {
                const int port = 1 + (t * 2000 + i) % 65000;
                const std::string v4 = "10." + std::to_string(t) + ".0." + std::to_string(i % 250) + ":" +
                                       std::to_string(port);
                const std::string v6 = "[2001:db8::" + std::to_string(t + 1) + "]:" + std::to_string(port);
                EndPoint a, b;
                if (str2endpoint(v4.c_str(), &a) != 0 || a.to_string() != v4) bad.fetch_add(1);
                if (str2endpoint(v6.c_str(), &b) != 0 || b.to_string() != v6) bad.fetch_add(1);
            }
        });
    }
    for (auto& th : ts) th.join();
    EXPECT_EQ(bad.load(), 0);
}
