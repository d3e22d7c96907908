// EndPoint and TCP helpers (role of butil/endpoint.h:87-138 and the
// extended endpoints of butil/details/extended_endpoint.hpp:155-311).
// Supports IPv4 ("1.2.3.4:80"), IPv6 ("[::1]:80") and unix-domain-socket
// ("unix:/path") endpoints.
#pragma once

#include <netinet/in.h>

#include <cstdint>
#include <cstring>
#include <functional>
#include <ostream>
#include <string>

namespace mrpc {

struct EndPoint {
    uint32_t ip;      // IPv4, network byte order; 0 for IPv6 and unix sockets
    int port;         // host order; -1 for unix sockets
    std::string path;  // unix socket path (empty for tcp)
    bool v6 = false;   // an IPv6 endpoint: the address is ip6
    unsigned char ip6[16] = {};
    uint32_t scope_id = 0;  // IPv6 zone (link-local), 0 otherwise

    EndPoint() : ip(0), port(0) {}
    EndPoint(uint32_t ip_, int port_) : ip(ip_), port(port_) {}
    bool is_unix() const { return !path.empty(); }
    bool is_ipv6() const { return v6; }
    bool operator==(const EndPoint& o) const {
        return ip == o.ip && port == o.port && path == o.path && v6 == o.v6 && scope_id == o.scope_id &&
               memcmp(ip6, o.ip6, sizeof(ip6)) == 0;
    }
    bool operator!=(const EndPoint& o) const { return !(*this == o); }
    bool operator<(const EndPoint& o) const {
        if (v6 != o.v6) return v6 < o.v6;
        if (v6) {
            const int c = memcmp(ip6, o.ip6, sizeof(ip6));
            if (c) return c < 0;
            if (scope_id != o.scope_id) return scope_id < o.scope_id;
        }
        if (ip != o.ip) return ip < o.ip;
        if (port != o.port) return port < o.port;
        return path < o.path;
    }
    std::string to_string() const;
    std::string ip_string() const;
};

std::ostream& operator<<(std::ostream& os, const EndPoint& ep);

// "1.2.3.4:80", "localhost:80", "unix:/tmp/x.sock", "0.0.0.0:80",
// "[::1]:80", "[fe80::1%eth0]:80", "[::]:80".
int str2endpoint(const char* str, EndPoint* ep);
int str2endpoint(const char* ip_str, int port, EndPoint* ep);
int hostname2endpoint(const char* host_and_port, EndPoint* ep);
int str2ip(const char* s, uint32_t* ip);
// An IPv6 address (no brackets; "%zone" allowed) into ep's v6 fields.
int str2ip6(const char* s, EndPoint* ep);
std::string ip2str(uint32_t ip);
uint32_t my_ip();
std::string my_hostname();

// Sockets. All returned fds are non-blocking-capable normal fds (blocking
// mode as stated), with CLOEXEC.
int tcp_listen(const EndPoint& ep, bool reuse_port = false, int backlog = 1024);
// Non-blocking connect. Returns fd (connect may be in progress: *in_progress=true).
int tcp_connect_nonblocking(const EndPoint& ep, bool* in_progress);
// Blocking connect with timeout (ms, -1 = forever).
int tcp_connect(const EndPoint& ep, int timeout_ms = -1);
int get_local_side(int fd, EndPoint* ep);
int get_remote_side(int fd, EndPoint* ep);
int make_non_blocking(int fd);
int make_blocking(int fd);
int make_no_delay(int fd);
int make_close_on_exec(int fd);

struct EndPointHash {
    size_t operator()(const EndPoint& e) const {
        size_t h = std::hash<uint64_t>()(((uint64_t)e.ip << 32) | (uint32_t)e.port) ^ std::hash<std::string>()(e.path);
        if (e.v6) {
            uint64_t a, b;
            memcpy(&a, e.ip6, 8);
            memcpy(&b, e.ip6 + 8, 8);
            h ^= std::hash<uint64_t>()(a * 0x9E3779B97F4A7C15ull ^ b) + e.scope_id;
        }
        return h;
    }
};

}  // namespace mrpc
