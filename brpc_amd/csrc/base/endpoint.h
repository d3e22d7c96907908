// EndPoint and TCP helpers (role of butil/endpoint.h:87-138).
// Supports IPv4 endpoints and unix-domain-socket endpoints ("unix:/path").
#pragma once

#include <netinet/in.h>

#include <cstdint>
#include <functional>
#include <ostream>
#include <string>

namespace mrpc {

struct EndPoint {
    uint32_t ip;      // network byte order, 0 for unix sockets
    int port;         // host order; -1 for unix sockets
    std::string path;  // unix socket path (empty for tcp)

    EndPoint() : ip(0), port(0) {}
    EndPoint(uint32_t ip_, int port_) : ip(ip_), port(port_) {}
    bool is_unix() const { return !path.empty(); }
    bool operator==(const EndPoint& o) const { return ip == o.ip && port == o.port && path == o.path; }
    bool operator!=(const EndPoint& o) const { return !(*this == o); }
    bool operator<(const EndPoint& o) const {
        if (ip != o.ip) return ip < o.ip;
        if (port != o.port) return port < o.port;
        return path < o.path;
    }
    std::string to_string() const;
    std::string ip_string() const;
};

std::ostream& operator<<(std::ostream& os, const EndPoint& ep);

// "1.2.3.4:80", "localhost:80", "unix:/tmp/x.sock", "0.0.0.0:80".
int str2endpoint(const char* str, EndPoint* ep);
int str2endpoint(const char* ip_str, int port, EndPoint* ep);
int hostname2endpoint(const char* host_and_port, EndPoint* ep);
int str2ip(const char* s, uint32_t* ip);
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
        return std::hash<uint64_t>()(((uint64_t)e.ip << 32) | (uint32_t)e.port) ^ std::hash<std::string>()(e.path);
    }
};

}  // namespace mrpc
