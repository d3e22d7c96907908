#include "base/endpoint.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <net/if.h>
#include <netdb.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cerrno>
#include <cstdlib>
#include <cstring>

#include "base/logging.h"

namespace mrpc {

std::string ip2str(uint32_t ip) {
    char buf[INET_ADDRSTRLEN];
    in_addr a;
    a.s_addr = ip;
    inet_ntop(AF_INET, &a, buf, sizeof(buf));
    return buf;
}

int str2ip(const char* s, uint32_t* ip) {
    while (*s == ' ') ++s;
    in_addr a;
    if (inet_pton(AF_INET, s, &a) != 1) return -1;
    *ip = a.s_addr;
    return 0;
}

int str2ip6(const char* s, EndPoint* ep) {
    while (*s == ' ') ++s;
    std::string addr(s);
    uint32_t scope = 0;
    const size_t pct = addr.find('%');
    if (pct != std::string::npos) {
        const std::string zone = addr.substr(pct + 1);
        addr.resize(pct);
        char* end = nullptr;
        const unsigned long z = strtoul(zone.c_str(), &end, 10);
        scope = (end && *end == 0 && !zone.empty()) ? (uint32_t)z : if_nametoindex(zone.c_str());
        if (scope == 0) return -1;
    }
    in6_addr a;
    if (inet_pton(AF_INET6, addr.c_str(), &a) != 1) return -1;
    memcpy(ep->ip6, &a, 16);
    ep->v6 = true;
    ep->scope_id = scope;
    ep->ip = 0;
    return 0;
}

static std::string ip6str(const EndPoint& ep) {
    char buf[INET6_ADDRSTRLEN];
    inet_ntop(AF_INET6, ep.ip6, buf, sizeof(buf));
    std::string s = buf;
    if (ep.scope_id) {
        char name[IF_NAMESIZE];
        s += "%";
        s += if_indextoname(ep.scope_id, name) ? name : std::to_string(ep.scope_id).c_str();
    }
    return s;
}

std::string EndPoint::ip_string() const {
    if (is_unix()) return "unix";
    return v6 ? ip6str(*this) : ip2str(ip);
}

std::string EndPoint::to_string() const {
    if (is_unix()) return "unix:" + path;
    if (v6) return "[" + ip6str(*this) + "]:" + std::to_string(port);
    return ip2str(ip) + ":" + std::to_string(port);
}

std::ostream& operator<<(std::ostream& os, const EndPoint& ep) { return os << ep.to_string(); }

int str2endpoint(const char* str, EndPoint* ep) {
    if (strncmp(str, "unix:", 5) == 0) {
        ep->ip = 0;
        ep->port = -1;
        ep->path = str + 5;
        return ep->path.empty() ? -1 : 0;
    }
    while (*str == ' ') ++str;
    if (*str == '[') {  // "[v6addr]:port"
        const char* close = strchr(str, ']');
        if (!close || close[1] != ':') return -1;
        char* end = nullptr;
        const long port = strtol(close + 2, &end, 10);
        if (end == close + 2 || (*end && *end != ' ') || port < 0 || port > 65535) return -1;
        EndPoint e;
        if (str2ip6(std::string(str + 1, close - str - 1).c_str(), &e) != 0) return -1;
        e.port = (int)port;
        *ep = e;
        return 0;
    }
    const char* colon = strrchr(str, ':');
    if (!colon) return -1;
    std::string host(str, colon - str);
    if (host.find(':') != std::string::npos) return -1;  // bare IPv6 needs brackets
    char* end = nullptr;
    long port = strtol(colon + 1, &end, 10);
    if (end == colon + 1 || (*end && *end != ' ') || port < 0 || port > 65535) return -1;
    uint32_t ip;
    if (str2ip(host.c_str(), &ip) != 0) return -1;
    *ep = EndPoint(ip, (int)port);
    return 0;
}

int str2endpoint(const char* ip_str, int port, EndPoint* ep) {
    if (port < 0 || port > 65535) return -1;
    uint32_t ip;
    if (str2ip(ip_str, &ip) == 0) {
        *ep = EndPoint(ip, port);
        return 0;
    }
    std::string s(ip_str);
    if (!s.empty() && s.front() == '[' && s.back() == ']') s = s.substr(1, s.size() - 2);
    EndPoint e;
    if (str2ip6(s.c_str(), &e) != 0) return -1;
    e.port = port;
    *ep = e;
    return 0;
}

int hostname2endpoint(const char* host_and_port, EndPoint* ep) {
    if (str2endpoint(host_and_port, ep) == 0) return 0;
    const char* colon = strrchr(host_and_port, ':');
    std::string host = colon ? std::string(host_and_port, colon - host_and_port) : std::string(host_and_port);
    int port = 80;
    if (colon) {
        char* end = nullptr;
        const long p = strtol(colon + 1, &end, 10);
        if (end == colon + 1 || (*end && *end != ' ') || p < 0 || p > 65535) return -1;
        port = (int)p;
    }
    addrinfo hints;
    memset(&hints, 0, sizeof(hints));
    hints.ai_family = AF_UNSPEC;  // an A record first, else AAAA
    hints.ai_socktype = SOCK_STREAM;
    addrinfo* res = nullptr;
    if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res) return -1;
    const addrinfo* pick = res;
    for (const addrinfo* r = res; r; r = r->ai_next) {
        if (r->ai_family == AF_INET) {
            pick = r;
            break;
        }
    }
    EndPoint e;
    if (pick->ai_family == AF_INET) {
        e.ip = ((sockaddr_in*)pick->ai_addr)->sin_addr.s_addr;
    } else if (pick->ai_family == AF_INET6) {
        const sockaddr_in6* in6 = (const sockaddr_in6*)pick->ai_addr;
        e.v6 = true;
        memcpy(e.ip6, &in6->sin6_addr, 16);
        e.scope_id = in6->sin6_scope_id;
    } else {
        freeaddrinfo(res);
        return -1;
    }
    e.port = port;
    *ep = e;
    freeaddrinfo(res);
    return 0;
}

std::string my_hostname() {
    char buf[256];
    if (gethostname(buf, sizeof(buf)) != 0) return "localhost";
    buf[sizeof(buf) - 1] = 0;
    return buf;
}

uint32_t my_ip() {
    static uint32_t cached = [] {
        EndPoint ep;
        if (hostname2endpoint((my_hostname() + ":0").c_str(), &ep) == 0) return ep.ip;
        uint32_t ip = 0;
        str2ip("127.0.0.1", &ip);
        return ip;
    }();
    return cached;
}

static socklen_t fill_sockaddr(const EndPoint& ep, sockaddr_storage* ss) {
    memset(ss, 0, sizeof(*ss));
    if (ep.is_unix()) {
        sockaddr_un* un = (sockaddr_un*)ss;
        un->sun_family = AF_UNIX;
        strncpy(un->sun_path, ep.path.c_str(), sizeof(un->sun_path) - 1);
        return sizeof(sockaddr_un);
    }
    if (ep.v6) {
        sockaddr_in6* in6 = (sockaddr_in6*)ss;
        in6->sin6_family = AF_INET6;
        memcpy(&in6->sin6_addr, ep.ip6, 16);
        in6->sin6_port = htons((uint16_t)ep.port);
        in6->sin6_scope_id = ep.scope_id;
        return sizeof(sockaddr_in6);
    }
    sockaddr_in* in = (sockaddr_in*)ss;
    in->sin_family = AF_INET;
    in->sin_addr.s_addr = ep.ip;
    in->sin_port = htons((uint16_t)ep.port);
    return sizeof(sockaddr_in);
}

int make_non_blocking(int fd) {
    int fl = fcntl(fd, F_GETFL, 0);
    if (fl < 0) return fl;
    if (fl & O_NONBLOCK) return 0;
    return fcntl(fd, F_SETFL, fl | O_NONBLOCK);
}

int make_blocking(int fd) {
    int fl = fcntl(fd, F_GETFL, 0);
    if (fl < 0) return fl;
    if (!(fl & O_NONBLOCK)) return 0;
    return fcntl(fd, F_SETFL, fl & ~O_NONBLOCK);
}

int make_no_delay(int fd) {
    int one = 1;
    return setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

int make_close_on_exec(int fd) { return fcntl(fd, F_SETFD, FD_CLOEXEC); }

static int family_of(const EndPoint& ep) { return ep.is_unix() ? AF_UNIX : ep.v6 ? AF_INET6 : AF_INET; }

int tcp_listen(const EndPoint& ep, bool reuse_port, int backlog) {
    int fd = socket(family_of(ep), SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (fd < 0) return -1;
    if (!ep.is_unix()) {
        int one = 1;
        setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
        if (reuse_port) setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one));
    } else {
        unlink(ep.path.c_str());
    }
    sockaddr_storage ss;
    socklen_t len = fill_sockaddr(ep, &ss);
    if (bind(fd, (sockaddr*)&ss, len) != 0 || listen(fd, backlog) != 0) {
        int e = errno;
        close(fd);
        errno = e;
        return -1;
    }
    return fd;
}

int tcp_connect_nonblocking(const EndPoint& ep, bool* in_progress) {
    *in_progress = false;
    int fd = socket(family_of(ep), SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
    if (fd < 0) return -1;
    if (!ep.is_unix()) make_no_delay(fd);
    sockaddr_storage ss;
    socklen_t len = fill_sockaddr(ep, &ss);
    if (connect(fd, (sockaddr*)&ss, len) != 0) {
        if (errno == EINPROGRESS) {
            *in_progress = true;
            return fd;
        }
        int e = errno;
        close(fd);
        errno = e;
        return -1;
    }
    return fd;
}

int tcp_connect(const EndPoint& ep, int timeout_ms) {
    bool in_progress = false;
    int fd = tcp_connect_nonblocking(ep, &in_progress);
    if (fd < 0) return -1;
    if (in_progress) {
        pollfd p{fd, POLLOUT, 0};
        int rc = poll(&p, 1, timeout_ms);
        if (rc <= 0) {
            close(fd);
            errno = rc == 0 ? ETIMEDOUT : errno;
            return -1;
        }
        int err = 0;
        socklen_t el = sizeof(err);
        getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &el);
        if (err) {
            close(fd);
            errno = err;
            return -1;
        }
    }
    make_blocking(fd);
    return fd;
}

static int sockaddr2ep(const sockaddr_storage& ss, EndPoint* ep) {
    if (ss.ss_family == AF_INET) {
        const sockaddr_in* in = (const sockaddr_in*)&ss;
        ep->ip = in->sin_addr.s_addr;
        ep->port = ntohs(in->sin_port);
        ep->path.clear();
        return 0;
    }
    if (ss.ss_family == AF_INET6) {
        const sockaddr_in6* in6 = (const sockaddr_in6*)&ss;
        EndPoint e;
        e.v6 = true;
        memcpy(e.ip6, &in6->sin6_addr, 16);
        e.scope_id = in6->sin6_scope_id;
        e.port = ntohs(in6->sin6_port);
        *ep = e;
        return 0;
    }
    if (ss.ss_family == AF_UNIX) {
        const sockaddr_un* un = (const sockaddr_un*)&ss;
        ep->ip = 0;
        ep->port = -1;
        ep->path = un->sun_path[0] ? un->sun_path : "anonymous";
        return 0;
    }
    return -1;
}

int get_local_side(int fd, EndPoint* ep) {
    sockaddr_storage ss;
    socklen_t len = sizeof(ss);
    if (getsockname(fd, (sockaddr*)&ss, &len) != 0) return -1;
    return sockaddr2ep(ss, ep);
}

int get_remote_side(int fd, EndPoint* ep) {
    sockaddr_storage ss;
    socklen_t len = sizeof(ss);
    if (getpeername(fd, (sockaddr*)&ss, &len) != 0) return -1;
    return sockaddr2ep(ss, ep);
}

}  // namespace mrpc
