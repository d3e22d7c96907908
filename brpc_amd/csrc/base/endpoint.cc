#include "base/endpoint.h"

#include <arpa/inet.h>
#include <fcntl.h>
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

std::string EndPoint::ip_string() const { return is_unix() ? std::string("unix") : ip2str(ip); }

std::string EndPoint::to_string() const {
    if (is_unix()) return "unix:" + path;
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
    const char* colon = strrchr(str, ':');
    if (!colon) return -1;
    std::string host(str, colon - str);
    char* end = nullptr;
    long port = strtol(colon + 1, &end, 10);
    if (end == colon + 1 || (*end && *end != ' ') || port < 0 || port > 65535) return -1;
    uint32_t ip;
    if (str2ip(host.c_str(), &ip) != 0) return -1;
    ep->ip = ip;
    ep->port = (int)port;
    ep->path.clear();
    return 0;
}

int str2endpoint(const char* ip_str, int port, EndPoint* ep) {
    uint32_t ip;
    if (str2ip(ip_str, &ip) != 0) return -1;
    if (port < 0 || port > 65535) return -1;
    ep->ip = ip;
    ep->port = port;
    ep->path.clear();
    return 0;
}

int hostname2endpoint(const char* host_and_port, EndPoint* ep) {
    if (str2endpoint(host_and_port, ep) == 0) return 0;
    const char* colon = strrchr(host_and_port, ':');
    std::string host = colon ? std::string(host_and_port, colon - host_and_port) : std::string(host_and_port);
    int port = colon ? atoi(colon + 1) : 80;
    addrinfo hints;
    memset(&hints, 0, sizeof(hints));
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    addrinfo* res = nullptr;
    if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res) return -1;
    ep->ip = ((sockaddr_in*)res->ai_addr)->sin_addr.s_addr;
    ep->port = port;
    ep->path.clear();
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

int tcp_listen(const EndPoint& ep, bool reuse_port, int backlog) {
    int fd = socket(ep.is_unix() ? AF_UNIX : AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
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
    int fd = socket(ep.is_unix() ? AF_UNIX : AF_INET, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
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
