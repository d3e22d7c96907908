#include "http/http_client.h"

#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>

#include "base/endpoint.h"
#include "base/time.h"
#include "base/util.h"
#include "fiber/fiber.h"
#include "http/http_header.h"

namespace mrpc {

static int wait_fd(int fd, unsigned ev, int64_t deadline_us) {
    int64_t left = deadline_us - realtime_us();
    if (left <= 0) {
        errno = ETIMEDOUT;
        return -1;
    }
    timespec ts = realtime_after_us(left);
    return fiber::fd_timedwait(fd, ev, &ts);
}

int HttpFetch(const std::string& method, const std::string& url, const std::string& req_body,
              HttpSimpleResponse* resp, int timeout_ms) {
    URI uri;
    uri.SetHttpURL(url);
    std::string host = uri.host();
    int port = uri.port() > 0 ? uri.port() : 80;
    EndPoint ep;
    if (str2endpoint(host.c_str(), port, &ep) != 0 &&
        hostname2endpoint((host + ":" + std::to_string(port)).c_str(), &ep) != 0) {
        return -1;
    }
    const int64_t deadline = realtime_us() + (int64_t)timeout_ms * 1000;
    bool in_progress = false;
    int fd = tcp_connect_nonblocking(ep, &in_progress);
    if (fd < 0) return -1;
    struct Closer {
        int fd;
        ~Closer() { fiber::close_fd(fd); }
    } closer{fd};
    if (in_progress) {
        if (wait_fd(fd, EPOLLOUT, deadline) != 0) return -1;
        int err = 0;
        socklen_t len = sizeof(err);
        getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &len);
        if (err) return -1;
    }
    std::string path = uri.path().empty() ? "/" : uri.path();
    const std::string q = uri.query_string();
    if (!q.empty()) path += "?" + q;
    std::string req = method + " " + path + " HTTP/1.1\r\nHost: " + host + "\r\nConnection: close\r\nUser-Agent: mrpc\r\n";
    if (!req_body.empty() || method == "POST" || method == "PUT") req += "Content-Length: " + std::to_string(req_body.size()) + "\r\n";
    req += "\r\n" + req_body;
    size_t off = 0;
    while (off < req.size()) {
        ssize_t n = ::write(fd, req.data() + off, req.size() - off);
        if (n > 0) {
            off += n;
        } else if (n < 0 && (errno == EAGAIN || errno == EINTR)) {
            if (wait_fd(fd, EPOLLOUT, deadline) != 0) return -1;
        } else {
            return -1;
        }
    }
    std::string data;
    char buf[16384];
    for (;;) {
        ssize_t n = ::read(fd, buf, sizeof(buf));
        if (n > 0) {
            data.append(buf, n);
        } else if (n == 0) {
            break;
        } else if (errno == EAGAIN || errno == EINTR) {
            if (wait_fd(fd, EPOLLIN, deadline) != 0) return -1;
        } else {
            return -1;
        }
    }
    size_t hend = data.find("\r\n\r\n");
    if (hend == std::string::npos) return -1;
    std::vector<std::string> lines = split_string(data.substr(0, hend), '\n');
    if (lines.empty()) return -1;
    std::vector<std::string> sl = split_string(trim(lines[0]), ' ');
    if (sl.size() < 2) return -1;
    resp->status = atoi(sl[1].c_str());
    bool chunked = false;
    for (size_t i = 1; i < lines.size(); ++i) {
        std::string l = trim(lines[i]);
        size_t c = l.find(':');
        if (c == std::string::npos) continue;
        std::string k = to_lower(trim(l.substr(0, c)));
        std::string v = trim(l.substr(c + 1));
        resp->headers[k] = v;
        if (k == "transfer-encoding" && to_lower(v).find("chunked") != std::string::npos) chunked = true;
    }
    std::string body = data.substr(hend + 4);
    if (chunked) {
        std::string out;
        size_t p = 0;
        for (;;) {
            size_t le = body.find("\r\n", p);
            if (le == std::string::npos) break;
            size_t len = strtoul(body.substr(p, le - p).c_str(), nullptr, 16);
            if (len == 0) break;
            out += body.substr(le + 2, len);
            p = le + 2 + len + 2;
        }
        body.swap(out);
    }
    resp->body.swap(body);
    return (resp->status >= 200 && resp->status < 300) ? 0 : -1;
}

int HttpGet(const std::string& url, std::string* body, int timeout_ms) {
    HttpSimpleResponse r;
    int rc = HttpFetch("GET", url, "", &r, timeout_ms);
    if (body) body->swap(r.body);
    return rc;
}

}  // namespace mrpc
