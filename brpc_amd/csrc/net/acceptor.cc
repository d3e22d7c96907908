#include "net/acceptor.h"

#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>

#include "base/logging.h"
#include "base/time.h"
#include "rpc/errno.h"

namespace mrpc {

Acceptor::Acceptor() : _listened_sid(INVALID_SOCKET_ID), _idle_timeout_sec(-1), _idle_tid(0), _stop(false) {}

Acceptor::~Acceptor() {
    StopAccept(0);
    Join();
}

int Acceptor::StartAccept(int listened_fd, int idle_timeout_sec) {
    if (listened_fd < 0) return -1;
    _idle_timeout_sec = idle_timeout_sec;
    _stop = false;
    SocketOptions opt;
    opt.fd = listened_fd;
    opt.user = this;
    opt.on_edge_triggered_events = OnNewConnections;
    if (Socket::Create(opt, &_listened_sid) != 0) {
        LOG(ERROR) << "Fail to create listening socket";
        return -1;
    }
    if (idle_timeout_sec > 0) {
        fiber::start_background(&_idle_tid, &fiber::ATTR_NORMAL, CloseIdleConnections, this);
    }
    // Connections may have been queued before the consumer was added.
    Socket::StartInputEvent(_listened_sid, 0);
    return 0;
}

void Acceptor::OnNewConnections(Socket* listened) {
    Acceptor* am = static_cast<Acceptor*>(listened->user());
    int progress = Socket::PROGRESS_INIT;
    for (;;) {
        sockaddr_storage ss;
        socklen_t len = sizeof(ss);
        int fd = ::accept4(listened->fd(), (sockaddr*)&ss, &len, SOCK_NONBLOCK | SOCK_CLOEXEC);
        if (fd < 0) {
            if (errno == EAGAIN || errno == EWOULDBLOCK) {
                if (listened->MoreReadEvents(&progress)) continue;
                return;
            }
            if (errno == EINTR || errno == ECONNABORTED) continue;
            if (errno == EMFILE || errno == ENFILE) {
                PLOG(ERROR) << "accept: too many open files";
                return;
            }
            if (listened->Failed()) return;
            PLOG(ERROR) << "accept";
            return;
        }
        SocketOptions opt;
        opt.fd = fd;
        opt.ssl_ctx = am->_ssl_ctx;
        if (am->_rdma) opt.rdma = SocketOptions::RDMA_SERVER;
        get_remote_side(fd, &opt.remote_side);
        SocketId sid;
        if (am->Create(opt, &sid) != 0) {
            LOG(ERROR) << "Fail to create socket for accepted fd=" << fd;
            ::close(fd);
            continue;
        }
        {
            std::lock_guard<std::mutex> g(am->_mu);
            if (am->_stop) {
                Socket::SetFailed(sid);
                continue;
            }
            am->_conns.insert(sid);
        }
    }
}

void* Acceptor::CloseIdleConnections(void* arg) {
    Acceptor* am = static_cast<Acceptor*>(arg);
    while (!am->_stop) {
        fiber::usleep(1000000);
        const int64_t now = monotonic_us();
        std::vector<SocketId> conns;
        am->ListConnections(&conns);
        for (SocketId sid : conns) {
            SocketUniquePtr s;
            if (Socket::Address(sid, &s) != 0) continue;
            if (now - s->last_active_us() > (int64_t)am->_idle_timeout_sec * 1000000) {
                s->SetFailed(EUNUSED, "close idle connection from %s", s->remote_side().to_string().c_str());
            }
        }
    }
    return nullptr;
}

void Acceptor::StopAccept(int closewait_ms) {
    if (_listened_sid == INVALID_SOCKET_ID) return;
    _stop = true;
    const SocketId listened = _listened_sid;
    Socket::SetFailed(_listened_sid);
    _listened_sid = INVALID_SOCKET_ID;
    if (closewait_ms > 0) fiber::usleep((uint64_t)closewait_ms * 1000);
    std::set<SocketId> conns;
    {
        std::lock_guard<std::mutex> g(_mu);
        conns.swap(_conns);
        _closing.insert(conns.begin(), conns.end());
        _closing.insert(listened);
    }
    for (SocketId sid : conns) Socket::SetFailed(sid);
}

void Acceptor::Join() {
    if (_idle_tid) {
        fiber::join(_idle_tid);
        _idle_tid = 0;
    }
    // Wait until every connection (and the listener) is recycled: reader
    // fibers still running on them use this messenger.
    std::set<SocketId> closing;
    {
        std::lock_guard<std::mutex> g(_mu);
        closing.swap(_closing);
    }
    for (SocketId sid : closing) {
        for (int i = 0; i < 10000; ++i) {
            SocketUniquePtr p;
            if (Socket::AddressFailedAsWell(sid, &p) < 0) break;
            p.reset();
            fiber::usleep(1000);
        }
    }
}

size_t Acceptor::ConnectionCount() const {
    std::vector<SocketId> v;
    ListConnections(&v);
    return v.size();
}

void Acceptor::ListConnections(std::vector<SocketId>* out) const {
    out->clear();
    std::lock_guard<std::mutex> g(_mu);
    auto& conns = const_cast<std::set<SocketId>&>(_conns);
    for (auto it = conns.begin(); it != conns.end();) {
        SocketUniquePtr s;
        if (Socket::Address(*it, &s) != 0) {
            it = conns.erase(it);
            continue;
        }
        out->push_back(*it);
        ++it;
    }
}

}  // namespace mrpc
