// Acceptor: listening socket + per-connection sockets driven by the
// InputMessenger, idle-connection reaping (role of src/brpc/acceptor.cpp:50-286).
#pragma once

#include <mutex>
#include <set>
#include <vector>

#include "net/input_messenger.h"

namespace mrpc {

class Acceptor : public InputMessenger {
public:
    Acceptor();
    ~Acceptor();
    // Takes ownership of listened_fd. idle_timeout_sec <= 0 disables reaping.
    int StartAccept(int listened_fd, int idle_timeout_sec);
    // Stop accepting and close all connections.
    void StopAccept(int closewait_ms);
    void Join();
    size_t ConnectionCount() const;
    void ListConnections(std::vector<SocketId>* out) const;
    bool accepting() const { return _listened_sid != INVALID_SOCKET_ID; }
    // Accepted connections detect TLS on their first bytes.
    void set_ssl_ctx(std::shared_ptr<SslContext> ctx) { _ssl_ctx = std::move(ctx); }
    // Accepted connections detect an RDMA hello on their first bytes.
    void set_rdma(bool on) { _rdma = on; }

private:
    static void OnNewConnections(Socket* listened);
    static void* CloseIdleConnections(void* arg);
    SocketId _listened_sid;
    int _idle_timeout_sec;
    mutable std::mutex _mu;
    std::set<SocketId> _conns;
    std::set<SocketId> _closing;
    fiber::fiber_t _idle_tid;
    std::atomic<bool> _stop;
    std::shared_ptr<SslContext> _ssl_ctx;
    bool _rdma = false;
};

}  // namespace mrpc
