// Socket: a connection addressed by a versioned 64-bit SocketId (weak
// reference semantics) with a wait-free MPSC write queue and edge-triggered
// read dispatch. Design parity with the reference's Socket
// (src/brpc/socket.cpp:596 Create, 1511-1850 Write/StartWrite/KeepWrite/
// DoWrite, 2047 StartInputEvent, 863-940 SetFailed/health-check revive;
// docs/en/io.md):
//  * Write() exchanges the request into _write_head; the first writer writes
//    in place, later writers return immediately and a KeepWrite fiber
//    drains the queue batching up to 256 requests per writev.
//  * one reader fiber per fd at a time via the _nevent counter.
//  * SetFailed() bumps the version so Address() fails; with health checking
//    the id is revived in place when the peer comes back (LBs keep ids).
// MI355X-native: a Socket can carry a Transport (e.g. the xGMI device
// payload endpoint in gpu/xgmi_transport.h) that moves HBM-resident payload
// segments outside the TCP byte stream.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <deque>
#include <mutex>
#include <vector>
#include <string>

#include "base/buf.h"
#include "base/endpoint.h"
#include "fiber/call_id.h"
#include "fiber/fiber.h"
#include "net/ssl.h"

namespace mrpc {
namespace rdma {
class Endpoint;
}

typedef uint64_t SocketId;
const SocketId INVALID_SOCKET_ID = (SocketId)-1;

class Socket;
class InputMessageBase;

// Releases one reference of a Socket on destruction.
class SocketUniquePtr {
public:
    SocketUniquePtr() : _s(nullptr) {}
    explicit SocketUniquePtr(Socket* s) : _s(s) {}
    SocketUniquePtr(SocketUniquePtr&& o) noexcept : _s(o._s) { o._s = nullptr; }
    SocketUniquePtr& operator=(SocketUniquePtr&& o) noexcept;
    ~SocketUniquePtr() { reset(); }
    SocketUniquePtr(const SocketUniquePtr&) = delete;
    SocketUniquePtr& operator=(const SocketUniquePtr&) = delete;
    Socket* get() const { return _s; }
    Socket* operator->() const { return _s; }
    Socket& operator*() const { return *_s; }
    explicit operator bool() const { return _s != nullptr; }
    void reset(Socket* s = nullptr);
    Socket* release() {
        Socket* s = _s;
        _s = nullptr;
        return s;
    }

private:
    Socket* _s;
};

// Base of per-connection protocol state kept on a Socket. The type tag
// lets a protocol's parse() tell its own context from another protocol's.
class ParsingContext {
public:
    virtual ~ParsingContext() {}
    virtual int protocol_tag() const = 0;
};

// Hook for non-fd connections (streams multiplexed on a host socket).
class SocketConnection {
public:
    virtual ~SocketConnection() {}
    virtual int Connect(Socket* s, const timespec* abstime) = 0;
    virtual ssize_t CutMessageIntoFileDescriptor(int fd, Buf** data_list, size_t size) = 0;
};

// Optional secondary data plane attached to a socket (xGMI, RDMA).
class Transport {
public:
    virtual ~Transport() {}
    virtual const char* name() const = 0;
    virtual void OnSocketFailed(Socket* s) {}
};

struct SocketOptions {
    int fd = -1;
    EndPoint remote_side;
    void* user = nullptr;  // owner (e.g. Server/Acceptor); not owned
    // Called in a fiber whenever the fd becomes readable (edge triggered).
    void (*on_edge_triggered_events)(Socket*) = nullptr;
    int health_check_interval_s = -1;
    std::shared_ptr<SocketConnection> conn;
    bool connect_lazily = false;  // fd < 0: connect to remote_side on first write
    // TLS: a server context makes the socket detect TLS on its first bytes;
    // a client context makes it start a TLS session after connecting.
    std::shared_ptr<SslContext> ssl_ctx;
    std::string ssl_sni;
    // RDMA (rdma/rdma.h): RDMA_CLIENT exchanges hellos right after connect
    // and then moves every byte over verbs; RDMA_SERVER detects the hello on
    // the first bytes of an accepted connection (plain TCP clients still work).
    enum { RDMA_NONE = 0, RDMA_CLIENT = 1, RDMA_SERVER = 2 };
    int rdma = RDMA_NONE;
};

struct WriteOptions {
    fiber::CallId id_wait = fiber::INVALID_CALL_ID;  // error this id if the write fails
    int abstime_ms = 0;
    bool ignore_eovercrowded = false;
    bool write_in_background = false;
    // Half-close (shutdown SHUT_WR) once this write is fully on the wire.
    bool shutdown_write_after = false;
    // >0: the protocol answers requests in order without correlation ids
    // (http/1.1, redis, memcache). The socket remembers (count, id_wait) in
    // write order so the parser can map the next response(s) to the call.
    int pipelined_count = 0;
    // protocol-private tag carried with the pipelined entry (e.g. HEAD)
    uint32_t pipelined_tag = 0;
    int pipelined_protocol = 0;  // ProtocolType of the request (parsers claim only their own)
    // The write carries the connection's credentials in front of the
    // request (redis AUTH/SELECT): the parser first consumes this many
    // replies; `auth_winner` ends this socket's authentication fight once
    // the write is queued (FightAuthentication losers wait for that).
    int auth_replies = 0;
    bool auth_winner = false;
};

struct PipelinedInfo {
    int count = 0;
    int auth_replies = 0;  // replies to credentials sent in front of the request
    uint32_t tag = 0;
    int protocol = 0;
    fiber::CallId id_wait = fiber::INVALID_CALL_ID;
};

class Socket {
public:
    static const int PROGRESS_INIT = 1;

    static int Create(const SocketOptions& opt, SocketId* id);
    // 0 and a new reference on success, -1 if the socket is failed/recycled.
    static int Address(SocketId id, SocketUniquePtr* ptr);
    static int AddressFailedAsWell(SocketId id, SocketUniquePtr* ptr);
    // SetFailed on an id (no-op if already failed).
    static int SetFailed(SocketId id);
    static void StartInputEvent(SocketId id, uint32_t events);
    static void HandleEpollOut(SocketId id);

    int SetFailed(int error_code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
    int SetFailed();
    bool Failed() const;
    int error_code() const { return _error_code.load(std::memory_order_relaxed); }
    std::string error_text() const;
    // Ask the socket to be recycled once no one references it (for sockets
    // created with health checking; see ReleaseAdditionalReference in ref).
    int ReleaseAdditionalReference();

    // Write. On success the data is taken (data is cleared).
    int Write(Buf* data, const WriteOptions* opt = nullptr);

    SocketId id() const { return _this_id; }
    int fd() const { return _fd.load(std::memory_order_acquire); }
    const EndPoint& remote_side() const { return _remote_side; }
    const EndPoint& local_side() const { return _local_side; }
    void* user() const { return _user; }
    int64_t last_active_us() const { return _last_active_us.load(std::memory_order_relaxed); }
    int64_t unwritten_bytes() const { return _unwritten_bytes.load(std::memory_order_relaxed); }
    uint32_t nref() const { return (uint32_t)_versioned_ref.load(std::memory_order_relaxed); }

    // read side
    ssize_t DoRead(size_t size_hint);
    bool MoreReadEvents(int* progress);
    BufPortal _read_buf;
    int _preferred_index = -1;          // protocol index that parsed the last message
    // Protocol private per-connection state (http parser, h2 context, ...).
    ParsingContext* parsing_context() const { return _parsing_context.load(std::memory_order_acquire); }
    void reset_parsing_context(ParsingContext* ctx);
    // Install ctx if none is set yet; false (ctx untouched) if another won.
    bool InstallParsingContext(ParsingContext* ctx);
    std::atomic<ParsingContext*> _parsing_context{nullptr};
    int64_t _avg_msg_size = 0;
    std::atomic<bool> _server_verified{false};  // server-side authentication done

    // Connection pool (client side)
    int GetPooledSocket(SocketUniquePtr* out);
    void ReturnToPool();
    int GetShortSocket(SocketUniquePtr* out);
    bool is_pooled() const { return _main_socket_id != INVALID_SOCKET_ID; }
    SocketId main_socket_id() const { return _main_socket_id; }

    // Authentication: the first writer on a socket sends credentials.
    bool FightAuthentication(int* auth_error);
    void SetAuthentication(int error);
    // The winner could not send its credentials: let the next writer fight.
    void ResetAuthentication();
    int auth_error() const { return _auth_error.load(); }

    // Pipelined protocols: peek/pop the entry of the oldest outstanding write.
    bool PopPipelinedInfo(PipelinedInfo* out);
    bool PeekPipelinedInfo(PipelinedInfo* out);
    // Give back one response slot of a multi-response entry (redis batch).
    void GivebackPipelinedInfo(const PipelinedInfo& pi);

    // Per-socket attached objects
    std::shared_ptr<Transport> transport() const;
    void set_transport(std::shared_ptr<Transport> t);
    // The peer's rank in this process's RCCL payload plane (gpu/rccl_plane.h):
    // kPlaneUnknown until the hello round trip, -1 when the peer is not a
    // rank of our plane.
    static const int kPlaneUnknown = -2;
    int plane_rank() const { return _plane_rank.load(std::memory_order_acquire); }
    void set_plane_rank(int r) { _plane_rank.store(r, std::memory_order_release); }
    // Device-transport negotiation of a client connection: the first
    // request carrying device payloads also carries the hellos (xGMI arena,
    // RCCL plane rank); the others wait for its answer (at most timeout_us)
    // so their payloads take the negotiated transport instead of being
    // staged inline — N large payloads staged at once overcrowd the socket.
    // Returns true for the request that negotiates.
    bool FightDeviceHello(int64_t timeout_us);
    void DeviceHelloAnswered();  // a response carried (or could have carried) the hellos
    void DeviceHelloAbandoned(); // the negotiating request never went out
    std::shared_ptr<SocketConnection> conn() const { return _conn; }
    // TLS state (nullptr when the connection is plaintext).
    std::shared_ptr<SslSession> ssl_session() const;
    bool is_ssl() const { return _ssl_state.load(std::memory_order_acquire) == SSL_ON; }
    // RDMA data plane (nullptr when the connection is plain TCP).
    bool is_rdma() const { return _rdma_state.load(std::memory_order_acquire) == RDMA_ON; }
    rdma::Endpoint* rdma_endpoint() const { return _rdma_ep_raw.load(std::memory_order_acquire); }

    // Callbacks run once when the socket fails (streams multiplexed on it).
    void AddFailureCallback(std::function<void()> cb);

    // Health-check / revive
    int Revive(int new_fd);
    int health_check_interval() const { return _health_check_interval_s; }
    int64_t ninflight_health_check = 0;

    // stats
    std::atomic<int64_t> in_bytes{0}, out_bytes{0}, in_messages{0}, out_messages{0};
    std::string description() const;

    static int64_t nsocket();

    // internals -----------------------------------------------------
    Socket();
    ~Socket();
    void AddRef() { _versioned_ref.fetch_add(1, std::memory_order_relaxed); }
    int Dereference();

    struct WriteRequest;

private:
    friend class SocketUniquePtr;
    int ResetFileDescriptor(int fd);
    int ConnectIfNot(const timespec* abstime, WriteRequest* req);
    int StartWrite(WriteRequest* req, const WriteOptions& opt);
    static void* KeepWrite(void* arg);
    ssize_t DoWrite(WriteRequest* req);
    bool IsWriteComplete(WriteRequest* old_head, bool singular_node, WriteRequest** new_tail);
    void ReturnFailedWriteRequest(WriteRequest* req, int error_code, const std::string& error_text);
    void ReleaseAllFailedWriteRequests(WriteRequest* req);
    int WaitEpollOut(int fd, bool pollin, const timespec* abstime);
    void OnRecycle();
    static void* ProcessEvent(void* arg);
    static void* HealthCheckThread(void* arg);
    void StartHealthCheck();

    std::atomic<uint64_t> _versioned_ref;
    SocketId _this_id;
    std::atomic<int> _fd;
    EndPoint _remote_side;
    EndPoint _local_side;
    void* _user;
    void (*_on_edge_triggered_events)(Socket*);
    std::shared_ptr<SocketConnection> _conn;
    int _health_check_interval_s;
    bool _connect_lazily;
    std::atomic<int> _nevent;
    std::atomic<WriteRequest*> _write_head;
    std::atomic<int64_t> _unwritten_bytes;
    std::atomic<int>* _epollout_butex;
    std::atomic<int64_t> _last_active_us;
    // set after the version bump that marks the socket failed: a reader that
    // sees Failed() before it lands falls back to EFAILEDSOCKET
    std::atomic<int> _error_code;
    std::string _error_text;
    mutable std::mutex _mu;  // protects transport, error text, pool
    std::shared_ptr<Transport> _transport;
    std::atomic<int> _auth_error;
    std::atomic<int> _auth_state;  // 0 none, 1 fighting, 2 done
    std::atomic<int> _plane_rank;
    std::atomic<int> _dev_hello{0};  // 0 not started, 1 in flight, 2 answered
    std::atomic<int>* _dev_hello_butex = nullptr;
    std::atomic<int>* _auth_butex;
    // pooled connections: the main socket keeps a free list of sub sockets
    SocketId _main_socket_id;
    struct SharedPart;
    std::shared_ptr<SharedPart> _shared;
    std::atomic<bool> _recycle_flag;
    std::mutex _pipeline_mu;
    std::deque<PipelinedInfo> _pipeline_q;
    std::atomic<bool> _hc_started;
    // TLS
    enum { SSL_OFF = 0, SSL_UNKNOWN = 1, SSL_ON = 2 };
    ssize_t SslRead(int fd, size_t size_hint);
    ssize_t WriteList(int fd, Buf** list, size_t n);
    std::shared_ptr<SslContext> _ssl_ctx;
    std::string _ssl_sni;
    std::shared_ptr<SslSession> _ssl;
    std::atomic<int> _ssl_state{SSL_OFF};
    // RDMA
    enum { RDMA_OFF = 0, RDMA_UNKNOWN = 1, RDMA_ON = 2 };
    ssize_t RdmaRead(int fd, size_t size_hint);
    void InstallRdmaEndpoint(std::shared_ptr<rdma::Endpoint> ep);
    int _rdma_mode = 0;
    std::atomic<int> _rdma_state{RDMA_OFF};
    std::shared_ptr<rdma::Endpoint> _rdma_ep;  // guarded by _mu
    std::atomic<rdma::Endpoint*> _rdma_ep_raw{nullptr};
};

// Dump /connections-style info of all live sockets.
std::string DescribeAllSockets();

}  // namespace mrpc
