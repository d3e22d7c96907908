#include "net/socket.h"
#include "rdma/rdma.h"

#include <fcntl.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstdarg>
#include <vector>

#include "base/flags.h"
#include "base/logging.h"
#include "base/pool.h"
#include "base/time.h"
#include "base/util.h"
#include "fiber/butex.h"
#include "http/http_client.h"
#include "net/event_dispatcher.h"
#include "rpc/errno.h"

DEFINE_int64(socket_max_unwritten_bytes, 64 * 1024 * 1024,
             "Max unwritten bytes in each socket; writes beyond fail with EOVERCROWDED");
DEFINE_int32(connect_timeout_ms_default, 200, "default timeout of lazily connecting sockets");
DEFINE_string(health_check_path, "",
              "HTTP path of the health check call: a failed socket whose server is connectable again is only "
              "revived once an HTTP GET of this path succeeds within -health_check_timeout_ms (empty: "
              "connectable is healthy)");
DEFINE_int32(health_check_timeout_ms, 500,
             "timeout of both the health check's connect and its HTTP call to -health_check_path");
DEFINE_int32(socket_recv_buffer_size, -1, "SO_RCVBUF of sockets if positive");
DEFINE_int32(socket_send_buffer_size, -1, "SO_SNDBUF of sockets if positive");
DEFINE_int32(max_connection_pool_size, 100, "max pooled connections to one endpoint");

namespace mrpc {

struct Socket::WriteRequest {
    Buf data;
    WriteRequest* next = nullptr;
    fiber::CallId id_wait = fiber::INVALID_CALL_ID;
    Socket* socket = nullptr;
    bool shutdown_after = false;  // half-close the connection once written
};

// A fully written request: honor WriteOptions.shutdown_write_after (the
// http server's "Connection: close"). Earlier requests were written before.
static void finish_write_request(Socket::WriteRequest* r, int fd) {
    if (r->shutdown_after && fd >= 0) ::shutdown(fd, SHUT_WR);
    return_object(r);
}

static Socket::WriteRequest* const UNCONNECTED = (Socket::WriteRequest*)(intptr_t)-1;

struct Socket::SharedPart {
    std::mutex mu;
    std::vector<SocketId> pool;  // free pooled sub-sockets
    std::vector<fiber::CallId> id_wait_list;
    size_t last_compact = 0;
    std::vector<std::function<void()>> failure_callbacks;
};

void Socket::AddFailureCallback(std::function<void()> cb) {
    std::shared_ptr<SharedPart> sp = _shared;
    if (Failed() || !sp) {
        cb();
        return;
    }
    std::lock_guard<std::mutex> g(sp->mu);
    sp->failure_callbacks.push_back(std::move(cb));
}

static std::atomic<int64_t> g_nsocket{0};

static inline uint64_t make_vref(uint32_t ver, uint32_t nref) { return ((uint64_t)ver << 32) | nref; }
static inline uint32_t vref_ver(uint64_t v) { return (uint32_t)(v >> 32); }
static inline int32_t vref_nref(uint64_t v) { return (int32_t)(uint32_t)v; }
static inline SocketId make_sid(uint32_t slot, uint32_t ver) { return ((uint64_t)slot << 32) | ver; }
static inline uint32_t sid_slot(SocketId id) { return (uint32_t)(id >> 32); }
static inline uint32_t sid_ver(SocketId id) { return (uint32_t)id; }

SocketUniquePtr& SocketUniquePtr::operator=(SocketUniquePtr&& o) noexcept {
    if (this != &o) {
        reset(o._s);
        o._s = nullptr;
    }
    return *this;
}

void SocketUniquePtr::reset(Socket* s) {
    Socket* old = _s;
    _s = s;
    if (old) old->Dereference();
}

Socket::Socket()
    : _versioned_ref(0),
      _this_id(INVALID_SOCKET_ID),
      _fd(-1),
      _user(nullptr),
      _on_edge_triggered_events(nullptr),
      _health_check_interval_s(-1),
      _connect_lazily(false),
      _nevent(0),
      _write_head(nullptr),
      _unwritten_bytes(0),
      _epollout_butex(fiber::butex_create()),
      _last_active_us(0),
      _error_code(0),
      _auth_error(0),
      _auth_state(0),
      _plane_rank(kPlaneUnknown),
      _dev_hello_butex(fiber::butex_create()),
      _auth_butex(fiber::butex_create()),
      _main_socket_id(INVALID_SOCKET_ID),
      _recycle_flag(false),
      _hc_started(false) {}

Socket::~Socket() {}

int64_t Socket::nsocket() { return g_nsocket.load(std::memory_order_relaxed); }

int Socket::ResetFileDescriptor(int fd) {
    _fd.store(fd, std::memory_order_release);
    if (fd < 0) return 0;
    make_non_blocking(fd);
    make_close_on_exec(fd);
    if (!_remote_side.is_unix()) make_no_delay(fd);
    if (FLAGS_socket_send_buffer_size > 0) {
        int v = FLAGS_socket_send_buffer_size;
        setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &v, sizeof(v));
    }
    if (FLAGS_socket_recv_buffer_size > 0) {
        int v = FLAGS_socket_recv_buffer_size;
        setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &v, sizeof(v));
    }
    get_local_side(fd, &_local_side);
    if (_on_edge_triggered_events) {
        if (GetGlobalEventDispatcher(fd).AddConsumer(_this_id, fd) != 0) {
            PLOG(ERROR) << "Fail to add consumer fd=" << fd;
            return -1;
        }
    }
    return 0;
}

int Socket::Create(const SocketOptions& opt, SocketId* id) {
    uint32_t slot;
    Socket* m = get_resource<Socket>(&slot);
    if (!m) return -1;
    const uint32_t ver = vref_ver(m->_versioned_ref.load(std::memory_order_relaxed));
    m->_this_id = make_sid(slot, ver);
    m->_remote_side = opt.remote_side;
    m->_local_side = EndPoint();
    m->_user = opt.user;
    m->_on_edge_triggered_events = opt.on_edge_triggered_events;
    m->_conn = opt.conn;
    m->_ssl_ctx = opt.ssl_ctx;
    m->_ssl_sni = opt.ssl_sni;
    {
        std::lock_guard<std::mutex> g(m->_mu);
        m->_ssl.reset();
    }
    m->_ssl_state.store(!opt.ssl_ctx ? SSL_OFF : (opt.ssl_ctx->is_server() ? SSL_UNKNOWN : SSL_ON));
    m->_rdma_mode = opt.rdma;
    m->InstallRdmaEndpoint(nullptr);
    m->_rdma_state.store(opt.rdma == SocketOptions::RDMA_SERVER && !opt.ssl_ctx ? RDMA_UNKNOWN : RDMA_OFF);
    m->_health_check_interval_s = opt.health_check_interval_s;
    m->_connect_lazily = opt.connect_lazily;
    m->_nevent.store(0, std::memory_order_relaxed);
    m->_write_head.store(nullptr, std::memory_order_relaxed);
    m->_unwritten_bytes.store(0, std::memory_order_relaxed);
    m->_last_active_us.store(monotonic_us(), std::memory_order_relaxed);
    m->_error_code.store(0, std::memory_order_relaxed);
    m->_error_text.clear();
    m->_preferred_index = -1;
    m->_parsing_context.store(nullptr, std::memory_order_relaxed);
    m->_avg_msg_size = 0;
    m->_server_verified.store(false);
    m->_auth_error.store(0);
    m->_auth_state.store(0);
    m->_plane_rank.store(kPlaneUnknown);
    m->_dev_hello.store(0);
    m->_main_socket_id = INVALID_SOCKET_ID;
    m->_shared = std::make_shared<SharedPart>();
    m->_recycle_flag.store(false);
    m->_hc_started.store(false);
    m->ninflight_health_check = 0;
    m->in_bytes = m->out_bytes = m->in_messages = m->out_messages = 0;
    {
        std::lock_guard<std::mutex> g(m->_mu);
        m->_transport.reset();
    }
    // One reference held until SetFailed().
    const SocketId sid = m->_this_id;  // once registered, the socket may fail and be reused before we return
    m->_versioned_ref.store(make_vref(ver, 1), std::memory_order_release);
    if (m->ResetFileDescriptor(opt.fd) != 0) {
        const int saved = errno;
        m->SetFailed(saved, "fail to register fd");
        return -1;
    }
    g_nsocket.fetch_add(1, std::memory_order_relaxed);
    *id = sid;
    return 0;
}

int Socket::Address(SocketId id, SocketUniquePtr* ptr) {
    Socket* m = address_resource<Socket>(sid_slot(id));
    if (!m) return -1;
    const uint64_t vref1 = m->_versioned_ref.fetch_add(1, std::memory_order_acquire);
    if (vref_ver(vref1) == sid_ver(id)) {
        ptr->reset(m);
        return 0;
    }
    const uint64_t vref2 = m->_versioned_ref.fetch_sub(1, std::memory_order_release);
    const int32_t nref = vref_nref(vref2);
    if (nref > 1) return -1;
    if (nref == 1) {
        const uint32_t ver2 = vref_ver(vref2);
        if (ver2 & 1) {
            uint64_t expected = vref2 - 1;
            if (m->_versioned_ref.compare_exchange_strong(expected, make_vref(ver2 + 1, 0), std::memory_order_acquire)) {
                m->OnRecycle();
                return_resource<Socket>(sid_slot(id));
            }
        }
    }
    return -1;
}

int Socket::AddressFailedAsWell(SocketId id, SocketUniquePtr* ptr) {
    Socket* m = address_resource<Socket>(sid_slot(id));
    if (!m) return -1;
    const uint64_t vref1 = m->_versioned_ref.fetch_add(1, std::memory_order_acquire);
    const uint32_t ver1 = vref_ver(vref1);
    if (ver1 == sid_ver(id) || ver1 == sid_ver(id) + 1) {
        ptr->reset(m);
        return ver1 == sid_ver(id) ? 0 : 1;
    }
    // Same undo path as Address(): the slot may be recycled or reused.
    const uint64_t vref2 = m->_versioned_ref.fetch_sub(1, std::memory_order_release);
    if (vref_nref(vref2) == 1) {
        const uint32_t ver2 = vref_ver(vref2);
        if (ver2 & 1) {
            uint64_t expected = vref2 - 1;
            if (m->_versioned_ref.compare_exchange_strong(expected, make_vref(ver2 + 1, 0), std::memory_order_acquire)) {
                m->OnRecycle();
                return_resource<Socket>(sid_slot(id));
            }
        }
    }
    return -1;
}

int Socket::Dereference() {
    const SocketId id = _this_id;
    const uint64_t vref = _versioned_ref.fetch_sub(1, std::memory_order_release);
    const int32_t nref = vref_nref(vref);
    if (nref > 1) return 0;
    if (nref == 1) {
        const uint32_t ver = vref_ver(vref);
        if (ver & 1) {
            uint64_t expected = vref - 1;
            if (_versioned_ref.compare_exchange_strong(expected, make_vref(ver + 1, 0), std::memory_order_acquire)) {
                OnRecycle();
                return_resource<Socket>(sid_slot(id));
                return 1;
            }
            return 0;
        }
        LOG(FATAL) << "Socket " << id << " dereferenced to 0 without SetFailed";
    }
    LOG(FATAL) << "Over dereferenced socket " << id;
    return -1;
}

bool Socket::Failed() const {
    return vref_ver(_versioned_ref.load(std::memory_order_acquire)) != sid_ver(_this_id);
}

std::string Socket::error_text() const {
    std::lock_guard<std::mutex> g(_mu);
    return _error_text;
}

int Socket::SetFailed(SocketId id) {
    SocketUniquePtr p;
    if (Address(id, &p) != 0) return -1;
    return p->SetFailed();
}

int Socket::SetFailed() { return SetFailed(EFAILEDSOCKET, "socket closed"); }

int Socket::SetFailed(int error_code, const char* fmt, ...) {
    if (error_code == 0) error_code = EFAILEDSOCKET;
    const uint32_t id_ver = sid_ver(_this_id);
    uint64_t vref = _versioned_ref.load(std::memory_order_relaxed);
    for (;;) {
        if (vref_ver(vref) != id_ver) return -1;
        if (_versioned_ref.compare_exchange_strong(vref, make_vref(id_ver + 1, vref_nref(vref)),
                                                   std::memory_order_release, std::memory_order_relaxed)) {
            break;
        }
    }
    std::string text;
    if (fmt) {
        va_list ap;
        va_start(ap, fmt);
        char buf[512];
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        text = buf;
    }
    std::shared_ptr<Transport> tr;
    {
        std::lock_guard<std::mutex> g(_mu);
        _error_code.store(error_code, std::memory_order_relaxed);
        _error_text = text.empty() ? ErrorText(error_code) : text;
        tr = _transport;
    }
    const int fd = _fd.load(std::memory_order_acquire);
    if (fd >= 0) {
        // Wake peers and our own pending reads; the fd is closed on recycle.
        if (_on_edge_triggered_events) GetGlobalEventDispatcher(fd).RemoveConsumer(fd);
        ::shutdown(fd, SHUT_RDWR);
    }
    _epollout_butex->fetch_add(1, std::memory_order_release);
    fiber::butex_wake_all(_epollout_butex);
    if (tr) tr->OnSocketFailed(this);
    if (rdma::Endpoint* ep = rdma_endpoint()) ep->Shutdown();
    // Fail every RPC waiting for a response on this socket.
    std::vector<fiber::CallId> ids;
    std::vector<std::function<void()>> cbs;
    {
        std::lock_guard<std::mutex> g(_shared->mu);
        ids.swap(_shared->id_wait_list);
        cbs.swap(_shared->failure_callbacks);
    }
    for (fiber::CallId cid : ids) fiber::call_id_error(cid, error_code, _error_text);
    for (auto& cb : cbs) cb();
    if (_health_check_interval_s > 0 && !_recycle_flag.load() && !_remote_side.path.size() && !is_pooled()) {
        StartHealthCheck();
    } else {
        Dereference();  // the creator's reference
    }
    return 0;
}

int Socket::ReleaseAdditionalReference() {
    if (_recycle_flag.exchange(true)) return -1;
    if (!Failed()) {
        // SetFailed sees the recycle flag and releases the creator reference.
        return SetFailed(EFAILEDSOCKET, "released");
    }
    // Failed with a health-check loop holding the creator ref: it exits and
    // releases it on its next iteration.
    return 0;
}

void Socket::OnRecycle() {
    const int fd = _fd.exchange(-1, std::memory_order_acq_rel);
    if (fd >= 0) {
        if (_on_edge_triggered_events) GetGlobalEventDispatcher(fd).RemoveConsumer(fd);
        ::close(fd);
    }
    _read_buf.clear();
    _read_buf.return_cached_blocks();
    delete _parsing_context.exchange(nullptr);
    {
        std::lock_guard<std::mutex> g(_pipeline_mu);
        _pipeline_q.clear();
    }
    {
        std::lock_guard<std::mutex> g(_mu);
        _transport.reset();
        _ssl.reset();
    }
    _conn.reset();
    _ssl_ctx.reset();
    InstallRdmaEndpoint(nullptr);
    _rdma_state.store(RDMA_OFF);
    // pooled sub sockets of a main socket are released with it
    if (_shared) {
        std::vector<SocketId> pool;
        {
            std::lock_guard<std::mutex> g(_shared->mu);
            pool.swap(_shared->pool);
        }
        for (SocketId sid : pool) {
            SocketUniquePtr p;
            if (Address(sid, &p) == 0) p->SetFailed(EUNUSED, "main socket recycled");
        }
    }
    _shared.reset();
    _user = nullptr;
    _on_edge_triggered_events = nullptr;
    g_nsocket.fetch_sub(1, std::memory_order_relaxed);
}

void Socket::reset_parsing_context(ParsingContext* ctx) { delete _parsing_context.exchange(ctx); }

bool Socket::InstallParsingContext(ParsingContext* ctx) {
    ParsingContext* expected = nullptr;
    return _parsing_context.compare_exchange_strong(expected, ctx, std::memory_order_acq_rel);
}

std::shared_ptr<Transport> Socket::transport() const {
    std::lock_guard<std::mutex> g(_mu);
    return _transport;
}

void Socket::set_transport(std::shared_ptr<Transport> t) {
    std::lock_guard<std::mutex> g(_mu);
    _transport = std::move(t);
}

// ---------------------------------------------------------------- read

void Socket::StartInputEvent(SocketId id, uint32_t events) {
    SocketUniquePtr s;
    if (Address(id, &s) < 0) return;
    if (s->_nevent.fetch_add(1, std::memory_order_acq_rel) == 0) {
        Socket* p = s.release();
        fiber::fiber_t tid;
        if (fiber::start_urgent(&tid, &fiber::ATTR_NORMAL, ProcessEvent, p) != 0) ProcessEvent(p);
    }
}

void* Socket::ProcessEvent(void* arg) {
    Socket* s = static_cast<Socket*>(arg);
    if (s->_on_edge_triggered_events) s->_on_edge_triggered_events(s);
    s->Dereference();
    return nullptr;
}

bool Socket::MoreReadEvents(int* progress) {
    return !_nevent.compare_exchange_strong(*progress, 0, std::memory_order_release, std::memory_order_acquire);
}

ssize_t Socket::DoRead(size_t size_hint) {
    const int fd = _fd.load(std::memory_order_acquire);
    if (fd < 0) {
        errno = EBADF;
        return -1;
    }
    if (_rdma_state.load(std::memory_order_acquire) != RDMA_OFF) return RdmaRead(fd, size_hint);
    if (_ssl_state.load(std::memory_order_acquire) != SSL_OFF) return SslRead(fd, size_hint);
    ssize_t n = _read_buf.append_from_fd(fd, size_hint);
    if (n > 0) {
        in_bytes.fetch_add(n, std::memory_order_relaxed);
        _last_active_us.store(monotonic_us(), std::memory_order_relaxed);
    }
    return n;
}

void Socket::InstallRdmaEndpoint(std::shared_ptr<rdma::Endpoint> ep) {
    std::lock_guard<std::mutex> g(_mu);
    _rdma_ep_raw.store(ep.get(), std::memory_order_release);
    _rdma_ep = std::move(ep);
}

ssize_t Socket::RdmaRead(int fd, size_t size_hint) {
    if (_rdma_state.load(std::memory_order_acquire) == RDMA_UNKNOWN) {
        // Server side, first bytes: an RDMA hello or a plain TCP client.
        const ssize_t n = _read_buf.append_from_fd(fd, size_hint);
        if (n <= 0) return n;
        in_bytes.fetch_add(n, std::memory_order_relaxed);
        _last_active_us.store(monotonic_us(), std::memory_order_relaxed);
        std::shared_ptr<rdma::Endpoint> ep;
        std::string err;
        const int rc = rdma::ServerTryHandshake(_this_id, fd, &_read_buf, &ep, &err);
        if (rc == 0) {
            errno = EAGAIN;  // hello incomplete: hide it from the parsers
            return -1;
        }
        if (rc < 0) {
            if (!err.empty()) {
                LOG(WARNING) << "RDMA handshake with " << _remote_side << " failed: " << err;
                errno = ERDMA;
                return -1;
            }
            _rdma_state.store(RDMA_OFF, std::memory_order_release);
            return n;
        }
        InstallRdmaEndpoint(std::move(ep));
        _rdma_state.store(RDMA_ON, std::memory_order_release);
        if (!_read_buf.empty()) {
            // bytes behind the hello on TCP: once verbs carry the traffic,
            // the TCP stream must stay silent (reference: FALLBACK_TCP /
            // EPROTO, test/brpc_rdma_unittest.cpp:577,1126)
            LOG(WARNING) << "data on TCP after the RDMA hello from " << _remote_side;
            errno = EPROTO;
            return -1;
        }
        errno = EAGAIN;
        return -1;
    }
    rdma::Endpoint* ep = rdma_endpoint();
    const ssize_t n = ep ? ep->ReadInto(&_read_buf) : -1;
    if (n > 0) {
        in_bytes.fetch_add(n, std::memory_order_relaxed);
        _last_active_us.store(monotonic_us(), std::memory_order_relaxed);
        return n;
    }
    // Nothing from the verbs side: the idle TCP connection tells us whether
    // the peer went away, or broke the protocol by writing on it.
    char c;
    const ssize_t r = ::recv(fd, &c, 1, MSG_PEEK | MSG_DONTWAIT);
    if (r == 0) return 0;
    if (r > 0) {
        LOG(WARNING) << "data on TCP after the RDMA hello from " << _remote_side;
        errno = EPROTO;
        return -1;
    }
    if (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK) return -1;
    errno = EAGAIN;
    return -1;
}

ssize_t Socket::WriteList(int fd, Buf** list, size_t n) {
    if (_rdma_state.load(std::memory_order_acquire) == RDMA_ON) {
        rdma::Endpoint* ep = rdma_endpoint();
        if (!ep) {
            errno = EPIPE;
            return -1;
        }
        return ep->CutFromBufList(list, n);
    }
    if (_conn) return _conn->CutMessageIntoFileDescriptor(fd, list, n);
    if (_ssl_state.load(std::memory_order_acquire) == SSL_ON) {
        std::shared_ptr<SslSession> ssl = ssl_session();
        if (!ssl) {
            std::lock_guard<std::mutex> g(_mu);
            if (!_ssl) _ssl = std::make_shared<SslSession>(_ssl_ctx, false, _ssl_sni);
            ssl = _ssl;
        }
        if (!ssl->ok()) {
            errno = EPROTO;
            return -1;
        }
        return ssl->Write(fd, list, n);
    }
    return Buf::cut_multiple_into_fd(fd, list, n);
}

std::shared_ptr<SslSession> Socket::ssl_session() const {
    std::lock_guard<std::mutex> g(_mu);
    return _ssl;
}

ssize_t Socket::SslRead(int fd, size_t size_hint) {
    for (;;) {
        BufPortal raw;
        const ssize_t n = raw.append_from_fd(fd, size_hint);
        if (n <= 0) return n;
        in_bytes.fetch_add(n, std::memory_order_relaxed);
        _last_active_us.store(monotonic_us(), std::memory_order_relaxed);
        if (_ssl_state.load(std::memory_order_acquire) == SSL_UNKNOWN) {
            char head[2];
            const size_t got = raw.copy_to(head, 2);
            if (LooksLikeTls(head, got) == 1) {
                std::lock_guard<std::mutex> g(_mu);
                _ssl = std::make_shared<SslSession>(_ssl_ctx, true, std::string());
                _ssl_state.store(SSL_ON, std::memory_order_release);
            } else {
                _ssl_state.store(SSL_OFF, std::memory_order_release);  // plaintext client
                _read_buf.append(std::move(raw));
                return n;
            }
        }
        std::shared_ptr<SslSession> ssl = ssl_session();
        if (!ssl) {
            std::lock_guard<std::mutex> g(_mu);
            if (!_ssl) _ssl = std::make_shared<SslSession>(_ssl_ctx, false, _ssl_sni);
            ssl = _ssl;
        }
        bool hs_done = false;
        const ssize_t produced = ssl->Feed(raw, &_read_buf, &hs_done);
        if (produced < 0) return -1;
        if (!ssl->Flush(fd)) {
            // Handshake records did not fit the socket buffer (rare): flush
            // them from a fiber that waits for EPOLLOUT.
            AddRef();
            fiber::fiber_t th;
            auto flusher = [](void* arg) -> void* {
                Socket* s = static_cast<Socket*>(arg);
                std::shared_ptr<SslSession> ss = s->ssl_session();
                for (int i = 0; ss && i < 200 && !s->Failed(); ++i) {
                    const int f = s->fd();
                    if (f < 0 || ss->Flush(f)) break;
                    timespec ts = realtime_after_us(50000);
                    s->WaitEpollOut(f, false, &ts);
                }
                s->Dereference();
                return nullptr;
            };
            if (fiber::start_background(&th, &fiber::ATTR_NORMAL, flusher, this) != 0) flusher(this);
        }
        if (hs_done) {
            _epollout_butex->fetch_add(1, std::memory_order_release);
            fiber::butex_wake_all(_epollout_butex);
        }
        if (produced > 0) return produced;
        if (ssl->peer_closed()) return 0;
    }
}

bool Socket::FightDeviceHello(int64_t timeout_us) {
    int st = _dev_hello.load(std::memory_order_acquire);
    if (st == 2) return false;
    if (st == 0 && _dev_hello.compare_exchange_strong(st, 1, std::memory_order_acq_rel)) return true;
    const int64_t deadline = monotonic_us() + timeout_us;
    for (;;) {
        const int seq = _dev_hello_butex->load(std::memory_order_acquire);
        st = _dev_hello.load(std::memory_order_acquire);
        if (st == 2) return false;
        if (st == 0) {  // the negotiator gave up: take over
            if (_dev_hello.compare_exchange_strong(st, 1, std::memory_order_acq_rel)) return true;
            continue;
        }
        const int64_t now = monotonic_us();
        if (now >= deadline || Failed()) return false;  // go ahead unnegotiated
        timespec ts = realtime_after_us(deadline - now);
        fiber::butex_wait(_dev_hello_butex, seq, &ts);
    }
}

void Socket::DeviceHelloAnswered() {
    if (_dev_hello.exchange(2, std::memory_order_acq_rel) == 2) return;
    _dev_hello_butex->fetch_add(1, std::memory_order_release);
    fiber::butex_wake_all(_dev_hello_butex);
}

void Socket::DeviceHelloAbandoned() {
    int st = 1;
    if (!_dev_hello.compare_exchange_strong(st, 0, std::memory_order_acq_rel)) return;
    _dev_hello_butex->fetch_add(1, std::memory_order_release);
    fiber::butex_wake_all(_dev_hello_butex);
}

void Socket::HandleEpollOut(SocketId id) {
    SocketUniquePtr s;
    if (AddressFailedAsWell(id, &s) < 0) return;
    s->_epollout_butex->fetch_add(1, std::memory_order_release);
    fiber::butex_wake_except(s->_epollout_butex, 0);
}

int Socket::WaitEpollOut(int fd, bool pollin, const timespec* abstime) {
    if (Failed()) {
        errno = EFAILEDSOCKET;
        return -1;
    }
    const int expected = _epollout_butex->load(std::memory_order_acquire);
    EventDispatcher& d = GetGlobalEventDispatcher(fd);
    if (d.AddEpollOut(_this_id, fd, pollin) != 0) return -1;
    int rc = 0;
    if (fiber::butex_wait(_epollout_butex, expected, abstime) < 0 && errno != EWOULDBLOCK && errno != EINTR) rc = -1;
    const int saved = errno;
    d.RemoveEpollOut(_this_id, fd, pollin);
    errno = saved;
    return rc;
}

// ---------------------------------------------------------------- write

int Socket::ConnectIfNot(const timespec* abstime, WriteRequest*) {
    if (_fd.load(std::memory_order_acquire) >= 0) return 0;
    if (_conn) return _conn->Connect(this, abstime);
    // Synchronous (fiber-aware) connect on first write.
    bool in_progress = false;
    int fd = tcp_connect_nonblocking(_remote_side, &in_progress);
    if (fd < 0) return -1;
    timespec ts;  // function scope: abstime may point here through the RDMA handshake
    if (in_progress) {
        if (!abstime) {
            ts = realtime_after_us((int64_t)FLAGS_connect_timeout_ms_default * 1000);
            abstime = &ts;
        }
        if (fiber::fd_timedwait(fd, EPOLLOUT, abstime) != 0) {
            const int saved = errno;
            fiber::close_fd(fd);
            errno = saved;
            return -1;
        }
        int err = 0;
        socklen_t len = sizeof(err);
        getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &len);
        if (err) {
            fiber::close_fd(fd);
            errno = err;
            return -1;
        }
    }
    if (_rdma_mode == SocketOptions::RDMA_CLIENT) {
        // Hello exchange before the fd joins the dispatcher, so the reply is
        // read here and not by the input messenger.
        std::string err;
        std::shared_ptr<rdma::Endpoint> ep = rdma::ClientHandshake(_this_id, fd, abstime, &err);
        if (!ep) {
            LOG(WARNING) << "RDMA handshake with " << _remote_side << " failed: " << err;
            fiber::close_fd(fd);
            errno = ERDMA;
            return -1;
        }
        InstallRdmaEndpoint(std::move(ep));
        _rdma_state.store(RDMA_ON, std::memory_order_release);
    }
    // Another writer can't race here: only the head writer connects.
    if (ResetFileDescriptor(fd) != 0) {
        const int saved = errno;
        _fd.store(-1);
        ::close(fd);
        errno = saved;
        return -1;
    }
    return 0;
}

void Socket::ReturnFailedWriteRequest(WriteRequest* req, int error_code, const std::string& error_text) {
    _unwritten_bytes.fetch_sub((int64_t)req->data.size(), std::memory_order_relaxed);
    req->data.clear();
    const fiber::CallId id = req->id_wait;
    return_object(req);
    if (id != fiber::INVALID_CALL_ID) fiber::call_id_error(id, error_code, error_text);
}

void Socket::ReleaseAllFailedWriteRequests(WriteRequest* req) {
    const int saved_ec = _error_code.load(std::memory_order_relaxed);
    const int error_code = saved_ec ? saved_ec : EFAILEDSOCKET;
    const std::string text = error_text();
    do {
        // release all but the last connected request
        while (req->next != nullptr) {
            WriteRequest* saved = req;
            req = req->next;
            ReturnFailedWriteRequest(saved, error_code, text);
        }
        _unwritten_bytes.fetch_sub((int64_t)req->data.size(), std::memory_order_relaxed);
        req->data.clear();  // MUST: otherwise IsWriteComplete never completes
    } while (!IsWriteComplete(req, true, nullptr));
    const fiber::CallId id = req->id_wait;
    return_object(req);
    if (id != fiber::INVALID_CALL_ID) fiber::call_id_error(id, error_code, text);
}

bool Socket::IsWriteComplete(WriteRequest* old_head, bool singular_node, WriteRequest** new_tail) {
    WriteRequest* new_head = old_head;
    WriteRequest* desired = nullptr;
    bool return_when_no_more = true;
    if (!old_head->data.empty() || !singular_node) {
        desired = old_head;
        return_when_no_more = false;
    }
    if (_write_head.compare_exchange_strong(new_head, desired, std::memory_order_acquire)) {
        if (new_tail) *new_tail = old_head;
        return return_when_no_more;
    }
    // New requests were pushed; new_head is the newest. Reverse them and
    // link after old_head.
    WriteRequest* tail = nullptr;
    WriteRequest* p = new_head;
    do {
        // the pusher links `next` right after its exchange (release store)
        while (__atomic_load_n(&p->next, __ATOMIC_ACQUIRE) == UNCONNECTED) sched_yield();
        WriteRequest* const saved_next = p->next;
        p->next = tail;
        tail = p;
        p = saved_next;
    } while (p != old_head);
    old_head->next = tail;
    if (new_tail) *new_tail = new_head;
    return false;
}

int Socket::Write(Buf* data, const WriteOptions* options) {
    static const WriteOptions kDefault;
    const WriteOptions& opt = options ? *options : kDefault;
    // an empty write only matters as a half-close after what is queued
    if (data->empty() && !opt.shutdown_write_after) return 0;
    if (Failed()) {
        const int saved_ec = _error_code.load(std::memory_order_relaxed);
        const int ec = saved_ec ? saved_ec : EFAILEDSOCKET;
        if (opt.id_wait != fiber::INVALID_CALL_ID) fiber::call_id_error(opt.id_wait, ec, error_text());
        errno = ec;
        if (opt.auth_winner) SetAuthentication(ec);
        return -1;
    }
    if (!opt.ignore_eovercrowded && _unwritten_bytes.load(std::memory_order_relaxed) > FLAGS_socket_max_unwritten_bytes) {
        if (opt.id_wait != fiber::INVALID_CALL_ID) fiber::call_id_error(opt.id_wait, EOVERCROWDED, "socket overcrowded");
        errno = EOVERCROWDED;
        if (opt.auth_winner) ResetAuthentication();  // the next writer sends the credentials
        return -1;
    }
    WriteRequest* req = get_object<WriteRequest>();
    req->data.swap(*data);
    req->next = UNCONNECTED;
    req->id_wait = opt.id_wait;
    req->socket = this;
    req->shutdown_after = opt.shutdown_write_after;
    if (opt.id_wait != fiber::INVALID_CALL_ID) {
        std::lock_guard<std::mutex> g(_shared->mu);
        auto& v = _shared->id_wait_list;
        v.push_back(opt.id_wait);
        if (v.size() > 256 && v.size() > 2 * _shared->last_compact) {
            size_t j = 0;
            for (size_t i = 0; i < v.size(); ++i) {
                if (fiber::call_id_exists(v[i])) v[j++] = v[i];
            }
            v.resize(j);
            _shared->last_compact = j;
        }
    }
    if (opt.pipelined_count > 0) {
        // the queue order must equal the wire order: enqueue the entry and
        // the write under one lock (StartWrite's exchange fixes the order)
        std::lock_guard<std::mutex> g(_pipeline_mu);
        PipelinedInfo pi;
        pi.count = opt.pipelined_count;
        pi.auth_replies = opt.auth_replies;
        pi.tag = opt.pipelined_tag;
        pi.protocol = opt.pipelined_protocol;
        pi.id_wait = opt.id_wait;
        _pipeline_q.push_back(pi);
        const int rc = StartWrite(req, opt);
        if (opt.auth_winner) SetAuthentication(0);  // later writers follow the credentials on the wire
        return rc;
    }
    const int rc = StartWrite(req, opt);
    if (opt.auth_winner) SetAuthentication(0);
    return rc;
}

bool Socket::PopPipelinedInfo(PipelinedInfo* out) {
    std::lock_guard<std::mutex> g(_pipeline_mu);
    if (_pipeline_q.empty()) return false;
    *out = _pipeline_q.front();
    _pipeline_q.pop_front();
    return true;
}

bool Socket::PeekPipelinedInfo(PipelinedInfo* out) {
    std::lock_guard<std::mutex> g(_pipeline_mu);
    if (_pipeline_q.empty()) return false;
    *out = _pipeline_q.front();
    return true;
}

void Socket::GivebackPipelinedInfo(const PipelinedInfo& pi) {
    std::lock_guard<std::mutex> g(_pipeline_mu);
    _pipeline_q.push_front(pi);
}

int Socket::StartWrite(WriteRequest* req, const WriteOptions& opt) {
    _unwritten_bytes.fetch_add((int64_t)req->data.size(), std::memory_order_relaxed);
    out_messages.fetch_add(1, std::memory_order_relaxed);
    WriteRequest* const prev_head = _write_head.exchange(req, std::memory_order_release);
    if (prev_head != nullptr) {
        // Someone is writing; it will pick up this request.
        __atomic_store_n(&req->next, prev_head, __ATOMIC_RELEASE);  // read by the writer's IsWriteComplete
        return 0;
    }
    req->next = nullptr;
    int saved_errno = 0;
    ssize_t nw = 0;
    if (ConnectIfNot(nullptr, req) != 0) {
        saved_errno = errno;
        SetFailed(saved_errno ? saved_errno : EFAILEDSOCKET, "fail to connect %s: %s", _remote_side.to_string().c_str(),
                  ErrorText(saved_errno));
        ReleaseAllFailedWriteRequests(req);
        errno = saved_errno;
        return -1;
    }
    if (!opt.write_in_background) {
        const int fd = _fd.load(std::memory_order_acquire);
        if (_conn || _ssl_state.load(std::memory_order_relaxed) == SSL_ON ||
            _rdma_state.load(std::memory_order_relaxed) == RDMA_ON) {
            Buf* list[1] = {&req->data};
            nw = WriteList(fd, list, 1);
        } else {
            nw = req->data.cut_into_fd(fd);
        }
        if (nw < 0) {
            if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EOVERCROWDED && errno != EINPROGRESS) {
                saved_errno = errno;
                SetFailed(saved_errno, "fail to write into fd: %s", ErrorText(saved_errno));
                ReleaseAllFailedWriteRequests(req);
                errno = saved_errno;
                return -1;
            }
        } else {
            _unwritten_bytes.fetch_sub(nw, std::memory_order_relaxed);
            out_bytes.fetch_add(nw, std::memory_order_relaxed);
        }
        if (IsWriteComplete(req, true, nullptr)) {
            finish_write_request(req, this->fd());
            return 0;
        }
    }
    // KeepWrite owns a reference: the caller's may go away while requests
    // are still queued, and a recycled slot would hand this write queue to
    // the next connection.
    AddRef();
    fiber::fiber_t th;
    if (fiber::start_background(&th, &fiber::ATTR_NORMAL, KeepWrite, req) != 0) KeepWrite(req);
    return 0;
}

ssize_t Socket::DoWrite(WriteRequest* req) {
    Buf* list[Buf::MAX_WRITEV_IOV];
    size_t n = 0;
    for (WriteRequest* p = req; p != nullptr && n < (size_t)Buf::MAX_WRITEV_IOV; p = p->next) list[n++] = &p->data;
    const int fd = _fd.load(std::memory_order_acquire);
    if (fd < 0) {
        errno = EBADF;
        return -1;
    }
    ssize_t nw = WriteList(fd, list, n);
    if (nw > 0) out_bytes.fetch_add(nw, std::memory_order_relaxed);
    return nw;
}

void* Socket::KeepWrite(void* arg) {
    WriteRequest* req = static_cast<WriteRequest*>(arg);
    Socket* s = req->socket;
    WriteRequest* cur_tail = nullptr;
    for (;;) {
        if (req->next != nullptr && req->data.empty()) {
            WriteRequest* saved = req;
            req = req->next;
            finish_write_request(saved, s->fd());
        }
        if (s->Failed()) break;
        const ssize_t nw = s->DoWrite(req);
        if (nw < 0) {
            if (errno == EINPROGRESS) {
                // TLS handshake in flight: the read side wakes us when done.
                const int expected = s->_epollout_butex->load(std::memory_order_acquire);
                if (s->_ssl && !s->_ssl->handshake_done()) {
                    timespec ts = realtime_after_us(50000);
                    fiber::butex_wait(s->_epollout_butex, expected, &ts);
                }
                continue;
            }
            if (errno != EAGAIN && errno != EWOULDBLOCK && errno != EOVERCROWDED) {
                const int saved_errno = errno;
                s->SetFailed(saved_errno, "fail to keep writing: %s", ErrorText(saved_errno));
                break;
            }
            timespec ts = realtime_after_us(50000);
            if (rdma::Endpoint* ep = s->is_rdma() ? s->rdma_endpoint() : nullptr) {
                // verbs window / send queue full: park until completions free it
                if (ep->WaitWritable(&ts) != 0 && errno != ETIMEDOUT) {
                    const int saved_errno = errno ? errno : EFAILEDSOCKET;
                    s->SetFailed(saved_errno, "fail to wait rdma window: %s", ErrorText(saved_errno));
                    break;
                }
                continue;
            }
            const int fd = s->fd();
            if (fd < 0 || s->WaitEpollOut(fd, s->_on_edge_triggered_events != nullptr, &ts) != 0) {
                if (errno != ETIMEDOUT && errno != EWOULDBLOCK && errno != EINTR) {
                    const int saved_errno = errno ? errno : EFAILEDSOCKET;
                    s->SetFailed(saved_errno, "fail to wait epollout: %s", ErrorText(saved_errno));
                    break;
                }
            }
        } else {
            s->_unwritten_bytes.fetch_sub(nw, std::memory_order_relaxed);
        }
        while (req->next != nullptr && req->data.empty()) {
            WriteRequest* saved = req;
            req = req->next;
            finish_write_request(saved, s->fd());
        }
        if (cur_tail == nullptr) {
            for (cur_tail = req; cur_tail->next != nullptr; cur_tail = cur_tail->next) {
            }
        }
        if (s->IsWriteComplete(cur_tail, req == cur_tail, &cur_tail)) {
            finish_write_request(req, s->fd());
            s->Dereference();
            return nullptr;
        }
    }
    s->ReleaseAllFailedWriteRequests(req);
    s->Dereference();
    return nullptr;
}

// ---------------------------------------------------------------- pool / short

int Socket::GetPooledSocket(SocketUniquePtr* out) {
    std::shared_ptr<SharedPart> sp = _shared;
    if (!sp) return -1;
    for (;;) {
        SocketId sid = INVALID_SOCKET_ID;
        {
            std::lock_guard<std::mutex> g(sp->mu);
            if (sp->pool.empty()) break;
            sid = sp->pool.back();
            sp->pool.pop_back();
        }
        if (Address(sid, out) == 0) return 0;
    }
    SocketOptions opt;
    opt.remote_side = _remote_side;
    opt.user = _user;
    opt.on_edge_triggered_events = _on_edge_triggered_events;
    opt.conn = _conn;
    opt.ssl_ctx = _ssl_ctx;
    opt.ssl_sni = _ssl_sni;
    opt.connect_lazily = true;
    SocketId sid;
    if (Create(opt, &sid) != 0) return -1;
    if (Address(sid, out) != 0) return -1;
    (*out)->_main_socket_id = _this_id;
    return 0;
}

void Socket::ReturnToPool() {
    SocketUniquePtr main;
    if (_main_socket_id == INVALID_SOCKET_ID || Address(_main_socket_id, &main) != 0 || Failed()) {
        SetFailed(EUNUSED, "pooled socket not returnable");
        return;
    }
    std::shared_ptr<SharedPart> sp = main->_shared;
    std::lock_guard<std::mutex> g(sp->mu);
    if ((int)sp->pool.size() >= FLAGS_max_connection_pool_size) {
        SetFailed(EUNUSED, "connection pool full");
        return;
    }
    sp->pool.push_back(_this_id);
}

int Socket::GetShortSocket(SocketUniquePtr* out) {
    SocketOptions opt;
    opt.remote_side = _remote_side;
    opt.user = _user;
    opt.on_edge_triggered_events = _on_edge_triggered_events;
    opt.conn = _conn;
    opt.ssl_ctx = _ssl_ctx;
    opt.ssl_sni = _ssl_sni;
    opt.connect_lazily = true;
    SocketId sid;
    if (Create(opt, &sid) != 0) return -1;
    return Address(sid, out);
}

// ---------------------------------------------------------------- auth

bool Socket::FightAuthentication(int* auth_error) {
    for (;;) {
        int expected = 0;
        if (_auth_state.compare_exchange_strong(expected, 1)) return true;
        if (expected == 2) {
            *auth_error = _auth_error.load();
            return false;
        }
        // someone is authenticating: wait for the outcome (or a reset)
        const int seq = _auth_butex->load(std::memory_order_acquire);
        if (_auth_state.load(std::memory_order_acquire) == 1) fiber::butex_wait(_auth_butex, seq, nullptr);
    }
}

void Socket::SetAuthentication(int error) {
    _auth_error.store(error);
    _auth_state.store(2, std::memory_order_release);
    _auth_butex->fetch_add(1, std::memory_order_release);
    fiber::butex_wake_all(_auth_butex);
}

void Socket::ResetAuthentication() {
    _auth_state.store(0, std::memory_order_release);
    _auth_butex->fetch_add(1, std::memory_order_release);
    fiber::butex_wake_all(_auth_butex);
}

// ---------------------------------------------------------------- health check / revive

int Socket::Revive(int new_fd) {
    const uint32_t id_ver = sid_ver(_this_id);
    uint64_t vref = _versioned_ref.load(std::memory_order_relaxed);
    for (;;) {
        if (vref_ver(vref) != id_ver + 1) return -1;
        // reset per-connection state before becoming visible again
        _read_buf.clear();
        _nevent.store(0);
        _preferred_index = -1;
        {
            // a new connection needs a new TLS session
            std::lock_guard<std::mutex> g(_mu);
            _ssl.reset();
        }
        if (_ssl_ctx) _ssl_state.store(_ssl_ctx->is_server() ? SSL_UNKNOWN : SSL_ON);
        if (_rdma_mode != SocketOptions::RDMA_NONE) {
            InstallRdmaEndpoint(nullptr);
            _rdma_state.store(_rdma_mode == SocketOptions::RDMA_SERVER ? RDMA_UNKNOWN : RDMA_OFF);
        }
        delete _parsing_context.exchange(nullptr);
        {
            std::lock_guard<std::mutex> g(_pipeline_mu);
            _pipeline_q.clear();
        }
        _auth_state.store(0);
        _plane_rank.store(kPlaneUnknown);
        _dev_hello.store(0);
        const int old = _fd.exchange(-1);
        if (old >= 0) ::close(old);
        if (_versioned_ref.compare_exchange_strong(vref, make_vref(id_ver, vref_nref(vref)), std::memory_order_release)) {
            break;
        }
    }
    {
        std::lock_guard<std::mutex> g(_mu);
        _error_code.store(0, std::memory_order_relaxed);
        _error_text.clear();
    }
    if (new_fd >= 0) ResetFileDescriptor(new_fd);
    LOG(INFO) << "Revived " << description();
    return 0;
}

std::atomic<int64_t> g_app_health_checks{0}, g_app_health_check_failures{0};

// The application-level half of the check (reference:
// src/brpc/details/health_check.cpp:34-39,147-190): the server must answer
// an HTTP GET of -health_check_path, not merely accept connections. It runs
// on a connection of its own (servers here take HTTP and the RPC protocols
// on one port, TLS or not), so the failed socket never carries user
// traffic before the check passed.
static bool app_health_check_ok(const EndPoint& remote) {
    const std::string path = FLAGS_health_check_path;
    if (path.empty()) return true;
    g_app_health_checks.fetch_add(1, std::memory_order_relaxed);
    std::string body;
    const std::string url = "http://" + remote.to_string() + (path[0] == '/' ? "" : "/") + path;
    if (HttpGet(url, &body, std::max(1, FLAGS_health_check_timeout_ms)) == 0) return true;
    g_app_health_check_failures.fetch_add(1, std::memory_order_relaxed);
    return false;
}

void* Socket::HealthCheckThread(void* arg) {
    Socket* s = static_cast<Socket*>(arg);
    for (;;) {
        fiber::usleep((uint64_t)std::max(1, s->_health_check_interval_s) * 1000000);
        if (s->_recycle_flag.load()) break;
        int fd = tcp_connect(s->_remote_side, std::max(1, FLAGS_health_check_timeout_ms));
        if (fd >= 0 && !app_health_check_ok(s->_remote_side)) {
            ::close(fd);  // connectable, not healthy: check again next interval
            continue;
        }
        if (fd >= 0) {
            s->_hc_started.store(false);
            if (s->_recycle_flag.load()) {
                ::close(fd);
                break;
            }
            if (s->_rdma_mode == SocketOptions::RDMA_CLIENT) {
                // reconnect (with a fresh hello exchange) on the next write
                ::close(fd);
                fd = -1;
            }
            s->Revive(fd);
            return nullptr;  // keep the creator reference: socket alive again
        }
    }
    s->_hc_started.store(false);
    s->Dereference();  // release the creator reference
    return nullptr;
}

void Socket::StartHealthCheck() {
    if (_hc_started.exchange(true)) return;
    fiber::fiber_t th;
    if (fiber::start_background(&th, &fiber::ATTR_NORMAL, HealthCheckThread, this) != 0) {
        _hc_started.store(false);
        Dereference();
    }
}

std::string Socket::description() const {
    return string_printf("Socket{id=%llu fd=%d remote=%s nref=%u%s%s%s}", (unsigned long long)_this_id, fd(),
                         _remote_side.to_string().c_str(), nref(), Failed() ? " failed" : "",
                         is_ssl() ? " tls" : "",
                         is_rdma() && rdma_endpoint() ? (" " + rdma_endpoint()->Describe()).c_str() : "");
}

std::string DescribeAllSockets() {
    std::string out;
    ResourcePool<Socket>::singleton()->for_each([&out](uint32_t, Socket* s) {
        const uint64_t v = s->nref();
        if (v == 0) return;
        if (s->fd() < 0 && s->Failed()) return;
        out += s->description();
        string_appendf(&out, " in=%lld out=%lld\n", (long long)s->in_bytes.load(), (long long)s->out_bytes.load());
    });
    return out;
}

}  // namespace mrpc
