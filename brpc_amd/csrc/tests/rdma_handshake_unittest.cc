// RDMA hello state machine under hostile or broken peers (spirit of the
// reference's test/brpc_rdma_unittest.cpp:170-1240: closes at every
// handshake step, invalid magic / length / version / queue and block sizes,
// data on TCP after the switch to verbs, option validation), plus RDMA
// under the connection types and combo channels. A raw TCP socket plays the
// client against a real RDMA server, and a raw listener plays the server
// against a real RDMA channel; the soft verbs provider gives the raw side a
// real queue pair when a test needs the handshake to succeed. Every case
// checks that the real side fails fast (no hang until a timeout), frees the
// connection and keeps serving.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "base/flags.h"
#include "base/time.h"
#include "mrpc/proto/echo.pb.h"
#include "net/socket.h"
#include "rdma/rdma.h"
#include "rpc/channel.h"
#include "rpc/combo_channels.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

DECLARE_string(rdma_provider);
DECLARE_int32(rdma_handshake_timeout_ms);

using namespace mrpc;

namespace {

void InitSoft() {
    FLAGS_rdma_provider = "auto";
    std::string err;
    if (rdma::GlobalRdmaInitialize(&err) != 0) fprintf(stderr, "rdma init: %s\n", err.c_str());
}

struct RdmaServer {
    Server server;
    EchoServiceImpl echo;
    int port = 0;
    explicit RdmaServer(bool rdma = true) {
        server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        ServerOptions o;
        o.use_rdma = rdma;
        if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
    }
    std::string addr() const { return "127.0.0.1:" + std::to_string(port); }
    int Connections() {
        std::vector<SocketId> conns;
        server.acceptor()->ListConnections(&conns);
        return (int)conns.size();
    }
    bool WaitConnections(int want, int timeout_ms = 3000) {
        const int64_t end = monotonic_us() + timeout_ms * 1000ll;
        while (monotonic_us() < end) {
            if (Connections() == want) return true;
            usleep(5000);
        }
        return Connections() == want;
    }
};

int RawConnect(int port) {
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a;
    memset(&a, 0, sizeof(a));
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (connect(fd, (sockaddr*)&a, sizeof(a)) != 0) {
        close(fd);
        return -1;
    }
    return fd;
}

// A raw listener on 127.0.0.1:<port>.
int RawListen(int* port) {
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a;
    memset(&a, 0, sizeof(a));
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (bind(fd, (sockaddr*)&a, sizeof(a)) != 0 || listen(fd, 16) != 0) {
        close(fd);
        return -1;
    }
    socklen_t len = sizeof(a);
    getsockname(fd, (sockaddr*)&a, &len);
    *port = ntohs(a.sin_port);
    return fd;
}

bool ReadExactly(int fd, char* b, size_t n, int timeout_ms) {
    size_t got = 0;
    const int64_t end = monotonic_us() + timeout_ms * 1000ll;
    while (got < n) {
        const int64_t left = (end - monotonic_us()) / 1000;
        if (left <= 0) return false;
        pollfd p{fd, POLLIN, 0};
        if (poll(&p, 1, (int)left) <= 0) return false;
        const ssize_t r = recv(fd, b + got, n - got, 0);
        if (r <= 0) return false;
        got += (size_t)r;
    }
    return true;
}

// The peer closed (EOF or reset) within timeout_ms.
bool PeerClosed(int fd, int timeout_ms) {
    const int64_t end = monotonic_us() + timeout_ms * 1000ll;
    char b[256];
    while (monotonic_us() < end) {
        pollfd p{fd, POLLIN, 0};
        const int64_t left = (end - monotonic_us()) / 1000;
        if (poll(&p, 1, (int)std::max<int64_t>(1, left)) <= 0) continue;
        const ssize_t r = recv(fd, b, sizeof(b), 0);
        if (r == 0 || (r < 0 && errno != EAGAIN && errno != EINTR)) return true;
    }
    return false;
}

// A queue pair of the soft provider, so a raw peer can offer a real address.
struct SoftPeer {
    std::unique_ptr<rdma::CompletionQueue> cq;
    std::unique_ptr<rdma::QueuePair> qp;
    SoftPeer() {
        rdma::Provider* pr = rdma::GetProvider();
        if (!pr) return;
        cq = pr->CreateCq(64);
        if (cq) qp = pr->CreateQp(cq.get(), 16, 16);
        if (qp) qp->Prepare();
    }
};

std::string HelloBytes(const rdma::QpAddress& addr, const std::function<void(rdma::Hello*)>& tweak = nullptr) {
    rdma::Hello h;
    h.sq_size = 16;
    h.rq_size = 16;
    h.block_size = 8128;
    h.addr = addr;
    if (tweak) tweak(&h);
    std::string b(rdma::Hello::kSize, '\0');
    h.Serialize(&b[0]);
    return b;
}

rdma::QpAddress BogusAddress() {
    rdma::QpAddress a;
    a.gid_hi = 0xfe80000000000000ull;
    a.gid_lo = 0x1234567890abcdefull;
    a.qpn = 0xFFFFFF;
    a.lid = 9;
    return a;
}

thread_local std::string g_last_error;  // the calling thread's last failure (tests call from many threads)

bool Echo(ChannelBase* ch, const std::string& msg, int* code = nullptr, int64_t sleep_us = 0) {
    example::EchoService_Stub stub(ch);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message(msg);
    if (sleep_us) req.set_sleep_us((int32_t)sleep_us);
    stub.Echo(&cntl, &req, &res, nullptr);
    if (code) *code = cntl.ErrorCode();
    g_last_error = cntl.ErrorText();
    return !cntl.Failed() && res.message() == msg;
}

// A real RDMA client still gets served (the server survived the abuse).
bool ServerStillServes(RdmaServer& s) {
    Channel ch;
    ChannelOptions o;
    o.use_rdma = true;
    o.timeout_ms = 3000;
    o.max_retry = 0;
    o.connection_group = "still-serves";
    if (ch.Init(s.addr().c_str(), &o) != 0) return false;
    return Echo(&ch, "alive");
}

// ---- server side: a raw client misbehaves at one step of the hello
void ExpectServerDropsHello(const std::string& bytes) {
    InitSoft();
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    const int fd = RawConnect(s.port);
    ASSERT_TRUE(fd >= 0);
    ASSERT_TRUE(s.WaitConnections(1));
    ASSERT_EQ(send(fd, bytes.data(), bytes.size(), 0), (ssize_t)bytes.size());
    EXPECT_TRUE(PeerClosed(fd, 3000));  // refused: the server closes
    close(fd);
    EXPECT_TRUE(s.WaitConnections(0));
    EXPECT_TRUE(ServerStillServes(s));
}

// ---- client side: a raw server misbehaves; the RDMA channel's call must
// fail well before its timeout
void ExpectClientFails(const std::function<void(int acc)>& server_script, int64_t max_us = 1500000) {
    InitSoft();
    const int saved = FLAGS_rdma_handshake_timeout_ms;
    FLAGS_rdma_handshake_timeout_ms = 400;
    int port = 0;
    const int lfd = RawListen(&port);
    ASSERT_TRUE(lfd >= 0);
    std::thread srv([&] {
        const int acc = accept(lfd, nullptr, nullptr);
        if (acc >= 0) {
            server_script(acc);
            close(acc);
        }
    });
    Channel ch;
    ChannelOptions o;
    o.use_rdma = true;
    o.timeout_ms = 5000;
    o.connect_timeout_ms = 1000;
    o.max_retry = 0;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(port)).c_str(), &o), 0);
    const int64_t t0 = monotonic_us();
    int code = 0;
    EXPECT_FALSE(Echo(&ch, "x", &code));
    EXPECT_TRUE_M(monotonic_us() - t0 < max_us,
                  std::to_string(monotonic_us() - t0) + " us, [E" + std::to_string(code) + "] " + g_last_error);
    EXPECT_NE(code, 0);
    shutdown(lfd, SHUT_RDWR);
    close(lfd);
    srv.join();
    FLAGS_rdma_handshake_timeout_ms = saved;
}

}  // namespace

TEST(RdmaHandshake, client_close_before_hello_send) {
    InitSoft();
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    const int fd = RawConnect(s.port);
    ASSERT_TRUE(fd >= 0);
    ASSERT_TRUE(s.WaitConnections(1));
    close(fd);
    EXPECT_TRUE(s.WaitConnections(0));
    EXPECT_TRUE(ServerStillServes(s));
}

TEST(RdmaHandshake, client_hello_invalid_magic) {
    std::string b = HelloBytes(BogusAddress());
    b[3] = 'X';  // "RDMX": not an RDMA hello, and not any protocol either
    ExpectServerDropsHello(b);
}

TEST(RdmaHandshake, client_close_during_hello_send) {
    InitSoft();
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    SoftPeer peer;
    ASSERT_TRUE(peer.qp != nullptr);
    const std::string b = HelloBytes(peer.qp->local());
    for (size_t cut : {1, 4, 5, 20, 43}) {
        const int fd = RawConnect(s.port);
        ASSERT_TRUE(fd >= 0);
        ASSERT_EQ(send(fd, b.data(), cut, 0), (ssize_t)cut);
        usleep(20000);  // the server holds the partial hello
        close(fd);
        EXPECT_TRUE_M(s.WaitConnections(0), "cut at " + std::to_string(cut));
    }
    EXPECT_TRUE(ServerStillServes(s));
}

TEST(RdmaHandshake, client_hello_invalid_version) {
    ExpectServerDropsHello(HelloBytes(BogusAddress(), [](rdma::Hello* h) { h->version = 7; }));
}

TEST(RdmaHandshake, client_hello_invalid_rq_size) {
    // no room for the receive ring's ACK reserve
    ExpectServerDropsHello(HelloBytes(BogusAddress(), [](rdma::Hello* h) { h->rq_size = 1; }));
}

TEST(RdmaHandshake, client_hello_invalid_sq_size) {
    ExpectServerDropsHello(HelloBytes(BogusAddress(), [](rdma::Hello* h) { h->sq_size = 0; }));
}

TEST(RdmaHandshake, client_hello_invalid_block_size) {
    ExpectServerDropsHello(HelloBytes(BogusAddress(), [](rdma::Hello* h) { h->block_size = 32; }));
}

TEST(RdmaHandshake, client_hello_unreachable_queue_pair) {
    // a well-formed hello naming a queue pair nobody owns: the server cannot
    // connect its QP and drops the connection
    ExpectServerDropsHello(HelloBytes(BogusAddress()));
}

TEST(RdmaHandshake, client_hello_in_fragments_is_answered) {
    InitSoft();
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    SoftPeer peer;
    ASSERT_TRUE(peer.qp != nullptr);
    const std::string b = HelloBytes(peer.qp->local());
    const int fd = RawConnect(s.port);
    ASSERT_TRUE(fd >= 0);
    // the magic split, then the rest a few bytes at a time
    size_t off = 0;
    for (size_t step : {2, 3, 9, 30}) {
        ASSERT_EQ(send(fd, b.data() + off, step, 0), (ssize_t)step);
        off += step;
        usleep(30000);
    }
    ASSERT_EQ(off, rdma::Hello::kSize);
    char reply[rdma::Hello::kSize];
    ASSERT_TRUE(ReadExactly(fd, reply, sizeof(reply), 3000));
    rdma::Hello h;
    EXPECT_TRUE(h.Parse(reply));
    EXPECT_GT(h.rq_size, 0);
    EXPECT_GE(h.block_size, 64u);
    close(fd);
    EXPECT_TRUE(s.WaitConnections(0));
    EXPECT_TRUE(ServerStillServes(s));
}

TEST(RdmaHandshake, client_close_after_hello_exchange) {
    InitSoft();
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    for (int round = 0; round < 3; ++round) {
        SoftPeer peer;
        ASSERT_TRUE(peer.qp != nullptr);
        const std::string b = HelloBytes(peer.qp->local());
        const int fd = RawConnect(s.port);
        ASSERT_TRUE(fd >= 0);
        ASSERT_EQ(send(fd, b.data(), b.size(), 0), (ssize_t)b.size());
        char reply[rdma::Hello::kSize];
        ASSERT_TRUE(ReadExactly(fd, reply, sizeof(reply), 3000));
        close(fd);  // the verbs side is up, the TCP side goes away
        EXPECT_TRUE(s.WaitConnections(0));
    }
    EXPECT_TRUE(ServerStillServes(s));
}

TEST(RdmaHandshake, client_sends_tcp_data_after_hello) {
    InitSoft();
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    SoftPeer peer;
    ASSERT_TRUE(peer.qp != nullptr);
    const std::string b = HelloBytes(peer.qp->local());
    {
        // bytes behind the hello in the same write
        const int fd = RawConnect(s.port);
        ASSERT_TRUE(fd >= 0);
        const std::string both = b + "PRPC garbage on tcp";
        ASSERT_EQ(send(fd, both.data(), both.size(), 0), (ssize_t)both.size());
        EXPECT_TRUE(PeerClosed(fd, 3000));
        close(fd);
    }
    SoftPeer peer2;
    ASSERT_TRUE(peer2.qp != nullptr);
    {
        // bytes on TCP once the hello was answered
        const std::string b2 = HelloBytes(peer2.qp->local());
        const int fd = RawConnect(s.port);
        ASSERT_TRUE(fd >= 0);
        ASSERT_EQ(send(fd, b2.data(), b2.size(), 0), (ssize_t)b2.size());
        char reply[rdma::Hello::kSize];
        ASSERT_TRUE(ReadExactly(fd, reply, sizeof(reply), 3000));
        ASSERT_EQ(send(fd, "PRPC", 4, 0), 4);
        EXPECT_TRUE(PeerClosed(fd, 3000));  // EPROTO: the server drops it
        close(fd);
    }
    EXPECT_TRUE(s.WaitConnections(0));
    EXPECT_TRUE(ServerStillServes(s));
}

TEST(RdmaHandshake, server_miss_hello) {
    // the listener accepts and never answers: the handshake times out
    ExpectClientFails([](int acc) {
        char b[rdma::Hello::kSize];
        ReadExactly(acc, b, sizeof(b), 2000);
        usleep(900000);
    });
}

TEST(RdmaHandshake, server_close_before_hello) {
    ExpectClientFails([](int acc) { (void)acc; });
}

TEST(RdmaHandshake, server_close_during_hello) {
    ExpectClientFails([](int acc) {
        char b[rdma::Hello::kSize];
        ReadExactly(acc, b, sizeof(b), 2000);
        const std::string h = HelloBytes(BogusAddress());
        send(acc, h.data(), 10, 0);
    });
}

TEST(RdmaHandshake, server_hello_invalid_magic) {
    ExpectClientFails([](int acc) {
        char b[rdma::Hello::kSize];
        ReadExactly(acc, b, sizeof(b), 2000);
        std::string h = HelloBytes(BogusAddress());
        h[0] = 'r';
        send(acc, h.data(), h.size(), 0);
        usleep(200000);
    });
}

TEST(RdmaHandshake, server_hello_invalid_version) {
    ExpectClientFails([](int acc) {
        char b[rdma::Hello::kSize];
        ReadExactly(acc, b, sizeof(b), 2000);
        const std::string h = HelloBytes(BogusAddress(), [](rdma::Hello* x) { x->version = 2; });
        send(acc, h.data(), h.size(), 0);
        usleep(200000);
    });
}

TEST(RdmaHandshake, server_hello_invalid_queue_sizes) {
    ExpectClientFails([](int acc) {
        char b[rdma::Hello::kSize];
        ReadExactly(acc, b, sizeof(b), 2000);
        const std::string h = HelloBytes(BogusAddress(), [](rdma::Hello* x) {
            x->sq_size = 0;
            x->rq_size = 0;
        });
        send(acc, h.data(), h.size(), 0);
        usleep(200000);
    });
}

TEST(RdmaHandshake, server_hello_unreachable_queue_pair) {
    ExpectClientFails([](int acc) {
        char b[rdma::Hello::kSize];
        ReadExactly(acc, b, sizeof(b), 2000);
        const std::string h = HelloBytes(BogusAddress());
        send(acc, h.data(), h.size(), 0);
        usleep(200000);
    });
}

TEST(RdmaHandshake, server_sends_tcp_data_after_hello) {
    // a real queue pair answers, then the "server" writes on TCP: the
    // client fails the connection (EPROTO) instead of waiting out its timeout
    SoftPeer peer;
    InitSoft();
    SoftPeer p2;
    ExpectClientFails([&](int acc) {
        char b[rdma::Hello::kSize];
        if (!ReadExactly(acc, b, sizeof(b), 2000) || !p2.qp) return;
        rdma::Hello theirs;
        if (theirs.Parse(b)) p2.qp->Connect(theirs.addr);
        const std::string h = HelloBytes(p2.qp->local());
        send(acc, h.data(), h.size(), 0);
        usleep(50000);
        send(acc, "PRPC junk", 9, 0);
        usleep(600000);
    }, 450000);
}

TEST(RdmaHandshake, server_close_after_hello) {
    InitSoft();
    SoftPeer p2;
    ExpectClientFails([&](int acc) {
        char b[rdma::Hello::kSize];
        if (!ReadExactly(acc, b, sizeof(b), 2000) || !p2.qp) return;
        rdma::Hello theirs;
        if (theirs.Parse(b)) p2.qp->Connect(theirs.addr);
        const std::string h = HelloBytes(p2.qp->local());
        send(acc, h.data(), h.size(), 0);
        usleep(100000);  // then the TCP side closes: EOF fails the socket
    });
}

TEST(RdmaHandshake, channel_and_server_options_invalid) {
    InitSoft();
    {
        Channel ch;
        ChannelOptions o;
        o.use_rdma = true;
        o.use_ssl = true;  // exclusive
        EXPECT_NE(ch.Init("127.0.0.1:1", &o), 0);
    }
    {
        Server srv;
        EchoServiceImpl echo;
        srv.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        ServerOptions o;
        o.use_rdma = true;
        o.ssl_cert_file = "/nonexistent/cert.pem";  // TLS and RDMA are exclusive
        EXPECT_NE(srv.Start("127.0.0.1:0", &o), 0);
    }
}

TEST(RdmaHandshake, pooled_and_short_connections) {
    InitSoft();
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    for (const char* type : {"pooled", "short"}) {
        Channel ch;
        ChannelOptions o;
        o.use_rdma = true;
        o.timeout_ms = 5000;
        o.connection_type = type;
        ASSERT_EQ(ch.Init(s.addr().c_str(), &o), 0);
        std::vector<std::thread> th;
        std::atomic<int> ok{0};
        for (int t = 0; t < 4; ++t) {
            th.emplace_back([&, t] {
                for (int i = 0; i < 25; ++i) ok += Echo(&ch, std::string(type) + std::to_string(t * 100 + i)) ? 1 : 0;
            });
        }
        for (auto& x : th) x.join();
        EXPECT_EQ(ok.load(), 100);
    }
    // short connections are closed after every call
    EXPECT_TRUE(s.WaitConnections(0, 5000) || s.Connections() <= 4);
}

TEST(RdmaHandshake, parallel_and_selective_channels_over_rdma) {
    InitSoft();
    RdmaServer a, b;
    ASSERT_GT(a.port, 0);
    ASSERT_GT(b.port, 0);
    auto sub = [](const std::string& addr) {
        Channel* c = new Channel;
        ChannelOptions o;
        o.use_rdma = true;
        o.timeout_ms = 3000;
        o.max_retry = 0;
        if (c->Init(addr.c_str(), &o) != 0) {
            delete c;
            return (Channel*)nullptr;
        }
        return c;
    };
    ParallelChannel pc;
    ParallelChannelOptions po;
    po.timeout_ms = 3000;
    pc.Init(&po);
    pc.AddChannel(sub(a.addr()), OWNS_CHANNEL, nullptr, nullptr);
    pc.AddChannel(sub(b.addr()), OWNS_CHANNEL, nullptr, nullptr);
    for (int i = 0; i < 20; ++i) EXPECT_TRUE(Echo(&pc, "pc" + std::to_string(i)));
    SelectiveChannel sc;
    ChannelOptions so;
    so.timeout_ms = 3000;
    so.max_retry = 2;
    ASSERT_EQ(sc.Init("rr", &so), 0);
    sc.AddChannel(sub(a.addr()));
    sc.AddChannel(sub(b.addr()));
    for (int i = 0; i < 20; ++i) EXPECT_TRUE(Echo(&sc, "sc" + std::to_string(i)));
    EXPECT_GE(a.Connections(), 1);
    EXPECT_GE(b.Connections(), 1);
}

TEST(RdmaHandshake, client_close_during_rpc) {
    InitSoft();
    RdmaServer s;
    ASSERT_GT(s.port, 0);
    {
        Channel ch;
        ChannelOptions o;
        o.use_rdma = true;
        o.timeout_ms = 300;  // the call gives up while the server still sleeps
        o.max_retry = 0;
        o.connection_group = "close-during";
        ASSERT_EQ(ch.Init(s.addr().c_str(), &o), 0);
        int code = 0;
        EXPECT_FALSE(Echo(&ch, "slow", &code, 600000));
        EXPECT_EQ(code, ERPCTIMEDOUT);
        SocketUniquePtr cs;
        if (Socket::Address(ch.server_id(), &cs) == 0) cs->SetFailed(ECLOSE, "client closes mid-call");
    }
    usleep(700000);  // the handler finishes and answers into a closed connection
    EXPECT_TRUE(ServerStillServes(s));
}

TEST(RdmaHandshake, server_close_during_rpc) {
    InitSoft();
    std::unique_ptr<RdmaServer> s(new RdmaServer);
    ASSERT_GT(s->port, 0);
    Channel ch;
    ChannelOptions o;
    o.use_rdma = true;
    o.timeout_ms = 5000;
    o.max_retry = 0;
    ASSERT_EQ(ch.Init(s->addr().c_str(), &o), 0);
    ASSERT_TRUE(Echo(&ch, "warm"));
    std::thread closer([&] {
        usleep(100000);
        std::vector<SocketId> conns;
        s->server.acceptor()->ListConnections(&conns);
        for (SocketId id : conns) {
            SocketUniquePtr p;
            if (Socket::Address(id, &p) == 0) p->SetFailed(ECLOSE, "server drops the connection");
        }
    });
    const int64_t t0 = monotonic_us();
    int code = 0;
    EXPECT_FALSE(Echo(&ch, "slow", &code, 1000000));
    EXPECT_LT(monotonic_us() - t0, 900000);  // failed with the connection, not at the timeout
    closer.join();
    // the channel revives the server through its health check and reconnects
    bool back = false;
    for (int i = 0; i < 100 && !back; ++i) {
        back = Echo(&ch, "reconnected");
        if (!back) usleep(100000);
    }
    EXPECT_TRUE_M(back, g_last_error);
}
