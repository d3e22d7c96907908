// Socket and concurrency-limiter suites (spirit of the reference's
// test/brpc_socket_unittest.cpp — socketpair fakes, partial writes through
// KeepWrite, EOVERCROWDED, versioned ids, health-check revive — and
// test/brpc_timeout_concurrency_limiter_unittest.cpp / auto limiter docs
// docs/cn/auto_concurrency_limiter.md:65).
#include <fcntl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "base/flags.h"
#include "base/time.h"
#include "mrpc/proto/echo.pb.h"
#include "net/socket.h"
#include "rpc/channel.h"
#include "rpc/concurrency_limiter.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "http/http_header.h"
#include "rpc/health_reporter.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

DECLARE_int64(socket_max_unwritten_bytes);
DECLARE_int32(health_check_interval);
DECLARE_string(health_check_path);
DECLARE_int32(health_check_timeout_ms);
DECLARE_int32(auto_cl_sample_window_size_ms);
DECLARE_int32(auto_cl_min_sample_count);
DECLARE_int32(auto_cl_max_sample_count);
DECLARE_int32(timeout_cl_default_timeout_ms);

using namespace mrpc;

namespace {

// A Socket over one end of an AF_UNIX socketpair; the other end is read by
// the test directly.
struct Pair {
    int peer = -1;
    SocketId id = INVALID_SOCKET_ID;
    Pair() {
        int fds[2];
        if (socketpair(AF_UNIX, SOCK_STREAM, 0, fds) != 0) return;
        fcntl(fds[0], F_SETFL, fcntl(fds[0], F_GETFL) | O_NONBLOCK);
        peer = fds[1];
        SocketOptions o;
        o.fd = fds[0];
        Socket::Create(o, &id);
    }
    ~Pair() {
        Socket::SetFailed(id);
        if (peer >= 0) close(peer);
    }
    // Reads exactly n bytes from the peer end (blocking).
    std::string read_n(size_t n) {
        std::string out;
        out.resize(n);
        size_t got = 0;
        while (got < n) {
            const ssize_t r = read(peer, &out[got], n - got);
            if (r <= 0) break;
            got += (size_t)r;
        }
        out.resize(got);
        return out;
    }
};

int write_str(SocketId id, const std::string& s, bool ignore_overcrowded = false) {
    SocketUniquePtr p;
    if (Socket::Address(id, &p) != 0) return -1;
    Buf b(s);
    WriteOptions wo;
    wo.ignore_eovercrowded = ignore_overcrowded;
    return p->Write(&b, &wo);
}

}  // namespace

TEST(Socket, concurrent_writers_keep_per_writer_order) {
    Pair p;
    ASSERT_GE(p.peer, 0);
    const int kThreads = 8, kMsgs = 500;
    std::vector<std::thread> ths;
    for (int t = 0; t < kThreads; ++t) {
        ths.emplace_back([&, t] {
            for (int i = 0; i < kMsgs; ++i) {
                char m[8];
                m[0] = (char)t;
                memcpy(m + 1, &i, 4);
                m[5] = m[6] = m[7] = 'x';
                EXPECT_EQ(write_str(p.id, std::string(m, 8)), 0);
            }
        });
    }
    const std::string all = p.read_n((size_t)kThreads * kMsgs * 8);
    for (auto& th : ths) th.join();
    ASSERT_EQ(all.size(), (size_t)kThreads * kMsgs * 8);
    std::vector<int> next(kThreads, 0);
    for (size_t off = 0; off < all.size(); off += 8) {
        const int t = all[off];
        int i;
        memcpy(&i, all.data() + off + 1, 4);
        ASSERT_TRUE(t >= 0 && t < kThreads);
        EXPECT_EQ(i, next[t]);  // a writer's messages never reorder or interleave
        next[t] = i + 1;
    }
}

TEST(Socket, partial_writes_complete_in_background) {
    // 8 MiB is far beyond the socketpair buffer: the first writer writes
    // what fits and KeepWrite finishes the rest once the peer drains.
    Pair p;
    std::string big(8 << 20, '\0');
    for (size_t i = 0; i < big.size(); ++i) big[i] = (char)(i * 7 + i / 4096);
    const int64_t t0 = monotonic_us();
    ASSERT_EQ(write_str(p.id, big), 0);
    EXPECT_LT(monotonic_us() - t0, 1000000);  // Write never blocks on the peer
    const std::string got = p.read_n(big.size());
    EXPECT_TRUE(got == big);
}

TEST(Socket, overcrowded_writes_fail_fast) {
    Pair p;
    const int64_t saved = FLAGS_socket_max_unwritten_bytes;
    FLAGS_socket_max_unwritten_bytes = 1 << 20;
    const std::string chunk(256 << 10, 'o');
    int ok = 0, rc = 0;
    for (int i = 0; i < 64 && rc == 0; ++i) {
        rc = write_str(p.id, chunk);
        if (rc == 0) ++ok;
    }
    EXPECT_EQ(rc, -1);
    EXPECT_EQ(errno, (int)EOVERCROWDED);
    EXPECT_GE(ok, 4);  // ~1 MiB queued (plus the socket buffer) before refusal
    // control traffic may bypass the limit
    EXPECT_EQ(write_str(p.id, "urgent", true), 0);
    FLAGS_socket_max_unwritten_bytes = saved;
    // draining the peer makes the socket writable again
    p.read_n((size_t)ok * chunk.size() + 6);
    EXPECT_EQ(write_str(p.id, "after"), 0);
    EXPECT_TRUE(p.read_n(5) == "after");
}

TEST(Socket, failed_ids_are_versioned) {
    Pair p;
    SocketUniquePtr ptr;
    ASSERT_EQ(Socket::Address(p.id, &ptr), 0);
    ptr.reset();
    Socket::SetFailed(p.id);
    EXPECT_NE(Socket::Address(p.id, &ptr), 0);
    EXPECT_NE(write_str(p.id, "x"), 0);
    // a new socket may reuse the slot, never the id
    Pair q;
    EXPECT_NE(q.id, p.id);
    EXPECT_EQ(Socket::Address(q.id, &ptr), 0);
}

TEST(Socket, peer_close_fails_the_socket) {
    // a client socket whose server goes away is failed by the read path
    EchoServiceImpl echo;
    Server s;
    s.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions so;
    ASSERT_EQ(s.Start("127.0.0.1:0", &so), 0);
    Channel ch;
    ChannelOptions co;
    co.timeout_ms = 1000;
    co.max_retry = 0;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(s.listen_port())).c_str(), &co), 0);
    example::EchoService_Stub stub(&ch);
    Controller c1;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("a");
    stub.Echo(&c1, &req, &res, nullptr);
    ASSERT_FALSE(c1.Failed());
    s.Stop(0);
    s.Join();
    Controller c2;
    stub.Echo(&c2, &req, &res, nullptr);
    EXPECT_TRUE(c2.Failed());
}

TEST(Socket, health_check_revives_the_connection) {
    // the server disappears and comes back on the same port: the failed
    // client socket is revived by its health check and calls resume
    const int saved = FLAGS_health_check_interval;
    FLAGS_health_check_interval = 1;
    EchoServiceImpl echo;
    std::unique_ptr<Server> s(new Server);
    s->AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions so;
    ASSERT_EQ(s->Start("127.0.0.1:0", &so), 0);
    const int port = s->listen_port();
    Channel ch;
    ChannelOptions co;
    co.timeout_ms = 500;
    co.max_retry = 0;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(port)).c_str(), &co), 0);
    example::EchoService_Stub stub(&ch);
    auto call = [&] {
        Controller c;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("hc");
        stub.Echo(&c, &req, &res, nullptr);
        return !c.Failed();
    };
    ASSERT_TRUE(call());
    s->Stop(0);
    s->Join();
    s.reset();
    EXPECT_FALSE(call());
    std::unique_ptr<Server> s2(new Server);
    s2->AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
    ASSERT_EQ(s2->Start(("127.0.0.1:" + std::to_string(port)).c_str(), &so), 0);
    bool revived = false;
    for (int i = 0; i < 40 && !revived; ++i) {
        usleep(100 * 1000);
        revived = call();
    }
    EXPECT_TRUE(revived);
    FLAGS_health_check_interval = saved;
}

namespace {
// /health answers 503 until `healthy` is set
struct FlipReporter : public HealthReporter {
    std::atomic<bool> healthy{false};
    std::atomic<int> reports{0};
    void GenerateReport(Controller* cntl, Closure* done) override {
        ClosureGuard g(done);
        reports.fetch_add(1);
        if (!healthy.load()) {
            cntl->http_response().set_status_code(503);
            cntl->response_attachment().append("not yet\n");
        } else {
            cntl->response_attachment().append("OK\n");
        }
    }
};
}  // namespace

// -health_check_path (reference: src/brpc/details/health_check.cpp:34-39):
// a connectable server is not healthy until GET path succeeds, so the
// socket stays failed (calls fail fast) while /health answers 503.
TEST(Socket, health_check_path_gates_revive) {
    const int saved = FLAGS_health_check_interval;
    const std::string saved_path = FLAGS_health_check_path;
    FLAGS_health_check_interval = 1;
    FLAGS_health_check_path = "/health";
    FLAGS_health_check_timeout_ms = 300;
    EchoServiceImpl echo;
    std::unique_ptr<Server> s(new Server);
    s->AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions so;
    ASSERT_EQ(s->Start("127.0.0.1:0", &so), 0);
    const int port = s->listen_port();
    Channel ch;
    ChannelOptions co;
    co.timeout_ms = 500;
    co.max_retry = 0;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(port)).c_str(), &co), 0);
    example::EchoService_Stub stub(&ch);
    auto call = [&] {
        Controller c;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("hc");
        stub.Echo(&c, &req, &res, nullptr);
        return !c.Failed();
    };
    ASSERT_TRUE(call());
    s->Stop(0);
    s->Join();
    s.reset();
    EXPECT_FALSE(call());
    FlipReporter reporter;
    std::unique_ptr<Server> s2(new Server);
    s2->AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
    ServerOptions so2;
    so2.health_reporter = &reporter;
    ASSERT_EQ(s2->Start(("127.0.0.1:" + std::to_string(port)).c_str(), &so2), 0);
    // connectable but unhealthy: checked, and still not revived
    const int64_t t0 = monotonic_us();
    while (reporter.reports.load() < 2 && monotonic_us() - t0 < 5000000) usleep(50 * 1000);
    EXPECT_GE(reporter.reports.load(), 2);
    EXPECT_FALSE(call());
    reporter.healthy.store(true);
    bool revived = false;
    for (int i = 0; i < 40 && !revived; ++i) {
        usleep(100 * 1000);
        revived = call();
    }
    EXPECT_TRUE(revived);
    FLAGS_health_check_interval = saved;
    FLAGS_health_check_path = saved_path;
    FLAGS_health_check_timeout_ms = 500;
}

// ------------------------------------------------------------------ limiters
TEST(Limiter, adaptive_max_concurrency_types) {
    EXPECT_EQ(AdaptiveMaxConcurrency(0).type(), std::string("unlimited"));
    EXPECT_EQ(AdaptiveMaxConcurrency(10).type(), std::string("constant"));
    EXPECT_EQ(AdaptiveMaxConcurrency(10).max_concurrency(), 10);
    EXPECT_EQ(AdaptiveMaxConcurrency(std::string("25")).max_concurrency(), 25);
    EXPECT_EQ(AdaptiveMaxConcurrency(std::string("auto")).type(), std::string("auto"));
    EXPECT_EQ(AdaptiveMaxConcurrency(std::string("timeout")).type(), std::string("timeout"));
    EXPECT_TRUE(CreateConcurrencyLimiter(AdaptiveMaxConcurrency(0)) == nullptr);
    EXPECT_TRUE(CreateConcurrencyLimiter(AdaptiveMaxConcurrency(std::string("bogus"))) == nullptr);
}

TEST(Limiter, constant_rejects_above_max) {
    std::unique_ptr<ConcurrencyLimiter> l(CreateConcurrencyLimiter(AdaptiveMaxConcurrency(5)));
    ASSERT_TRUE(l != nullptr);
    EXPECT_TRUE(l->OnRequested(5, nullptr));
    EXPECT_FALSE(l->OnRequested(6, nullptr));
    EXPECT_EQ(l->MaxConcurrency(), 5);
}

TEST(Limiter, auto_tracks_littles_law) {
    // a server with 1 ms no-load latency answering 20k qps: the auto limiter
    // settles near min_latency * max_qps * (1 + explore) = 20..26
    FLAGS_auto_cl_sample_window_size_ms = 50;
    FLAGS_auto_cl_min_sample_count = 50;
    FLAGS_auto_cl_max_sample_count = 100;
    std::unique_ptr<ConcurrencyLimiter> l(CreateConcurrencyLimiter(AdaptiveMaxConcurrency(std::string("auto"))));
    ASSERT_TRUE(l != nullptr);
    for (int w = 0; w < 30; ++w) {
        for (int i = 0; i < 100; ++i) {
            l->OnResponded(0, 1000);
            if (i % 20 == 19) usleep(1000);  // 100 samples per ~5 ms = 20k qps
        }
    }
    const int m = l->MaxConcurrency();
    fprintf(stderr, "auto limiter settled at %d\n", m);
    EXPECT_GE(m, 8);
    EXPECT_LE(m, 60);
    EXPECT_TRUE(l->OnRequested(m, nullptr));
    EXPECT_FALSE(l->OnRequested(m + 1, nullptr));
}

TEST(Limiter, auto_backs_off_when_latency_rises) {
    FLAGS_auto_cl_sample_window_size_ms = 50;
    FLAGS_auto_cl_min_sample_count = 50;
    FLAGS_auto_cl_max_sample_count = 100;
    std::unique_ptr<ConcurrencyLimiter> l(CreateConcurrencyLimiter(AdaptiveMaxConcurrency(std::string("auto"))));
    auto feed = [&](int64_t lat_us, int windows, int sleep_every) {
        for (int w = 0; w < windows; ++w) {
            for (int i = 0; i < 100; ++i) {
                l->OnResponded(0, lat_us);
                if (i % sleep_every == sleep_every - 1) usleep(1000);
            }
        }
    };
    feed(1000, 20, 20);
    const int before = l->MaxConcurrency();
    // overload: latency x5 and throughput halves
    feed(5000, 20, 10);
    const int after = l->MaxConcurrency();
    fprintf(stderr, "auto limiter %d -> %d under overload\n", before, after);
    EXPECT_LE(after, before);
}

TEST(Limiter, timeout_limiter_rejects_what_cannot_finish_in_time) {
    FLAGS_timeout_cl_default_timeout_ms = 50;
    std::unique_ptr<ConcurrencyLimiter> l(CreateConcurrencyLimiter(AdaptiveMaxConcurrency(std::string("timeout"))));
    ASSERT_TRUE(l != nullptr);
    for (int i = 0; i < 200; ++i) l->OnResponded(0, 10000);  // avg latency -> 10 ms
    // queueing estimate cur * 10ms / 8 must stay within the 50 ms budget
    EXPECT_TRUE(l->OnRequested(40, nullptr));
    EXPECT_FALSE(l->OnRequested(41, nullptr));
    // failed calls do not move the estimate
    for (int i = 0; i < 200; ++i) l->OnResponded(ETIMEDOUT, 1);
    EXPECT_FALSE(l->OnRequested(41, nullptr));
    FLAGS_timeout_cl_default_timeout_ms = 500;
}

TEST(Limiter, server_method_limit_end_to_end) {
    // "constant" per-method limit through the server: a burst of slow calls
    // beyond the limit gets ELIMIT, the rest succeeds
    EchoServiceImpl echo;
    Server s;
    s.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
    ASSERT_EQ(s.SetMaxConcurrencyOf("example.EchoService.Echo", 4), 0);
    ServerOptions so;
    ASSERT_EQ(s.Start("127.0.0.1:0", &so), 0);
    Channel ch;
    ChannelOptions co;
    co.timeout_ms = 3000;
    co.max_retry = 0;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(s.listen_port())).c_str(), &co), 0);
    std::atomic<int> ok{0}, limited{0};
    std::vector<std::thread> ths;
    for (int t = 0; t < 12; ++t) {
        ths.emplace_back([&] {
            example::EchoService_Stub stub(&ch);
            Controller c;
            example::EchoRequest req;
            example::EchoResponse res;
            req.set_message("slow");
            req.set_sleep_us(200000);
            stub.Echo(&c, &req, &res, nullptr);
            if (!c.Failed()) ok.fetch_add(1);
            else if (c.ErrorCode() == ELIMIT) limited.fetch_add(1);
        });
    }
    for (auto& th : ths) th.join();
    EXPECT_EQ(ok.load() + limited.load(), 12);
    EXPECT_GE(limited.load(), 1);
    EXPECT_LE(ok.load(), 8);
}
