// Socket depth, round 6 (spirit of the reference's test/brpc_socket_unittest.cpp:
// write ordering through KeepWrite, partial writes, SetFailed semantics with
// queued data and waiters, error delivery to the write's call id, and the
// socket map): all over AF_UNIX socketpairs whose far end the test reads.
#include <fcntl.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "base/flags.h"
#include "base/time.h"
#include "fiber/call_id.h"
#include "fiber/fiber.h"
#include "net/socket.h"
#include "rpc/errno.h"
#include "tests/test.h"

DECLARE_int64(socket_max_unwritten_bytes);

using namespace mrpc;

namespace {

struct SockPair {
    int peer = -1;
    SocketId id = INVALID_SOCKET_ID;
    explicit SockPair(int sndbuf = 0) {
        int fds[2];
        if (socketpair(AF_UNIX, SOCK_STREAM, 0, fds) != 0) return;
        if (sndbuf > 0) setsockopt(fds[0], SOL_SOCKET, SO_SNDBUF, &sndbuf, sizeof(sndbuf));
        fcntl(fds[0], F_SETFL, fcntl(fds[0], F_GETFL) | O_NONBLOCK);
        peer = fds[1];
        SocketOptions o;
        o.fd = fds[0];
        Socket::Create(o, &id);
    }
    ~SockPair() {
        Socket::SetFailed(id);
        if (peer >= 0) close(peer);
    }
    std::string read_n(size_t n, int timeout_ms = 5000) {
        std::string out(n, '\0');
        size_t got = 0;
        const int64_t deadline = monotonic_us() + (int64_t)timeout_ms * 1000;
        while (got < n && monotonic_us() < deadline) {
            pollfd p{peer, POLLIN, 0};
            if (poll(&p, 1, 50) <= 0) continue;
            const ssize_t r = read(peer, &out[got], n - got);
            if (r <= 0) break;
            got += (size_t)r;
        }
        out.resize(got);
        return out;
    }
    // Whatever arrives within timeout_ms.
    std::string read_some(int timeout_ms) {
        std::string out;
        char buf[65536];
        const int64_t deadline = monotonic_us() + (int64_t)timeout_ms * 1000;
        while (monotonic_us() < deadline) {
            pollfd p{peer, POLLIN, 0};
            if (poll(&p, 1, 20) <= 0) continue;
            const ssize_t r = read(peer, buf, sizeof(buf));
            if (r <= 0) break;
            out.append(buf, (size_t)r);
        }
        return out;
    }
};

int write_buf(SocketId id, Buf* b, const WriteOptions* wo = nullptr) {
    SocketUniquePtr p;
    if (Socket::Address(id, &p) != 0) return -1;
    return p->Write(b, wo);
}

int write_str(SocketId id, const std::string& s, const WriteOptions* wo = nullptr) {
    Buf b(s);
    return write_buf(id, &b, wo);
}

std::string pattern(size_t n, int seed) {
    std::string s(n, '\0');
    for (size_t i = 0; i < n; ++i) s[i] = (char)((i * 131 + seed * 7 + (i >> 10)) & 0xff);
    return s;
}

}  // namespace

TEST(SocketMore, empty_write_is_a_no_op) {
    SockPair p;
    Buf empty;
    EXPECT_EQ(write_buf(p.id, &empty), 0);
    EXPECT_EQ(write_str(p.id, "x"), 0);
    EXPECT_EQ(p.read_n(1), "x");
}

TEST(SocketMore, write_consumes_the_callers_buf) {
    SockPair p;
    Buf b(std::string("hello"));
    ASSERT_EQ(write_buf(p.id, &b), 0);
    EXPECT_TRUE(b.empty());  // the data moved into the write queue
    EXPECT_EQ(p.read_n(5), "hello");
}

TEST(SocketMore, multi_block_buf_arrives_contiguously) {
    SockPair p;
    Buf b;
    std::string want;
    for (int i = 0; i < 100; ++i) {
        const std::string piece = pattern(777 + i, i);
        b.append(piece);
        want += piece;
    }
    ASSERT_EQ(write_buf(p.id, &b), 0);
    EXPECT_TRUE(p.read_n(want.size()) == want);
}

TEST(SocketMore, user_data_blocks_are_written_zero_copy) {
    SockPair p;
    static std::atomic<int> freed{0};
    char* mem = new char[10000];
    memset(mem, 'u', 10000);
    Buf b;
    b.append_user_data(mem, 10000, [](void* d, void*) {
        delete[] static_cast<char*>(d);
        freed.fetch_add(1);
    });
    ASSERT_EQ(write_buf(p.id, &b), 0);
    EXPECT_EQ(p.read_n(10000), std::string(10000, 'u'));
    for (int i = 0; i < 200 && freed.load() == 0; ++i) usleep(1000);
    EXPECT_EQ(freed.load(), 1);  // released once written
}

TEST(SocketMore, small_sndbuf_large_write_drains_in_order) {
    SockPair p(4096);
    const std::string a = pattern(1 << 20, 1), b = pattern(300000, 2);
    ASSERT_EQ(write_str(p.id, a), 0);
    ASSERT_EQ(write_str(p.id, b), 0);
    const std::string got = p.read_n(a.size() + b.size());
    EXPECT_TRUE(got == a + b);
}

TEST(SocketMore, many_fibers_write_without_interleaving) {
    SockPair p;
    const int kFibers = 32, kMsgs = 50, kLen = 100;
    std::atomic<int> done{0};
    std::vector<fiber::fiber_t> ts(kFibers);
    struct Arg {
        SocketId id;
        int idx;
        std::atomic<int>* done;
    };
    std::vector<Arg> args(kFibers);
    for (int i = 0; i < kFibers; ++i) {
        args[i] = Arg{p.id, i, &done};
        fiber::start_background(&ts[i], nullptr,
                                [](void* x) -> void* {
                                    Arg* a = static_cast<Arg*>(x);
                                    for (int m = 0; m < kMsgs; ++m) {
                                        std::string msg(kLen, (char)('A' + a->idx % 26));
                                        msg[0] = (char)a->idx;
                                        memcpy(&msg[1], &m, 4);
                                        write_str(a->id, msg);
                                    }
                                    a->done->fetch_add(1);
                                    return nullptr;
                                },
                                &args[i]);
    }
    const std::string all = p.read_n((size_t)kFibers * kMsgs * kLen);
    for (auto t : ts) fiber::join(t, nullptr);
    ASSERT_EQ(all.size(), (size_t)kFibers * kMsgs * kLen);
    std::vector<int> next(kFibers, 0);
    for (size_t off = 0; off < all.size(); off += kLen) {
        const int f = (unsigned char)all[off];
        int m;
        memcpy(&m, &all[off + 1], 4);
        ASSERT_TRUE(f < kFibers);
        EXPECT_EQ(m, next[f]);
        next[f] = m + 1;
        // the body of one message is never split by another
        EXPECT_EQ(all[off + kLen - 1], (char)('A' + f % 26));
    }
    EXPECT_EQ(done.load(), kFibers);
}

TEST(SocketMore, set_failed_refuses_later_writes_with_the_error) {
    SockPair p;
    SocketUniquePtr ptr;
    ASSERT_EQ(Socket::Address(p.id, &ptr), 0);
    ptr->SetFailed(ECLOSE, "closed by test");
    EXPECT_TRUE(ptr->Failed());
    Buf b(std::string("late"));
    WriteOptions wo;
    EXPECT_EQ(ptr->Write(&b, &wo), -1);
    EXPECT_EQ(errno, (int)ECLOSE);
}

TEST(SocketMore, set_failed_twice_keeps_the_first_error) {
    SockPair p;
    SocketUniquePtr ptr;
    ASSERT_EQ(Socket::Address(p.id, &ptr), 0);
    EXPECT_EQ(ptr->SetFailed(ECLOSE, "first"), 0);
    EXPECT_EQ(ptr->SetFailed(EFAILEDSOCKET, "second"), -1);
    Buf b(std::string("x"));
    EXPECT_EQ(ptr->Write(&b), -1);
    EXPECT_EQ(errno, (int)ECLOSE);
}

TEST(SocketMore, write_error_reaches_the_call_id) {
    SockPair p;
    fiber::CallId cid;
    struct Seen {
        std::atomic<int> code{0};
    } seen;
    ASSERT_EQ(fiber::call_id_create(&cid, &seen,
                                    [](fiber::CallId id, void* data, int ec, const std::string&) -> int {
                                        static_cast<Seen*>(data)->code.store(ec);
                                        return fiber::call_id_unlock_and_destroy(id);
                                    }),
              0);
    SocketUniquePtr ptr;
    ASSERT_EQ(Socket::Address(p.id, &ptr), 0);  // our reference keeps it alive after the failure
    ptr->SetFailed(EFAILEDSOCKET, "failed by test");
    Buf b(std::string("doomed"));
    WriteOptions wo;
    wo.id_wait = cid;
    EXPECT_EQ(ptr->Write(&b, &wo), -1);
    for (int i = 0; i < 500 && seen.code.load() == 0; ++i) usleep(1000);
    EXPECT_NE(seen.code.load(), 0);
}

TEST(SocketMore, address_of_invalid_id_fails) {
    SocketUniquePtr ptr;
    EXPECT_NE(Socket::Address(INVALID_SOCKET_ID, &ptr), 0);
    EXPECT_NE(Socket::Address((SocketId)0x7fffffff12345678ull, &ptr), 0);
}

TEST(SocketMore, unwritten_bytes_drop_to_zero_after_drain) {
    SockPair p(4096);
    SocketUniquePtr ptr;
    ASSERT_EQ(Socket::Address(p.id, &ptr), 0);
    const std::string big = pattern(2 << 20, 3);
    Buf b(big);
    ASSERT_EQ(ptr->Write(&b), 0);
    EXPECT_GT(ptr->unwritten_bytes(), 0);
    EXPECT_TRUE(p.read_n(big.size()) == big);
    for (int i = 0; i < 500 && ptr->unwritten_bytes() != 0; ++i) usleep(1000);
    EXPECT_EQ(ptr->unwritten_bytes(), 0);
}

TEST(SocketMore, overcrowded_limit_is_reloadable) {
    SockPair p(4096);
    const int64_t saved = FLAGS_socket_max_unwritten_bytes;
    FLAGS_socket_max_unwritten_bytes = 64 << 10;
    const std::string chunk(48 << 10, 'c');
    EXPECT_EQ(write_str(p.id, chunk), 0);
    int rc = 0;
    for (int i = 0; i < 8 && rc == 0; ++i) rc = write_str(p.id, chunk);
    EXPECT_EQ(rc, -1);
    // raising the limit admits more without draining
    FLAGS_socket_max_unwritten_bytes = 64 << 20;
    EXPECT_EQ(write_str(p.id, chunk), 0);
    FLAGS_socket_max_unwritten_bytes = saved;
    p.read_some(300);
}

TEST(SocketMore, background_write_option_returns_immediately) {
    SockPair p;
    WriteOptions wo;
    wo.write_in_background = true;
    const std::string s = pattern(100000, 9);
    ASSERT_EQ(write_str(p.id, s, &wo), 0);
    EXPECT_TRUE(p.read_n(s.size()) == s);
}

TEST(SocketMore, background_and_inline_writes_keep_call_order) {
    SockPair p;
    WriteOptions bg;
    bg.write_in_background = true;
    std::string want;
    for (int i = 0; i < 200; ++i) {
        const std::string piece = "[" + std::to_string(i) + "]";
        want += piece;
        ASSERT_EQ(write_str(p.id, piece, i % 3 == 0 ? &bg : nullptr), 0);
    }
    EXPECT_EQ(p.read_n(want.size()), want);
}

TEST(SocketMore, shutdown_write_after_half_closes) {
    SockPair p;
    WriteOptions wo;
    wo.shutdown_write_after = true;
    ASSERT_EQ(write_str(p.id, "bye", &wo), 0);
    EXPECT_EQ(p.read_n(3), "bye");
    // the peer then sees EOF
    char c;
    pollfd pf{p.peer, POLLIN, 0};
    ASSERT_GT(poll(&pf, 1, 2000), 0);
    EXPECT_EQ(read(p.peer, &c, 1), 0);
}

TEST(SocketMore, description_names_the_socket) {
    SockPair p;
    SocketUniquePtr ptr;
    ASSERT_EQ(Socket::Address(p.id, &ptr), 0);
    const std::string d = ptr->description();
    EXPECT_FALSE(d.empty());
    EXPECT_GE(ptr->fd(), 0);
}
