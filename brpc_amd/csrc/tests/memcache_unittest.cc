// Memcache binary client against an in-process fake memcached (blocking
// sockets on a plain thread) — spirit of test/brpc_memcache_unittest.cpp,
// which needs a real memcached.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <map>
#include <thread>

#include "policy/authenticators.h"
#include "redis/memcache.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

struct FakeMemcached {
    int lfd = -1;
    int port = 0;
    std::thread th;
    std::atomic<bool> stop{false};
    std::map<std::string, std::pair<std::string, uint32_t>> kv;
    uint64_t cas = 1;
    // couchbase bucket auth: when set, every connection must start with a
    // SASL PLAIN for it (opcode 0x21), else commands are refused
    std::string bucket, password;
    std::atomic<int> sasl_ok{0}, sasl_bad{0}, unauthenticated{0};

    FakeMemcached() {
        lfd = socket(AF_INET, SOCK_STREAM, 0);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        bind(lfd, (sockaddr*)&a, sizeof(a));
        socklen_t l = sizeof(a);
        getsockname(lfd, (sockaddr*)&a, &l);
        port = ntohs(a.sin_port);
        listen(lfd, 4);
        th = std::thread([this] { serve(); });
    }
    ~FakeMemcached() {
        stop = true;
        shutdown(lfd, SHUT_RDWR);
        close(lfd);
        th.join();
    }
    static bool readn(int fd, void* p, size_t n) {
        char* c = (char*)p;
        while (n) {
            ssize_t r = read(fd, c, n);
            if (r <= 0) return false;
            c += r;
            n -= r;
        }
        return true;
    }
    static uint64_t be(const unsigned char* p, int n) {
        uint64_t v = 0;
        for (int i = 0; i < n; ++i) v = (v << 8) | p[i];
        return v;
    }
    static void put(std::string* s, uint64_t v, int n) {
        for (int i = n - 1; i >= 0; --i) s->push_back((char)(v >> (8 * i)));
    }
    void reply(int fd, uint8_t op, uint16_t status, const std::string& ext, const std::string& value, uint64_t c) {
        std::string s;
        s.push_back((char)0x81);
        s.push_back((char)op);
        put(&s, 0, 2);
        s.push_back((char)ext.size());
        s.push_back(0);
        put(&s, status, 2);
        put(&s, ext.size() + value.size(), 4);
        put(&s, 0, 4);
        put(&s, c, 8);
        s += ext + value;
        (void)!write(fd, s.data(), s.size());
    }
    void serve() {
        while (!stop) {
            int fd = accept(lfd, nullptr, nullptr);
            if (fd < 0) return;
            unsigned char h[24];
            bool authed = bucket.empty();
            while (readn(fd, h, 24)) {
                const uint8_t op = h[1];
                const uint16_t keylen = (uint16_t)be(h + 2, 2);
                const uint8_t extlen = h[4];
                const uint32_t body = (uint32_t)be(h + 8, 4);
                std::string b(body, '\0');
                if (body && !readn(fd, &b[0], body)) break;
                const std::string ext = b.substr(0, extlen), key = b.substr(extlen, keylen),
                                  val = b.substr(extlen + keylen);
                if (op == 0x21) {  // SASL auth: "PLAIN", "<bucket>\0<bucket>\0<password>"
                    const std::string want = bucket + std::string(1, '\0') + bucket + std::string(1, '\0') + password;
                    authed = key == "PLAIN" && val == want;
                    (authed ? sasl_ok : sasl_bad).fetch_add(1);
                    reply(fd, op, authed ? 0 : 0x20, "", authed ? "Authenticated" : "Auth failure", 0);
                    continue;
                }
                if (!authed) {
                    unauthenticated.fetch_add(1);
                    reply(fd, op, 0x20, "", "Auth required", 0);
                    continue;
                }
                if (op == 0x01) {  // set
                    kv[key] = {val, (uint32_t)be((const unsigned char*)ext.data(), 4)};
                    reply(fd, op, 0, "", "", ++cas);
                } else if (op == 0x00) {  // get
                    auto it = kv.find(key);
                    if (it == kv.end()) {
                        reply(fd, op, 1, "", "Not found", 0);
                    } else {
                        std::string fl;
                        put(&fl, it->second.second, 4);
                        reply(fd, op, 0, fl, it->second.first, cas);
                    }
                } else if (op == 0x05) {  // incr
                    const uint64_t delta = be((const unsigned char*)ext.data(), 8);
                    const uint64_t init = be((const unsigned char*)ext.data() + 8, 8);
                    auto it = kv.find(key);
                    uint64_t v = it == kv.end() ? init : strtoull(it->second.first.c_str(), nullptr, 10) + delta;
                    kv[key] = {std::to_string(v), 0};
                    std::string out;
                    put(&out, v, 8);
                    reply(fd, op, 0, "", out, ++cas);
                } else if (op == 0x04) {  // delete
                    reply(fd, op, kv.erase(key) ? 0 : 1, "", "", 0);
                } else if (op == 0x0b) {
                    reply(fd, op, 0, "", "1.6.fake", 0);
                } else {
                    reply(fd, op, 0x81, "", "Unknown command", 0);
                }
            }
            close(fd);
        }
    }
};

}  // namespace

TEST(Memcache, pipelined_ops) {
    FakeMemcached mc;
    Channel ch;
    ChannelOptions co;
    co.protocol = "memcache";
    co.timeout_ms = 3000;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(mc.port)).c_str(), &co), 0);
    MemcacheRequest req;
    req.Set("hello", "world", 0xdead, 0, 0);
    req.Get("hello");
    req.Get("nope");
    req.Increment("ctr", 5, 100, 0);
    req.Increment("ctr", 5, 100, 0);
    req.Delete("hello");
    req.Version();
    MemcacheResponse res;
    Controller cntl;
    ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
    ASSERT_FALSE(cntl.Failed());
    uint64_t cas = 0;
    EXPECT_TRUE(res.PopSet(&cas));
    EXPECT_GT(cas, 0u);
    std::string v;
    uint32_t flags = 0;
    EXPECT_TRUE(res.PopGet(&v, &flags, nullptr));
    EXPECT_EQ(v, "world");
    EXPECT_EQ(flags, 0xdeadu);
    EXPECT_FALSE(res.PopGet(&v, nullptr, nullptr));
    uint64_t n = 0;
    EXPECT_TRUE(res.PopIncrement(&n, nullptr));
    EXPECT_EQ(n, 100u);
    EXPECT_TRUE(res.PopIncrement(&n, nullptr));
    EXPECT_EQ(n, 105u);
    EXPECT_TRUE(res.PopDelete());
    std::string ver;
    EXPECT_TRUE(res.PopVersion(&ver));
    EXPECT_EQ(ver, "1.6.fake");
}

static std::string mc_header(uint8_t magic, uint8_t op, uint16_t keylen, uint8_t extlen, uint16_t status,
                             uint32_t body, uint64_t cas) {
    std::string s;
    s.push_back((char)magic);
    s.push_back((char)op);
    s.push_back((char)(keylen >> 8));
    s.push_back((char)keylen);
    s.push_back((char)extlen);
    s.push_back(0);
    s.push_back((char)(status >> 8));
    s.push_back((char)status);
    for (int i = 3; i >= 0; --i) s.push_back((char)(body >> (8 * i)));
    for (int i = 0; i < 4; ++i) s.push_back(0);
    for (int i = 7; i >= 0; --i) s.push_back((char)(cas >> (8 * i)));
    return s;
}

TEST(Memcache, request_wire_format) {
    MemcacheRequest req;
    ASSERT_TRUE(req.Set("k", "vv", 0x01020304, 60, 7));
    ASSERT_TRUE(req.Touch("k", 30));
    ASSERT_TRUE(req.Decrement("n", 2, 9, 0));
    ASSERT_TRUE(req.Flush(0));
    EXPECT_EQ(req.op_count(), 4);
    const std::string w = req.raw().to_string();
    // SET: extras = flags(4) + exptime(4); key; value; cas in the header
    std::string want = mc_header(0x80, 0x01, 1, 8, 0, 8 + 1 + 2, 7);
    want += std::string("\x01\x02\x03\x04\x00\x00\x00\x3c", 8) + "k" + "vv";
    // TOUCH: extras = exptime(4)
    want += mc_header(0x80, 0x1c, 1, 4, 0, 4 + 1, 0) + std::string("\x00\x00\x00\x1e", 4) + "k";
    // DECR: extras = delta(8) + initial(8) + exptime(4)
    want += mc_header(0x80, 0x06, 1, 20, 0, 20 + 1, 0) + std::string("\0\0\0\0\0\0\0\x02", 8) +
            std::string("\0\0\0\0\0\0\0\x09", 8) + std::string("\0\0\0\0", 4) + "n";
    // FLUSH: extras = expiration(4)
    want += mc_header(0x80, 0x08, 0, 4, 0, 4, 0) + std::string("\0\0\0\0", 4);
    ASSERT_EQ(w.size(), want.size());
    EXPECT_TRUE(w == want);
    // keys longer than the protocol's 250 bytes are refused
    EXPECT_FALSE(req.Get(std::string(251, 'x')));
    EXPECT_EQ(req.op_count(), 4);
}

TEST(Memcache, response_errors_and_partial_input) {
    std::string wire = mc_header(0x81, 0x01, 0, 0, 0, 0, 11);                                // SET ok
    wire += mc_header(0x81, 0x02, 0, 0, MC_STATUS_KEY_EEXISTS, 10, 0) + "Data exists";        // ADD fails
    wire.erase(wire.size() - 1);  // "Data exist" (body length 10)
    wire += mc_header(0x81, 0x0b, 0, 0, 0, 5, 0) + "1.6.x";                                  // VERSION
    MemcacheResponse res;
    Buf in;
    for (size_t i = 0; i + 1 < wire.size(); i += 7) {  // arrives in 7-byte pieces
        in.append(wire.data() + i, std::min<size_t>(7, wire.size() - 1 - i));
        EXPECT_EQ(res.ConsumePartial(&in, 3), 0);
    }
    in.append(wire.data() + wire.size() - 1, 1);
    ASSERT_EQ(res.ConsumePartial(&in, 3), 1);
    uint64_t cas = 0;
    EXPECT_TRUE(res.PopSet(&cas));
    EXPECT_EQ(cas, 11u);
    EXPECT_FALSE(res.PopAdd(&cas));
    EXPECT_FALSE(res.LastError().empty());
    std::string v;
    EXPECT_TRUE(res.PopVersion(&v));
    EXPECT_EQ(v, "1.6.x");
    EXPECT_EQ(res.result_count(), 0);
    // popping the wrong kind fails instead of misreading the result
    MemcacheResponse r2;
    Buf in2;
    in2.append(mc_header(0x81, 0x04, 0, 0, 0, 0, 0));
    ASSERT_EQ(r2.ConsumePartial(&in2, 1), 1);
    EXPECT_FALSE(r2.PopSet(&cas));
    // a request magic in a response stream is malformed
    MemcacheResponse r3;
    Buf in3;
    in3.append(mc_header(0x80, 0x01, 0, 0, 0, 0, 0));
    EXPECT_LT(r3.ConsumePartial(&in3, 1), 0);
}

TEST(Memcache, couchbase_bucket_sasl_once_per_connection) {
    FakeMemcached mc;
    mc.bucket = "travel";
    mc.password = "pw";
    policy::CouchbaseAuthenticator auth("travel", "pw");
    Channel ch;
    ChannelOptions opt;
    opt.protocol = "memcache";
    opt.auth = &auth;
    opt.timeout_ms = 3000;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(mc.port)).c_str(), &opt), 0);
    for (int i = 0; i < 10; ++i) {
        MemcacheRequest req;
        MemcacheResponse res;
        Controller cntl;
        ASSERT_TRUE(req.Set("k" + std::to_string(i), "v" + std::to_string(i), 0, 0, 0));
        ASSERT_TRUE(req.Get("k" + std::to_string(i)));
        ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        std::string v;
        uint32_t flags = 0;
        uint64_t c = 0;
        ASSERT_TRUE(res.PopSet(&c));
        ASSERT_TRUE(res.PopGet(&v, &flags, &c));
        EXPECT_EQ(v, "v" + std::to_string(i));
    }
    EXPECT_EQ(mc.sasl_ok.load(), 1);  // one connection, one SASL exchange
    EXPECT_EQ(mc.sasl_bad.load(), 0);
    EXPECT_EQ(mc.unauthenticated.load(), 0);
    // wrong bucket password: the connection fails instead of running the ops
    // (a second fake: the first one serves one connection at a time)
    FakeMemcached mc2;
    mc2.bucket = "travel";
    mc2.password = "pw";
    policy::CouchbaseAuthenticator bad("travel", "nope");
    Channel ch2;
    opt.auth = &bad;
    opt.max_retry = 0;
    ASSERT_EQ(ch2.Init(("127.0.0.1:" + std::to_string(mc2.port)).c_str(), &opt), 0);
    MemcacheRequest req;
    MemcacheResponse res;
    Controller cntl;
    ASSERT_TRUE(req.Get("k1"));
    ch2.CallMethod(nullptr, &cntl, &req, &res, nullptr);
    EXPECT_TRUE(cntl.Failed());
    EXPECT_EQ(mc2.sasl_bad.load(), 1);
}
