// Redis client/server over RESP (spirit of the reference's
// test/brpc_redis_unittest.cpp): pipelined commands, reply types, server
// command handlers and MULTI/EXEC.
#include <map>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

#include "base/time.h"
#include "policy/authenticators.h"
#include "redis/redis.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/server.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

struct KV {
    std::mutex mu;
    std::map<std::string, std::string> m;
};

class SetHandler : public RedisCommandHandler {
public:
    explicit SetHandler(KV* kv) : _kv(kv) {}
    Result Run(const std::vector<std::string>& args, RedisReply* out, bool) override {
        if (args.size() != 3) {
            out->SetError("ERR wrong number of arguments for 'set'");
            return OK;
        }
        std::lock_guard<std::mutex> g(_kv->mu);
        _kv->m[args[1]] = args[2];
        out->SetStatus("OK");
        return OK;
    }

private:
    KV* _kv;
};

class GetHandler : public RedisCommandHandler {
public:
    explicit GetHandler(KV* kv) : _kv(kv) {}
    Result Run(const std::vector<std::string>& args, RedisReply* out, bool) override {
        std::lock_guard<std::mutex> g(_kv->mu);
        auto it = _kv->m.find(args.size() > 1 ? args[1] : "");
        if (it == _kv->m.end()) out->SetNil();
        else out->SetString(it->second);
        return OK;
    }

private:
    KV* _kv;
};

class IncrHandler : public RedisCommandHandler {
public:
    explicit IncrHandler(KV* kv) : _kv(kv) {}
    Result Run(const std::vector<std::string>& args, RedisReply* out, bool) override {
        std::lock_guard<std::mutex> g(_kv->mu);
        const int64_t v = atoll(_kv->m[args[1]].c_str()) + 1;
        _kv->m[args[1]] = std::to_string(v);
        out->SetInteger(v);
        return OK;
    }

private:
    KV* _kv;
};

// MULTI the reference's way (test/brpc_redis_unittest.cpp MultiCommandHandler):
// "multi" answers +OK and returns CONTINUE; its transaction handler answers
// +QUEUED (CONTINUE) for every command, a nested MULTI with an error, and
// runs the queue at EXEC, returning OK with one reply per queued command.
class MultiHandler : public RedisCommandHandler {
public:
    explicit MultiHandler(RedisService* svc) : _svc(svc) {}
    Result Run(const std::vector<std::string>&, RedisReply* out, bool) override {
        out->SetStatus("OK");
        return CONTINUE;
    }
    RedisCommandHandler* NewTransactionHandler() override {
        struct Tx : public RedisCommandHandler {
            RedisService* svc;
            std::vector<std::vector<std::string>> queued;
            Result Run(const std::vector<std::string>& args, RedisReply* out, bool) override {
                if (args[0] == "multi") {
                    out->SetError("ERR MULTI calls can not be nested");
                    return CONTINUE;
                }
                if (args[0] == "exec") {
                    out->SetArray(queued.size());
                    for (size_t i = 0; i < queued.size(); ++i) {
                        RedisCommandHandler* h = svc->FindCommandHandler(queued[i][0]);
                        if (h) h->Run(queued[i], &(*out)[i], true);
                        else (*out)[i].SetError("ERR unknown command");
                    }
                    return OK;
                }
                queued.push_back(args);
                out->SetStatus("QUEUED");
                return CONTINUE;
            }
        };
        Tx* t = new Tx;
        t->svc = _svc;
        return t;
    }

private:
    RedisService* _svc;
};

}  // namespace

TEST(Redis, reply_parsing) {
    Buf b;
    b.append("+OK\r\n-ERR bad\r\n:42\r\n$5\r\nhel");
    RedisResponse res;
    EXPECT_EQ(res.ConsumePartial(&b, 4), 0);  // bulk string incomplete
    b.append("lo\r\n*3\r\n$1\r\na\r\n$-1\r\n:7\r\n");
    EXPECT_EQ(res.ConsumePartial(&b, 5), 1);
    ASSERT_EQ(res.reply_size(), 5);
    EXPECT_EQ(res.reply(0).data(), "OK");
    EXPECT_TRUE(res.reply(1).is_error());
    EXPECT_EQ(res.reply(2).integer(), 42);
    EXPECT_EQ(res.reply(3).data(), "hello");
    ASSERT_TRUE(res.reply(4).is_array());
    EXPECT_TRUE(res.reply(4)[1].is_nil());
    EXPECT_EQ(res.reply(4)[2].integer(), 7);
    EXPECT_TRUE(b.empty());
}

TEST(Redis, client_server_pipeline_multi) {
    KV kv;
    RedisService svc;
    SetHandler set(&kv);
    GetHandler get(&kv);
    IncrHandler incr(&kv);
    MultiHandler multi(&svc);
    svc.AddCommandHandler("set", &set);
    svc.AddCommandHandler("get", &get);
    svc.AddCommandHandler("incr", &incr);
    svc.AddCommandHandler("multi", &multi);
    Server server;
    ServerOptions so;
    so.redis_service = &svc;
    so.has_builtin_services = false;
    ASSERT_EQ(server.Start("127.0.0.1:0", &so), 0);
    Channel ch;
    ChannelOptions co;
    co.protocol = "redis";
    co.timeout_ms = 3000;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &co), 0);
    for (int round = 0; round < 20; ++round) {
        RedisRequest req;
        RedisResponse res;
        Controller cntl;
        ASSERT_TRUE(req.AddCommand("SET k%d %s", round, "hello world"));
        ASSERT_TRUE(req.AddCommand("GET k%d", round));
        ASSERT_TRUE(req.AddCommand("INCR counter"));
        ASSERT_TRUE(req.AddCommand("GET missing"));
        ASSERT_TRUE(req.AddCommand("NOSUCH x"));
        ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        ASSERT_EQ(res.reply_size(), 5);
        EXPECT_EQ(res.reply(0).data(), "OK");
        EXPECT_EQ(res.reply(1).data(), "hello world");
        EXPECT_EQ(res.reply(2).integer(), round + 1);
        EXPECT_TRUE(res.reply(3).is_nil());
        EXPECT_TRUE(res.reply(4).is_error());
    }
    RedisRequest req;
    RedisResponse res;
    Controller cntl;
    req.AddCommand("MULTI");
    req.AddCommand("INCR tx");
    req.AddCommand("INCR tx");
    req.AddCommand("EXEC");
    ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
    ASSERT_FALSE(cntl.Failed());
    ASSERT_EQ(res.reply_size(), 4);
    EXPECT_EQ(res.reply(1).data(), "QUEUED");
    ASSERT_TRUE(res.reply(3).is_array());
    EXPECT_EQ(res.reply(3)[1].integer(), 2);
}

TEST(Redis, command_formatting) {
    RedisRequest req;
    const char bin[] = {'a', '\0', '\r', '\n', 'b'};
    ASSERT_TRUE(req.AddCommand("SET key%d %b", 7, bin, sizeof(bin)));
    ASSERT_TRUE(req.AddCommand("INCRBY %s %lld", "cnt", -5000000000LL));
    ASSERT_TRUE(req.AddCommandByComponents({"MSET", "k 1", "v"}));
    ASSERT_TRUE(req.AddCommand("ECHO 100%%"));
    EXPECT_EQ(req.command_size(), 4);
    Buf out;
    ASSERT_TRUE(req.SerializeTo(&out));
    const std::string want = std::string("*3\r\n$3\r\nSET\r\n$4\r\nkey7\r\n$5\r\n") + std::string(bin, sizeof(bin)) +
                             "\r\n*3\r\n$6\r\nINCRBY\r\n$3\r\ncnt\r\n$11\r\n-5000000000\r\n"
                             "*3\r\n$4\r\nMSET\r\n$3\r\nk 1\r\n$1\r\nv\r\n"
                             "*2\r\n$4\r\nECHO\r\n$4\r\n100%\r\n";
    EXPECT_EQ(out.to_string(), want);
    RedisRequest bad;
    EXPECT_FALSE(bad.AddCommand("GET %q", 1));
    EXPECT_TRUE(bad.has_error());
    Buf b2;
    EXPECT_FALSE(bad.SerializeTo(&b2));
    EXPECT_FALSE(bad.AddCommandByComponents({}));
}

TEST(Redis, reply_serialize_roundtrip_bytewise) {
    RedisReply r;
    r.SetArray(4);
    r[0].SetStatus("OK");
    r[1].SetInteger(-12);
    r[2].SetArray(2);
    r[2][0].SetString(std::string("bin\0\r\nary", 9));
    r[2][1].SetNil();
    r[3].SetError("ERR nested");
    Buf wire;
    r.SerializeTo(&wire);
    const std::string bytes = wire.to_string();
    // feed one byte at a time: incomplete prefixes return 0 and consume nothing
    Buf in;
    RedisReply back;
    int rc = 0;
    for (size_t i = 0; i < bytes.size(); ++i) {
        in.append(bytes.data() + i, 1);
        rc = back.ConsumePartial(&in);
        if (i + 1 < bytes.size()) {
            ASSERT_EQ(rc, 0);
            ASSERT_EQ(in.size(), i + 1);
        }
    }
    ASSERT_EQ(rc, 1);
    EXPECT_TRUE(in.empty());
    ASSERT_TRUE(back.is_array());
    EXPECT_EQ(back[0].data(), "OK");
    EXPECT_EQ(back[1].integer(), -12);
    EXPECT_EQ(back[2][0].data(), std::string("bin\0\r\nary", 9));
    EXPECT_TRUE(back[2][1].is_nil());
    EXPECT_TRUE(back[3].is_error());
    EXPECT_EQ(back.ToString(), r.ToString());
}

TEST(Redis, malformed_replies_rejected) {
    for (const char* bad : {"?oops\r\n", "*99999999\r\n", "$-7\r\n", "$4x\r\nabcd\r\n", ":12a\r\n", "*\r\n"}) {
        Buf b;
        b.append(bad);
        RedisReply r;
        const int rc = r.ConsumePartial(&b);
        EXPECT_LT(rc, 0);
    }
    Buf nil;
    nil.append("$-1\r\n*-1\r\n");
    RedisResponse res;
    ASSERT_EQ(res.ConsumePartial(&nil, 2), 1);
    EXPECT_TRUE(res.reply(0).is_nil());
    EXPECT_TRUE(res.reply(1).is_nil());
}

TEST(Redis, concurrent_clients_and_large_values) {
    KV kv;
    RedisService svc;
    SetHandler set(&kv);
    GetHandler get(&kv);
    IncrHandler incr(&kv);
    svc.AddCommandHandler("set", &set);
    svc.AddCommandHandler("get", &get);
    svc.AddCommandHandler("incr", &incr);
    Server server;
    ServerOptions so;
    so.redis_service = &svc;
    so.has_builtin_services = false;
    ASSERT_EQ(server.Start("127.0.0.1:0", &so), 0);
    const std::string addr = "127.0.0.1:" + std::to_string(server.listen_port());
    // 8 pooled-connection callers x 200 INCRs of one key: replies are
    // matched to their requests, and no increment is lost
    Channel ch;
    ChannelOptions co;
    co.protocol = "redis";
    co.connection_type = "pooled";
    co.timeout_ms = 5000;
    ASSERT_EQ(ch.Init(addr.c_str(), &co), 0);
    std::atomic<int> errors{0};
    std::vector<std::thread> ts;
    for (int t = 0; t < 8; ++t) {
        ts.emplace_back([&] {
            for (int i = 0; i < 200; ++i) {
                RedisRequest req;
                RedisResponse res;
                Controller cntl;
                req.AddCommand("INCR shared");
                ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
                if (cntl.Failed() || res.reply_size() != 1 || !res.reply(0).is_integer()) errors.fetch_add(1);
            }
        });
    }
    const int64_t t0 = monotonic_us();
    for (auto& t : ts) t.join();
    EXPECT_LT(monotonic_us() - t0, 5000000);
    EXPECT_EQ(errors.load(), 0);
    {
        RedisRequest req;
        RedisResponse res;
        Controller cntl;
        req.AddCommand("GET shared");
        ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        EXPECT_EQ(res.reply(0).data(), "1600");
    }
    // values spanning many socket reads: the server keeps its parse state
    // across reads (reference: redis_protocol.cpp:167-194)
    for (size_t size : {size_t(48) << 10, size_t(1) << 20, size_t(4) << 20}) {
        std::string big(size, 'v');
        for (size_t i = 0; i < big.size(); i += 4093) big[i] = (char)('a' + (i / 4093) % 26);
        RedisRequest req;
        RedisResponse res;
        Controller cntl;
        req.AddCommandByComponents({"SET", "big", big});
        req.AddCommandByComponents({"GET", "big"});
        const int64_t t1 = monotonic_us();
        ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        ASSERT_EQ(res.reply_size(), 2);
        EXPECT_EQ(res.reply(0).data(), "OK");
        EXPECT_TRUE(res.reply(1).data() == big);
        EXPECT_LT(monotonic_us() - t1, 3000000);
    }
}

namespace {
// AUTH/SELECT handlers that record the order commands reach the server
struct AuthLog {
    std::mutex mu;
    std::vector<std::string> seen;
    void add(const std::string& s) {
        std::lock_guard<std::mutex> g(mu);
        seen.push_back(s);
    }
};
class AuthHandler : public RedisCommandHandler {
public:
    explicit AuthHandler(AuthLog* log) : _log(log) {}
    Result Run(const std::vector<std::string>& args, RedisReply* out, bool) override {
        _log->add(args[0] + " " + (args.size() > 1 ? args[1] : ""));
        if (args.size() == 2 && args[1] == "s3cret") out->SetStatus("OK");
        else out->SetError("ERR invalid password");
        return OK;
    }
    AuthLog* _log;
};
class SelectHandler : public RedisCommandHandler {
public:
    explicit SelectHandler(AuthLog* log) : _log(log) {}
    Result Run(const std::vector<std::string>& args, RedisReply* out, bool) override {
        _log->add(args[0] + " " + (args.size() > 1 ? args[1] : ""));
        out->SetStatus("OK");
        return OK;
    }
    AuthLog* _log;
};
class LoggedGet : public RedisCommandHandler {
public:
    explicit LoggedGet(AuthLog* log) : _log(log) {}
    Result Run(const std::vector<std::string>& args, RedisReply* out, bool) override {
        _log->add(args[0]);
        out->SetString("value");
        return OK;
    }
    AuthLog* _log;
};
}  // namespace

TEST(Redis, auth_and_select_once_per_connection) {
    AuthLog log;
    RedisService svc;
    AuthHandler auth(&log);
    SelectHandler sel(&log);
    LoggedGet get(&log);
    svc.AddCommandHandler("auth", &auth);
    svc.AddCommandHandler("select", &sel);
    svc.AddCommandHandler("get", &get);
    Server server;
    ServerOptions so;
    so.redis_service = &svc;
    so.has_builtin_services = false;
    ASSERT_EQ(server.Start("127.0.0.1:0", &so), 0);
    const std::string addr = "127.0.0.1:" + std::to_string(server.listen_port());
    policy::RedisAuthenticator good("s3cret", 3);
    Channel ch;
    ChannelOptions co;
    co.protocol = "redis";
    co.auth = &good;
    ASSERT_EQ(ch.Init(addr.c_str(), &co), 0);
    // concurrent first calls: exactly one of them carries AUTH + SELECT,
    // and both go out before any command of the connection
    std::vector<std::thread> ts;
    std::atomic<int> errors{0};
    for (int t = 0; t < 8; ++t) {
        ts.emplace_back([&] {
            for (int i = 0; i < 20; ++i) {
                RedisRequest req;
                RedisResponse res;
                Controller cntl;
                req.AddCommand("GET k");
                ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
                if (cntl.Failed() || res.reply_size() != 1 || res.reply(0).data() != "value") errors.fetch_add(1);
            }
        });
    }
    for (auto& t : ts) t.join();
    EXPECT_EQ(errors.load(), 0);
    ASSERT_EQ(log.seen.size(), 162u);
    EXPECT_EQ(log.seen[0], "auth s3cret");
    EXPECT_EQ(log.seen[1], "select 3");
    for (size_t i = 2; i < log.seen.size(); ++i) EXPECT_EQ(log.seen[i], "get");
    // a wrong password fails the calls instead of running them unauthenticated
    policy::RedisAuthenticator bad("nope");
    Channel ch2;
    co.auth = &bad;
    co.timeout_ms = 2000;
    co.max_retry = 0;
    ASSERT_EQ(ch2.Init(addr.c_str(), &co), 0);
    RedisRequest req;
    RedisResponse res;
    Controller cntl;
    req.AddCommand("GET k");
    ch2.CallMethod(nullptr, &cntl, &req, &res, nullptr);
    EXPECT_TRUE(cntl.Failed());
    // credentials themselves
    std::string cred;
    good.GenerateCredential(&cred);
    EXPECT_EQ(cred, "*2\r\n$4\r\nAUTH\r\n$6\r\ns3cret\r\n*2\r\n$6\r\nSELECT\r\n$1\r\n3\r\n");
    EXPECT_EQ(good.auth_replies(), 2);
}

namespace {
int raw_connect(int port) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)port);
    sa.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (connect(fd, (sockaddr*)&sa, sizeof(sa)) != 0) {
        close(fd);
        return -1;
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    return fd;
}
bool send_all(int fd, const std::string& s) {
    size_t off = 0;
    while (off < s.size()) {
        const ssize_t n = ::send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
        if (n <= 0) return false;
        off += (size_t)n;
    }
    return true;
}
// read until `want` bytes arrived (or 3 s passed)
std::string recv_n(int fd, size_t want) {
    std::string out;
    const int64_t end = monotonic_us() + 3000000;
    char buf[4096];
    while (out.size() < want && monotonic_us() < end) {
        pollfd p{fd, POLLIN, 0};
        if (poll(&p, 1, 100) <= 0) continue;
        const ssize_t n = ::recv(fd, buf, sizeof(buf), 0);
        if (n <= 0) break;
        out.append(buf, (size_t)n);
    }
    return out;
}
}  // namespace

// a SET whose value starts with another protocol's magic
// ("PRPC" is baidu_std's) arrives split across reads. Once the redis
// parser installed its context the connection is redis's: the value at the
// front of the buffer must not be offered to baidu_std.
TEST(Redis, split_value_with_foreign_magic_stays_redis) {
    KV kv;
    RedisService svc;
    SetHandler set(&kv);
    GetHandler get(&kv);
    svc.AddCommandHandler("set", &set);
    svc.AddCommandHandler("get", &get);
    Server server;
    ServerOptions so;
    so.redis_service = &svc;
    so.has_builtin_services = false;
    ASSERT_EQ(server.Start("127.0.0.1:0", &so), 0);
    const int fd = raw_connect(server.listen_port());
    ASSERT_GE(fd, 0);
    const std::string value = "PRPC\x00\x00\x00\x10\x00\x00\x00\x04" + std::string("abcd");
    const std::string v(value.data(), 16);
    // header and bulk length first, the value in a later read
    ASSERT_TRUE(send_all(fd, "*3\r\n$3\r\nSET\r\n$1\r\nk\r\n$16\r\n"));
    usleep(50000);
    ASSERT_TRUE(send_all(fd, v.substr(0, 6)));
    usleep(50000);
    ASSERT_TRUE(send_all(fd, v.substr(6) + "\r\n"));
    EXPECT_EQ(recv_n(fd, 5), "+OK\r\n");
    ASSERT_TRUE(send_all(fd, "*2\r\n$3\r\nGET\r\n$1\r\nk\r\n"));
    const std::string want = "$16\r\n" + v + "\r\n";
    EXPECT_EQ(recv_n(fd, want.size()), want);
    {
        std::lock_guard<std::mutex> g(kv.mu);
        EXPECT_EQ(kv.m["k"], v);
    }
    close(fd);
    server.Stop(0);
    server.Join();
}

namespace {

// A server with the test's handlers, and a redis channel to it.
struct RedisFixture {
    KV kv;
    RedisService svc;
    SetHandler set{&kv};
    GetHandler get{&kv};
    IncrHandler incr{&kv};
    MultiHandler multi{&svc};
    Server server;
    Channel ch;
    bool ok = false;
    RedisFixture() {
        svc.AddCommandHandler("set", &set);
        svc.AddCommandHandler("get", &get);
        svc.AddCommandHandler("incr", &incr);
        svc.AddCommandHandler("multi", &multi);
    }
    bool Start() {
        ServerOptions so;
        so.redis_service = &svc;
        so.has_builtin_services = false;
        if (server.Start("127.0.0.1:0", &so) != 0) return false;
        ChannelOptions co;
        co.protocol = "redis";
        co.timeout_ms = 3000;
        return ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &co) == 0;
    }
};

std::string wire(const RedisRequest& r) { return r.ToString(); }

// INCRBY/DECR/DECRBY over the shared KV (the reference runs them against a
// real redis-server; here the server side is ours)
class AddHandler : public RedisCommandHandler {
public:
    AddHandler(KV* kv, int sign, bool by) : _kv(kv), _sign(sign), _by(by) {}
    Result Run(const std::vector<std::string>& args, RedisReply* out, bool) override {
        if (args.size() != (_by ? 3u : 2u)) {
            out->SetError("ERR wrong number of arguments");
            return OK;
        }
        const int64_t d = _by ? atoll(args[2].c_str()) : 1;
        std::lock_guard<std::mutex> g(_kv->mu);
        const int64_t v = atoll(_kv->m[args[1]].c_str()) + _sign * d;
        _kv->m[args[1]] = std::to_string(v);
        out->SetInteger(v);
        return OK;
    }

private:
    KV* _kv;
    int _sign;
    bool _by;
};

}  // namespace

TEST(Redis, keys_with_spaces) {
    RedisFixture f;
    ASSERT_TRUE(f.Start());
    RedisRequest req;
    RedisResponse res;
    Controller cntl;
    ASSERT_TRUE(req.AddCommand("set %s 'he1 he1 da1'", "hello world"));
    ASSERT_TRUE(req.AddCommand("set 'hello2 world2' 'he2 he2 da2'"));
    ASSERT_TRUE(req.AddCommand("set \"hello3 world3\" \"he3 he3 da3\""));
    ASSERT_TRUE(req.AddCommand("get \"hello world\""));
    ASSERT_TRUE(req.AddCommand("get 'hello world'"));
    ASSERT_TRUE(req.AddCommand("get 'hello2 world2'"));
    ASSERT_TRUE(req.AddCommand("get 'hello3 world3'"));
    f.ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
    ASSERT_FALSE(cntl.Failed());
    ASSERT_EQ(res.reply_size(), 7);
    for (int i = 0; i < 3; ++i) EXPECT_EQ(res.reply(i).data(), "OK");
    EXPECT_EQ(res.reply(3).data(), "he1 he1 da1");
    EXPECT_EQ(res.reply(4).data(), "he1 he1 da1");
    EXPECT_EQ(res.reply(5).data(), "he2 he2 da2");
    EXPECT_EQ(res.reply(6).data(), "he3 he3 da3");
}

TEST(Redis, incr_and_decr) {
    RedisFixture f;
    AddHandler decr(&f.kv, -1, false), incrby(&f.kv, 1, true), decrby(&f.kv, -1, true);
    f.svc.AddCommandHandler("decr", &decr);
    f.svc.AddCommandHandler("incrby", &incrby);
    f.svc.AddCommandHandler("decrby", &decrby);
    ASSERT_TRUE(f.Start());
    RedisRequest req;
    RedisResponse res;
    Controller cntl;
    req.AddCommand("incr counter1");
    req.AddCommand("decr counter1");
    req.AddCommand("incrby counter1 %d", 10);
    req.AddCommand("decrby counter1 %d", 20);
    f.ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
    ASSERT_FALSE(cntl.Failed());
    ASSERT_EQ(res.reply_size(), 4);
    for (int i = 0; i < 4; ++i) EXPECT_EQ(res.reply(i).type(), REDIS_REPLY_INTEGER);
    EXPECT_EQ(res.reply(0).integer(), 1);
    EXPECT_EQ(res.reply(1).integer(), 0);
    EXPECT_EQ(res.reply(2).integer(), 10);
    EXPECT_EQ(res.reply(3).integer(), -10);
}

TEST(Redis, cmd_format_empty_and_adjacent_quotes) {
    struct Case {
        const char* fmt;
        const char* want;
    } cases[] = {
        {"set a ''", "*3\r\n$3\r\nset\r\n$1\r\na\r\n$0\r\n\r\n"},
        {"mset b '' c ''", "*5\r\n$4\r\nmset\r\n$1\r\nb\r\n$0\r\n\r\n$1\r\nc\r\n$0\r\n\r\n"},
        {"set a 123", "*3\r\n$3\r\nset\r\n$1\r\na\r\n$3\r\n123\r\n"},
        {"mset b '' c ccc", "*5\r\n$4\r\nmset\r\n$1\r\nb\r\n$0\r\n\r\n$1\r\nc\r\n$3\r\nccc\r\n"},
        {"get ''key value", "*4\r\n$3\r\nget\r\n$0\r\n\r\n$3\r\nkey\r\n$5\r\nvalue\r\n"},
        {"get key'' value", "*4\r\n$3\r\nget\r\n$3\r\nkey\r\n$0\r\n\r\n$5\r\nvalue\r\n"},
        {"get 'ext'key   value  ", "*4\r\n$3\r\nget\r\n$3\r\next\r\n$3\r\nkey\r\n$5\r\nvalue\r\n"},
        {"  get   key'ext'   value  ", "*4\r\n$3\r\nget\r\n$3\r\nkey\r\n$3\r\next\r\n$5\r\nvalue\r\n"},
    };
    for (const Case& c : cases) {
        RedisRequest req;
        ASSERT_TRUE(req.AddCommand(c.fmt));
        EXPECT_TRUE_M(wire(req) == c.want, std::string(c.fmt));
    }
    RedisRequest bad;
    EXPECT_FALSE(bad.AddCommand("set a 'unterminated"));
    EXPECT_TRUE(bad.has_error());
}

TEST(Redis, quote_and_escape) {
    struct Case {
        const char* fmt;
        const char* value;
    } cases[] = {
        {"set a 'foo bar'", "foo bar"},      {"set a 'foo \\'bar'", "foo 'bar"},
        {"set a 'foo \"bar'", "foo \"bar"},  {"set a 'foo \\\"bar'", "foo \\\"bar"},
        {"set a \"foo 'bar\"", "foo 'bar"},  {"set a \"foo \\'bar\"", "foo \\'bar"},
        {"set a \"foo \\\"bar\"", "foo \"bar"},
    };
    for (const Case& c : cases) {
        RedisRequest req;
        ASSERT_TRUE(req.AddCommand(c.fmt));
        const std::string v = c.value;
        const std::string want = "*3\r\n$3\r\nset\r\n$1\r\na\r\n$" + std::to_string(v.size()) + "\r\n" + v + "\r\n";
        EXPECT_TRUE_M(wire(req) == want, std::string(c.fmt));
    }
}

// The server's incremental command parser: a command delivered one byte
// at a time, then a command with a non-bulk argument (refused), and
// connections opening with a non-array (not redis).
TEST(Redis, command_parser_incremental_and_refusals) {
    RedisFixture f;
    ASSERT_TRUE(f.Start());
    {
        const int fd = raw_connect(f.server.listen_port());
        ASSERT_GE(fd, 0);
        const std::string cmd = "*3\r\n$3\r\nset\r\n$3\r\nabc\r\n$3\r\ndef\r\n";
        for (int round = 0; round < 20; ++round) {
            for (char c : cmd) ASSERT_TRUE(send_all(fd, std::string(1, c)));
            EXPECT_EQ(recv_n(fd, 5), "+OK\r\n");
        }
        ASSERT_TRUE(send_all(fd, "*2\r\n$3\r\nget\r\n$3\r\nabc\r\n"));
        EXPECT_EQ(recv_n(fd, 9), "$3\r\ndef\r\n");
        // an integer where a bulk argument must be: the connection is dropped
        ASSERT_TRUE(send_all(fd, "*3\r\n$3\r\nset\r\n:123\r\n$3\r\ndef\r\n"));
        EXPECT_EQ(recv_n(fd, 1), "");
        close(fd);
    }
    for (const char* first : {":123456\r\n", "+OK\r\n", "$5\r\nhello\r\n"}) {
        const int fd = raw_connect(f.server.listen_port());
        ASSERT_GE(fd, 0);
        ASSERT_TRUE(send_all(fd, first));
        EXPECT_EQ(recv_n(fd, 1), "");  // no protocol claims it: closed
        close(fd);
    }
}

TEST(Redis, server_command_continue) {
    RedisFixture f;
    ASSERT_TRUE(f.Start());
    {
        RedisRequest req;
        RedisResponse res;
        Controller cntl;
        ASSERT_TRUE(req.AddCommand("set hello world"));
        ASSERT_TRUE(req.AddCommand("get hello"));
        f.ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        ASSERT_EQ(res.reply_size(), 2);
        EXPECT_EQ(res.reply(1).data(), "world");
    }
    {
        RedisRequest req;
        RedisResponse res;
        Controller cntl;
        ASSERT_TRUE(req.AddCommand("multi"));
        ASSERT_TRUE(req.AddCommand("mUltI"));
        const int count = 10;
        for (int i = 0; i < count; ++i) ASSERT_TRUE(req.AddCommand("incr hello2"));
        ASSERT_TRUE(req.AddCommand("exec"));
        f.ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        ASSERT_EQ(res.reply_size(), count + 3);
        EXPECT_EQ(res.reply(0).data(), "OK");
        EXPECT_TRUE(res.reply(1).is_error());
        for (int i = 2; i < count + 2; ++i) EXPECT_EQ(res.reply(i).data(), "QUEUED");
        const RedisReply& m = res.reply(count + 2);
        ASSERT_TRUE(m.is_array());
        ASSERT_EQ((int)m.size(), count);
        for (int i = 0; i < count; ++i) EXPECT_EQ(m[i].integer(), i + 1);
    }
    {
        // after EXEC the connection is back to plain commands
        RedisRequest req;
        RedisResponse res;
        Controller cntl;
        ASSERT_TRUE(req.AddCommand("get hello"));
        ASSERT_TRUE(req.AddCommand("get nothere"));
        ASSERT_TRUE(req.AddCommand("set key1 value1"));
        ASSERT_TRUE(req.AddCommand("get key1"));
        f.ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        EXPECT_EQ(res.reply(0).data(), "world");
        EXPECT_TRUE(res.reply(1).is_nil());
        EXPECT_EQ(res.reply(2).data(), "OK");
        EXPECT_EQ(res.reply(3).data(), "value1");
    }
}

namespace {
// Batched handlers (reference: RedisServiceImpl::OnBatched): commands that
// arrive together are deferred (BATCHED) and settled by the last one of the
// read (flush_batched) with one reply per command, in one array.
struct BatchKV {
    KV kv;
    std::vector<std::vector<std::string>> pending;
    int batches = 0;
    void Do(const std::vector<std::string>& a, RedisReply* out) {
        std::lock_guard<std::mutex> g(kv.mu);
        if (a[0] == "set") {
            kv.m[a[1]] = a[2];
            out->SetStatus("OK");
        } else {
            auto it = kv.m.find(a[1]);
            if (it == kv.m.end()) out->SetNil();
            else out->SetString(it->second);
        }
    }
    RedisCommandHandler::Result OnBatched(const std::vector<std::string>& a, RedisReply* out, bool flush) {
        if (pending.empty() && flush) {
            Do(a, out);
            return RedisCommandHandler::OK;
        }
        pending.push_back(a);
        if (!flush) return RedisCommandHandler::BATCHED;
        out->SetArray(pending.size());
        for (size_t i = 0; i < pending.size(); ++i) Do(pending[i], &(*out)[i]);
        pending.clear();
        ++batches;
        return RedisCommandHandler::OK;
    }
};
class BatchedHandler : public RedisCommandHandler {
public:
    explicit BatchedHandler(BatchKV* b) : _b(b) {}
    Result Run(const std::vector<std::string>& args, RedisReply* out, bool flush) override {
        if (args.size() < 2) {
            out->SetError("ERR wrong number of arguments");
            return OK;
        }
        return _b->OnBatched(args, out, flush);
    }

private:
    BatchKV* _b;
};
}  // namespace

TEST(Redis, server_handle_pipeline_batched) {
    BatchKV b;
    BatchedHandler h(&b);
    RedisService svc;
    svc.AddCommandHandler("set", &h);
    svc.AddCommandHandler("get", &h);
    Server server;
    ServerOptions so;
    so.redis_service = &svc;
    so.has_builtin_services = false;
    ASSERT_EQ(server.Start("127.0.0.1:0", &so), 0);
    // one write, so all eight commands arrive in one read
    const int fd = raw_connect(server.listen_port());
    ASSERT_GE(fd, 0);
    RedisRequest req;
    for (const char* c : {"set key1 v1", "set key2 v2", "set key3 v3", "get hello", "get hello", "set key1 world",
                          "set key2 world", "get key2"})
        ASSERT_TRUE(req.AddCommand(c));
    ASSERT_TRUE(send_all(fd, wire(req)));
    const std::string want = "+OK\r\n+OK\r\n+OK\r\n$-1\r\n$-1\r\n+OK\r\n+OK\r\n$5\r\nworld\r\n";
    EXPECT_EQ(recv_n(fd, want.size()), want);
    EXPECT_EQ(b.batches, 1);
    close(fd);
    // through a channel, too
    Channel ch;
    ChannelOptions co;
    co.protocol = "redis";
    co.timeout_ms = 3000;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &co), 0);
    RedisResponse res;
    Controller cntl;
    ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
    ASSERT_FALSE(cntl.Failed());
    ASSERT_EQ(res.reply_size(), 8);
    EXPECT_EQ(res.reply(7).data(), "world");
}
