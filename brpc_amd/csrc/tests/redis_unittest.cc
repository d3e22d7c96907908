// Redis client/server over RESP (spirit of the reference's
// test/brpc_redis_unittest.cpp): pipelined commands, reply types, server
// command handlers and MULTI/EXEC.
#include <map>
#include <mutex>

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

class MultiHandler : public RedisCommandHandler {
public:
    explicit MultiHandler(RedisService* svc) : _svc(svc) {}
    Result Run(const std::vector<std::string>&, RedisReply* out, bool) override {
        out->SetStatus("OK");
        return OK;
    }
    RedisCommandHandler* NewTransactionHandler() override {
        struct Tx : public RedisCommandHandler {
            RedisService* svc;
            Result Run(const std::vector<std::string>& args, RedisReply* out, bool b) override {
                RedisCommandHandler* h = svc->FindCommandHandler(args[0]);
                if (!h) {
                    out->SetError("ERR unknown command");
                    return OK;
                }
                return h->Run(args, out, b);
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
