// Redis server + client (reference example/redis_c++): a RedisService with
// SET/GET/INCR handlers over an in-memory map, driven by the redis protocol
// client with several commands pipelined in one request.
#include <map>
#include <mutex>

#include "examples/common.h"
#include "redis/redis.h"

namespace {
std::mutex g_mu;
std::map<std::string, std::string> g_kv;

class SetHandler : public mrpc::RedisCommandHandler {
public:
    Result Run(const std::vector<std::string>& a, mrpc::RedisReply* out, bool) override {
        if (a.size() != 3) {
            out->SetError("ERR wrong number of arguments for 'set'");
            return OK;
        }
        std::lock_guard<std::mutex> g(g_mu);
        g_kv[a[1]] = a[2];
        out->SetStatus("OK");
        return OK;
    }
};
class GetHandler : public mrpc::RedisCommandHandler {
public:
    Result Run(const std::vector<std::string>& a, mrpc::RedisReply* out, bool) override {
        std::lock_guard<std::mutex> g(g_mu);
        auto it = a.size() == 2 ? g_kv.find(a[1]) : g_kv.end();
        if (it == g_kv.end()) out->SetNil();
        else out->SetString(it->second);
        return OK;
    }
};
class IncrHandler : public mrpc::RedisCommandHandler {
public:
    Result Run(const std::vector<std::string>& a, mrpc::RedisReply* out, bool) override {
        std::lock_guard<std::mutex> g(g_mu);
        const long long v = atoll(g_kv[a[1]].c_str()) + 1;
        g_kv[a[1]] = std::to_string(v);
        out->SetInteger(v);
        return OK;
    }
};
}  // namespace

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    mrpc::RedisService svc;
    SetHandler set;
    GetHandler get;
    IncrHandler incr;
    svc.AddCommandHandler("set", &set);
    svc.AddCommandHandler("get", &get);
    svc.AddCommandHandler("incr", &incr);
    mrpc::Server server;
    mrpc::ServerOptions so;
    so.redis_service = &svc;
    if (server.Start("127.0.0.1:0", &so) != 0) return 1;
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.protocol = "redis";
    opt.timeout_ms = 2000;
    if (ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &opt) != 0) return 1;
    mrpc::RedisRequest req;
    mrpc::RedisResponse res;
    req.AddCommand("SET greeting %s", "hello-mi355x");
    req.AddCommand("GET greeting");
    req.AddCommand("INCR visits");
    req.AddCommand("INCR visits");
    req.AddCommand("GET nothing");
    mrpc::Controller cntl;
    ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
    if (cntl.Failed()) return demo::Check(false, cntl.ErrorText().c_str());
    printf("SET -> %s, GET -> %s, INCR -> %lld, INCR -> %lld, GET nothing -> %s\n", res.reply(0).data().c_str(),
           res.reply(1).data().c_str(), (long long)res.reply(2).integer(), (long long)res.reply(3).integer(),
           res.reply(4).is_nil() ? "(nil)" : "?");
    return demo::Check(res.reply(1).data() == "hello-mi355x" && res.reply(3).integer() == 2 && res.reply(4).is_nil(),
                       "pipelined redis commands");
}
