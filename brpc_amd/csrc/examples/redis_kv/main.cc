// Redis server + client (reference example/redis_c++): a RedisService with
// SET/GET/INCR handlers over an in-memory map, driven by the redis protocol
// client with several commands pipelined in one request. A load phase then
// runs -thread_num fibers each sending GET batches of -batch commands (the
// shape of the reference's docs/cn/redis_client.md figures: batches of 10
// from 1 / 50 / 200 bthreads, single or pooled connection).
#include <atomic>
#include <map>
#include <mutex>
#include <vector>

#include "base/time.h"
#include "fiber/fiber.h"

#include "examples/common.h"
#include "redis/redis.h"

DEFINE_int32(thread_num, 0, "load phase: fibers sending GET batches (0: no load phase)");
DEFINE_int32(batch, 10, "load phase: commands per pipelined request");
DEFINE_double(duration_s, 1.0, "load phase: seconds");
DEFINE_string(connection_type, "", "load phase: single / pooled");

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
    bool ok = res.reply(1).data() == "hello-mi355x" && res.reply(3).integer() == 2 && res.reply(4).is_nil();
    if (ok && FLAGS_thread_num > 0) {
        mrpc::Channel lch;
        mrpc::ChannelOptions lo = opt;
        lo.connection_type = FLAGS_connection_type;
        if (lch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &lo) != 0) return 1;
        std::atomic<bool> stop{false};
        std::atomic<int64_t> cmds{0}, errors{0}, lat_sum{0}, calls{0};
        std::vector<mrpc::fiber::fiber_t> fs(FLAGS_thread_num);
        for (auto& f : fs) {
            mrpc::fiber::start(
                [&] {
                    while (!stop.load(std::memory_order_relaxed)) {
                        mrpc::RedisRequest r;
                        mrpc::RedisResponse rs;
                        mrpc::Controller c;
                        for (int k = 0; k < FLAGS_batch; ++k) r.AddCommand("GET greeting");
                        lch.CallMethod(nullptr, &c, &r, &rs, nullptr);
                        if (c.Failed() || rs.reply_size() != FLAGS_batch) {
                            errors.fetch_add(1);
                        } else {
                            cmds.fetch_add(FLAGS_batch);
                            lat_sum.fetch_add(c.latency_us());
                            calls.fetch_add(1);
                        }
                    }
                },
                false, nullptr, &f);
        }
        mrpc::fiber::usleep((uint64_t)(FLAGS_duration_s * 1e6));
        stop = true;
        for (auto f : fs) mrpc::fiber::join(f);
        printf("load: %lld commands/s (%lld batches/s, avg %lld us) over %d fibers, %s connection, %lld failed calls\n",
               (long long)(cmds.load() / FLAGS_duration_s), (long long)(calls.load() / FLAGS_duration_s),
               calls.load() ? (long long)(lat_sum.load() / calls.load()) : 0ll, FLAGS_thread_num,
               FLAGS_connection_type.empty() ? "single" : FLAGS_connection_type.c_str(), (long long)errors.load());
        ok = errors.load() == 0 && cmds.load() > 0;
    }
    return demo::Check(ok, "pipelined redis commands");
}
