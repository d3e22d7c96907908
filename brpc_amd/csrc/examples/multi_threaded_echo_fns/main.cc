// Multi-threaded echo against a cluster from a naming service (reference
// example/multi_threaded_echo_fns_c++ with its random_kill.sh): -thread_num
// threads call through ONE channel whose servers come from a file naming
// service and are balanced by -load_balancer. While they run, a server is
// killed (calls to it fail over to the others through retries) and later
// restarted on the same port (the health checker revives the connection and
// traffic returns to it). Prints per-phase QPS and each server's share.
#include <atomic>
#include <fstream>
#include <memory>
#include <thread>
#include <vector>

#include "base/time.h"
#include "examples/common.h"
#include "services/echo_service.h"

DECLARE_int32(health_check_interval);
DEFINE_int32(thread_num, 8, "caller threads");
DEFINE_int32(server_num, 4, "servers in the naming service file");
DEFINE_string(load_balancer, "rr", "rr / random / la / c_murmurhash ...");
DEFINE_double(phase_s, 0.4, "seconds per phase (all up / one killed / restarted)");

namespace {
struct Node {
    int port = 0;
    std::unique_ptr<mrpc::EchoServiceImpl> echo;
    std::unique_ptr<mrpc::Server> server;
    bool Start(int want_port) {
        echo.reset(new mrpc::EchoServiceImpl);
        server.reset(new mrpc::Server);
        server->AddService(echo.get(), mrpc::SERVER_DOESNT_OWN_SERVICE);
        if (server->Start(("127.0.0.1:" + std::to_string(want_port)).c_str(), nullptr) != 0) return false;
        port = server->listen_port();
        return true;
    }
    void Kill() {
        server->Stop(0);
        server->Join();
        server.reset();
    }
    int64_t calls() const { return echo ? echo->ncalls() : 0; }
};
}  // namespace

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    FLAGS_health_check_interval = 1;
    std::vector<Node> nodes(FLAGS_server_num);
    for (auto& n : nodes) {
        if (!n.Start(0)) return 1;
    }
    char path[] = "/tmp/mrpc_fns_XXXXXX";
    const int fd = mkstemp(path);
    if (fd < 0) return 1;
    close(fd);
    {
        std::ofstream f(path);
        for (auto& n : nodes) f << "127.0.0.1:" << n.port << "\n";
    }
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.timeout_ms = 1000;
    opt.max_retry = 3;
    if (ch.Init((std::string("file://") + path).c_str(), FLAGS_load_balancer.c_str(), &opt) != 0) return 1;

    std::atomic<bool> stop{false};
    std::atomic<int64_t> ok_calls{0}, failed{0};
    std::vector<std::thread> th;
    for (int t = 0; t < FLAGS_thread_num; ++t) {
        th.emplace_back([&, t] {
            example::EchoService_Stub stub(&ch);
            for (uint64_t i = 0; !stop.load(std::memory_order_relaxed); ++i) {
                mrpc::Controller cntl;
                example::EchoRequest req;
                example::EchoResponse res;
                req.set_message("fns");
                cntl.set_request_code(i * 131 + t);  // used by the hashing balancers
                stub.Echo(&cntl, &req, &res, nullptr);
                (cntl.Failed() ? failed : ok_calls).fetch_add(1);
            }
        });
    }
    auto phase = [&](const char* name) {
        std::vector<int64_t> before;
        for (auto& n : nodes) before.push_back(n.calls());
        const int64_t ok0 = ok_calls.load(), f0 = failed.load();
        mrpc::fiber::usleep((uint64_t)(FLAGS_phase_s * 1e6));
        printf("%-22s %8.0f calls/s, %lld failed; per server:", name, (ok_calls.load() - ok0) / FLAGS_phase_s,
               (long long)(failed.load() - f0));
        std::vector<int64_t> got;
        for (size_t i = 0; i < nodes.size(); ++i) {
            got.push_back(nodes[i].calls() - before[i]);
            printf(" %lld", (long long)got.back());
        }
        printf("\n");
        return got;
    };
    std::vector<int64_t> all_up = phase("all servers up");
    const int victim = FLAGS_server_num / 2;
    const int victim_port = nodes[victim].port;
    nodes[victim].Kill();
    std::vector<int64_t> killed = phase("one server killed");
    const int64_t failed_after_kill = failed.load();
    bool restarted = nodes[victim].Start(victim_port);
    // wait for the health checker to revive the connection
    for (int i = 0; i < 40 && restarted && nodes[victim].calls() == 0; ++i) mrpc::fiber::usleep(100000);
    std::vector<int64_t> back = phase("server restarted");
    stop = true;
    for (auto& t : th) t.join();
    unlink(path);
    bool ok = restarted && failed_after_kill == 0;
    for (size_t i = 0; i < nodes.size(); ++i) {
        ok = ok && all_up[i] > 0 && back[i] > 0;
        if ((int)i != victim) ok = ok && killed[i] > 0;
    }
    ok = ok && killed[victim] == 0 && ok_calls.load() > 0;
    return demo::Check(ok, "failover and revival behind a naming service");
}
