// Multi-threaded sync echo (reference example/multi_threaded_echo_c++):
// -thread_num pthreads (or fibers with -use_fiber) send synchronous calls of
// -request_size bytes + -attachment_size bytes for -duration_s seconds and
// the QPS / latency percentiles are printed.
#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

#include "base/time.h"
#include "builtin/cpu_profiler.h"
#include "examples/common.h"

DEFINE_int32(thread_num, 8, "concurrent senders");
DEFINE_bool(use_fiber, false, "senders are fibers instead of pthreads");
DEFINE_int32(request_size, 16, "bytes of the echoed message");
DEFINE_int32(attachment_size, 0, "bytes of attachment");
DEFINE_double(duration_s, 1.0, "seconds to run");
DEFINE_string(server, "", "ip:port of an external server (empty: start one in-process)");
DEFINE_string(protocol, "baidu_std", "protocol");
DEFINE_string(connection_type, "", "single / pooled / short");
DEFINE_string(profile_folded, "", "write a CPU profile of the run (folded stacks) to this file");

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    std::unique_ptr<demo::LocalServer> local;
    std::string addr = FLAGS_server;
    if (addr.empty()) {
        local.reset(new demo::LocalServer("mt"));
        addr = local->addr();
    }
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.protocol = FLAGS_protocol;
    opt.connection_type = FLAGS_connection_type;
    opt.timeout_ms = 1000;
    if (ch.Init(addr.c_str(), &opt) != 0) return 1;
    std::mutex lat_mu;
    std::vector<int64_t> lat;
    std::atomic<int64_t> errors{0};
    std::atomic<bool> stop{false};
    const std::string msg(FLAGS_request_size, 'x');
    const std::string att(FLAGS_attachment_size, 'a');
    auto sender = [&] {
        example::EchoService_Stub stub(&ch);
        std::vector<int64_t> mine;
        while (!stop.load(std::memory_order_relaxed)) {
            mrpc::Controller cntl;
            example::EchoRequest req;
            example::EchoResponse res;
            req.set_message(msg);
            cntl.request_attachment().append(att);
            stub.Echo(&cntl, &req, &res, nullptr);
            if (cntl.Failed()) {
                errors.fetch_add(1);
            } else {
                mine.push_back(cntl.latency_us());
            }
        }
        std::lock_guard<std::mutex> g(lat_mu);
        lat.insert(lat.end(), mine.begin(), mine.end());
    };
    std::vector<std::thread> threads;
    std::vector<mrpc::fiber::fiber_t> fibers;
    for (int i = 0; i < FLAGS_thread_num; ++i) {
        if (FLAGS_use_fiber) {
            mrpc::fiber::fiber_t t;
            mrpc::fiber::start(sender, false, nullptr, &t);
            fibers.push_back(t);
        } else {
            threads.emplace_back(sender);
        }
    }
    const int64_t t0 = mrpc::monotonic_us();
    if (!FLAGS_profile_folded.empty()) {
        std::string folded;
        int64_t nsamples = 0;
        mrpc::profiler::ProfileCpu(FLAGS_duration_s, 997, &folded, nullptr, &nsamples);
        FILE* f = fopen(FLAGS_profile_folded.c_str(), "w");
        if (f) {
            fwrite(folded.data(), 1, folded.size(), f);
            fclose(f);
        }
    } else {
        usleep((useconds_t)(FLAGS_duration_s * 1e6));
    }
    stop = true;
    for (auto& t : threads) t.join();
    for (auto t : fibers) mrpc::fiber::join(t);
    const double sec = (mrpc::monotonic_us() - t0) / 1e6;
    std::sort(lat.begin(), lat.end());
    auto pct = [&](double r) { return lat.empty() ? 0ll : (long long)lat[std::min(lat.size() - 1, (size_t)(r * lat.size()))]; };
    long long sum = 0;
    for (int64_t v : lat) sum += v;
    printf("qps=%.0f count=%zu errors=%lld avg=%lldus p50=%lldus p99=%lldus p999=%lldus max=%lldus\n",
           lat.size() / sec, lat.size(), (long long)errors.load(), lat.empty() ? 0ll : sum / (long long)lat.size(),
           pct(0.5), pct(0.99), pct(0.999), lat.empty() ? 0ll : (long long)lat.back());
    return demo::Check(!lat.empty() && errors.load() == 0, "multi-threaded echo");
}
