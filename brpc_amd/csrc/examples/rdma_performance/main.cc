// RDMA performance (reference example/rdma_performance): closed-loop echo
// over the RDMA data plane with -queue_depth outstanding async calls per
// sender, sweeping attachment size and sender count, printing avg / p99
// latency, MB/s and kQPS per point. Without an HCA the in-process soft verbs
// provider is used (numbers then measure the endpoint + runtime, not a NIC).
#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

#include "base/time.h"
#include "examples/common.h"
#include "fiber/sync.h"
#include "rdma/rdma.h"

DEFINE_int32(queue_depth, 4, "outstanding async calls per sender");
DEFINE_double(seconds_per_point, 0.3, "measurement time per sweep point");
DEFINE_string(sizes, "1,1024,65536,1048576", "attachment sizes");
DEFINE_string(senders, "1,4", "sender counts");
DEFINE_bool(use_rdma, true, "RDMA data plane (false: plain TCP for comparison)");

namespace {
std::vector<int> parse(const std::string& s) {
    std::vector<int> v;
    size_t b = 0;
    while (b < s.size()) {
        size_t e = s.find(',', b);
        v.push_back(atoi(s.substr(b, e == std::string::npos ? std::string::npos : e - b).c_str()));
        if (e == std::string::npos) break;
        b = e + 1;
    }
    return v;
}
}  // namespace

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    mrpc::ServerOptions so;
    so.use_rdma = FLAGS_use_rdma;
    demo::LocalServer s("rdma", 0, so);
    printf("%s", mrpc::rdma::DescribeRdma().c_str());
    printf("%10s %7s %9s %9s %10s %9s\n", "size", "senders", "avg_us", "p99_us", "MB/s", "kQPS");
    int failures = 0;
    for (int senders : parse(FLAGS_senders)) {
        for (int size : parse(FLAGS_sizes)) {
            mrpc::Channel ch;
            mrpc::ChannelOptions opt;
            opt.use_rdma = FLAGS_use_rdma;
            opt.timeout_ms = 5000;
            opt.connection_group = "s" + std::to_string(size) + "x" + std::to_string(senders);
            if (ch.Init(s.addr().c_str(), &opt) != 0) return 1;
            const std::string att(size, 'r');
            std::atomic<bool> stop{false};
            std::atomic<int64_t> done{0}, errs{0};
            std::mutex mu;
            std::vector<int64_t> lats;
            std::vector<std::thread> th;
            const int64_t t0 = mrpc::monotonic_us();
            for (int t = 0; t < senders; ++t) {
                th.emplace_back([&] {
                    example::EchoService_Stub stub(&ch);
                    std::vector<int64_t> mine;
                    while (!stop.load()) {
                        mrpc::fiber::CountdownEvent batch(FLAGS_queue_depth);
                        std::vector<std::unique_ptr<mrpc::Controller>> cs(FLAGS_queue_depth);
                        std::vector<example::EchoRequest> rq(FLAGS_queue_depth);
                        std::vector<example::EchoResponse> rs(FLAGS_queue_depth);
                        for (int q = 0; q < FLAGS_queue_depth; ++q) {
                            cs[q].reset(new mrpc::Controller);
                            rq[q].set_message("p");
                            cs[q]->request_attachment().append(att);
                            stub.Echo(cs[q].get(), &rq[q], &rs[q], mrpc::NewCallback([&batch] { batch.signal(); }));
                        }
                        batch.wait();
                        for (auto& c : cs) {
                            if (c->Failed()) errs.fetch_add(1);
                            else mine.push_back(c->latency_us());
                        }
                        done.fetch_add(FLAGS_queue_depth);
                    }
                    std::lock_guard<std::mutex> g(mu);
                    lats.insert(lats.end(), mine.begin(), mine.end());
                });
            }
            usleep((useconds_t)(FLAGS_seconds_per_point * 1e6));
            stop = true;
            for (auto& t : th) t.join();
            const double sec = (mrpc::monotonic_us() - t0) / 1e6;
            std::sort(lats.begin(), lats.end());
            long long sum = 0;
            for (int64_t v : lats) sum += v;
            const double avg = lats.empty() ? 0 : (double)sum / lats.size();
            const long long p99 = lats.empty() ? 0 : lats[std::min(lats.size() - 1, lats.size() * 99 / 100)];
            printf("%10d %7d %9.1f %9lld %10.1f %9.1f\n", size, senders, avg, p99,
                   2.0 * size * lats.size() / sec / 1e6, lats.size() / sec / 1e3);
            failures += errs.load() > 0 || lats.empty();
        }
    }
    return demo::Check(failures == 0, FLAGS_use_rdma ? "rdma sweep" : "tcp sweep");
}
