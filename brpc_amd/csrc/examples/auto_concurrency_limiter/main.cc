// Auto concurrency limiter (reference example/auto_concurrency_limiter):
// a server with max_concurrency="auto" under a burst far above what its
// 2 ms handler can absorb sheds the excess with ELIMIT instead of letting
// latency grow without bound; a constant limit behaves the same way.
#include <atomic>
#include <thread>
#include <vector>

#include "examples/common.h"
#include "rpc/errno.h"

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    int failures = 0;
    for (const char* limit : {"8", "auto"}) {
        mrpc::ServerOptions so;
        so.max_concurrency = mrpc::AdaptiveMaxConcurrency(std::string(limit));
        demo::LocalServer s(std::string("lim-") + limit, 2000, so);
        mrpc::Channel ch;
        mrpc::ChannelOptions opt;
        opt.timeout_ms = 15000;  // shedding, not timeouts, must bound latency (even on a loaded CI box)
        opt.max_retry = 0;
        opt.connection_type = "pooled";
        if (ch.Init(s.addr().c_str(), &opt) != 0) return 1;
        std::atomic<int> ok{0}, limited{0}, other{0};
        std::vector<std::thread> th;
        for (int t = 0; t < 64; ++t) {
            th.emplace_back([&] {
                example::EchoService_Stub stub(&ch);
                for (int i = 0; i < 40; ++i) {
                    mrpc::Controller cntl;
                    example::EchoRequest req;
                    example::EchoResponse res;
                    req.set_message("l");
                    stub.Echo(&cntl, &req, &res, nullptr);
                    if (!cntl.Failed()) ++ok;
                    else if (cntl.ErrorCode() == mrpc::ELIMIT) ++limited;
                    else ++other;
                }
            });
        }
        for (auto& t : th) t.join();
        printf("max_concurrency=%-5s ok=%d rejected(ELIMIT)=%d other=%d\n", limit, ok.load(), limited.load(),
               other.load());
        failures += ok.load() == 0 || other.load() != 0 || (std::string(limit) == "8" && limited.load() == 0);
    }
    return demo::Check(failures == 0, "concurrency limiting");
}
