// Cancel (reference example/cancel_c++): an async call to a slow server is
// cancelled with StartCancel; its done runs at once with ECANCELED.
#include <atomic>

#include "base/time.h"
#include "examples/common.h"
#include "rpc/errno.h"

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    demo::LocalServer s("slow", 2000000);
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.timeout_ms = 5000;
    if (ch.Init(s.addr().c_str(), &opt) != 0) return 1;
    example::EchoService_Stub stub(&ch);
    mrpc::Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("cancel me");
    std::atomic<bool> done{false};
    const int64_t t0 = mrpc::monotonic_us();
    stub.Echo(&cntl, &req, &res, mrpc::NewCallback([&done] { done = true; }));
    usleep(20000);
    cntl.StartCancel();
    cntl.Join();
    const int64_t ms = (mrpc::monotonic_us() - t0) / 1000;
    printf("call ended after %lld ms: %s\n", (long long)ms, cntl.ErrorText().c_str());
    return demo::Check(cntl.Failed() && cntl.ErrorCode() == ECANCELED && ms < 1000, "StartCancel");
}
