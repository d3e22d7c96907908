// Asynchronous echo (reference example/asynchronous_echo_c++): calls return
// immediately and a closure runs when the response arrives.
#include <atomic>

#include "examples/common.h"
#include "fiber/sync.h"

DEFINE_int32(calls, 100, "async calls to issue");

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    demo::LocalServer s("async");
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.timeout_ms = 2000;
    if (ch.Init(s.addr().c_str(), &opt) != 0) return 1;
    example::EchoService_Stub stub(&ch);
    std::atomic<int> ok{0};
    mrpc::fiber::CountdownEvent all(FLAGS_calls);
    for (int i = 0; i < FLAGS_calls; ++i) {
        auto* cntl = new mrpc::Controller;
        auto* req = new example::EchoRequest;
        auto* res = new example::EchoResponse;
        req->set_message("async-" + std::to_string(i));
        stub.Echo(cntl, req, res, mrpc::NewCallback([cntl, req, res, &ok, &all] {
            if (!cntl->Failed() && res->message() == req->message() + "@async") ok.fetch_add(1);
            delete cntl;
            delete req;
            delete res;
            all.signal();
        }));
    }
    all.wait();
    printf("%d/%d async calls completed\n", ok.load(), FLAGS_calls);
    return demo::Check(ok.load() == FLAGS_calls, "asynchronous echo");
}
