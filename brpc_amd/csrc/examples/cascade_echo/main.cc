// Cascade echo (reference example/cascade_echo_c++): a server's handler
// calls the next server synchronously (the fiber parks, no pthread blocks),
// forming a chain of -depth servers; the response carries every hop.
#include <memory>
#include <vector>

#include "examples/common.h"

DEFINE_int32(depth, 4, "servers in the chain");

namespace {
class CascadeEcho : public example::EchoService {
public:
    CascadeEcho(std::string tag, mrpc::Channel* next) : _tag(std::move(tag)), _next(next) {}
    void Echo(mrpc::RpcController* c, const example::EchoRequest* req, example::EchoResponse* res,
              mrpc::Closure* done) override {
        mrpc::ClosureGuard g(done);
        if (!_next) {
            res->set_message(req->message() + ">" + _tag);
            return;
        }
        example::EchoService_Stub stub(_next);
        mrpc::Controller sub;
        example::EchoRequest r2;
        r2.set_message(req->message() + ">" + _tag);
        stub.Echo(&sub, &r2, res, nullptr);
        if (sub.Failed()) static_cast<mrpc::Controller*>(c)->SetFailed(sub.ErrorCode(), "%s", sub.ErrorText().c_str());
    }

private:
    std::string _tag;
    mrpc::Channel* _next;
};
}  // namespace

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    std::vector<std::unique_ptr<mrpc::Server>> servers;
    std::vector<std::unique_ptr<CascadeEcho>> svcs;
    std::vector<std::unique_ptr<mrpc::Channel>> chans;
    mrpc::Channel* next = nullptr;
    std::string expect = "x";
    for (int i = FLAGS_depth - 1; i >= 0; --i) {
        svcs.emplace_back(new CascadeEcho("s" + std::to_string(i), next));
        servers.emplace_back(new mrpc::Server);
        servers.back()->AddService(svcs.back().get(), mrpc::SERVER_DOESNT_OWN_SERVICE);
        if (servers.back()->Start("127.0.0.1:0", nullptr) != 0) return 1;
        chans.emplace_back(new mrpc::Channel);
        mrpc::ChannelOptions opt;
        opt.timeout_ms = 3000;
        chans.back()->Init(("127.0.0.1:" + std::to_string(servers.back()->listen_port())).c_str(), &opt);
        next = chans.back().get();
    }
    for (int i = 0; i < FLAGS_depth; ++i) expect += ">s" + std::to_string(i);
    example::EchoService_Stub stub(next);
    mrpc::Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("x");
    stub.Echo(&cntl, &req, &res, nullptr);
    printf("response: %s\n", res.message().c_str());
    return demo::Check(!cntl.Failed() && res.message() == expect, "cascaded calls");
}
