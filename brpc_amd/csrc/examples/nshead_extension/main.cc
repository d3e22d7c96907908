// nshead extension (reference example/nshead_extension_c++): a server
// whose whole protocol is "36-byte nshead + opaque body", handled by an
// NsheadService (ServerOptions::nshead_service), and a client Channel with
// protocol "nshead" sending NsheadMessage requests. nshead carries no
// correlation id, so the server answers each connection in request order
// even when handlers finish out of order (asynchronous calls below).
#include <algorithm>
#include <atomic>
#include <memory>
#include <vector>

#include "examples/common.h"
#include "rpc/nshead.h"

DEFINE_int32(calls, 64, "asynchronous calls in flight on one connection");

namespace {
// Answers with the body upper-cased; odd log ids take longer, so the
// completions happen out of order.
class UpperService : public mrpc::NsheadService {
public:
    void ProcessNsheadRequest(const mrpc::Server&, mrpc::Controller*, const mrpc::NsheadMessage& req,
                              mrpc::NsheadMessage* res, mrpc::NsheadClosure* done) override {
        if (req.head.log_id % 2) mrpc::fiber::usleep(2000);
        std::string s = req.body.to_string();
        std::transform(s.begin(), s.end(), s.begin(), ::toupper);
        res->head = req.head;  // echo id/log_id/provider back
        res->body.append(s);
        done->Run();
        ++handled;
    }
    std::atomic<int> handled{0};
};
}  // namespace

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    UpperService svc;
    mrpc::Server server;
    mrpc::ServerOptions so;
    so.nshead_service = &svc;
    if (server.Start("127.0.0.1:0", &so) != 0) return 1;
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.protocol = "nshead";
    opt.timeout_ms = 3000;
    if (ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &opt) != 0) return 1;

    const int n = FLAGS_calls;
    std::vector<std::unique_ptr<mrpc::Controller>> cntls(n);
    std::vector<mrpc::NsheadMessage> reqs(n), ress(n);
    for (int i = 0; i < n; ++i) {
        cntls[i].reset(new mrpc::Controller);
        reqs[i].head.log_id = (uint32_t)i;
        reqs[i].head.id = 7;
        memcpy(reqs[i].head.provider, "demo", 5);
        reqs[i].body.append("hello nshead " + std::to_string(i));
        ch.CallMethod(nullptr, cntls[i].get(), &reqs[i], &ress[i], mrpc::NewCallback([] {}));
    }
    bool ok = true;
    for (int i = 0; i < n; ++i) {
        cntls[i]->Join();
        std::string want = "HELLO NSHEAD " + std::to_string(i);
        ok = ok && !cntls[i]->Failed() && ress[i].body.to_string() == want && ress[i].head.log_id == (uint32_t)i &&
             strcmp(ress[i].head.provider, "demo") == 0;
    }
    printf("%d nshead calls answered in order, head fields preserved, handled=%d\n", n, svc.handled.load());
    server.Stop(0);
    server.Join();
    return demo::Check(ok, "nshead service");
}
