// Session-local data (reference example/session_data_and_thread_local):
// ServerOptions.session_local_data_factory hands every call a pooled object
// reused across calls, so handlers keep per-call scratch without mallocs.
#include <atomic>

#include "examples/common.h"

namespace {
struct Scratch {
    int uses = 0;
    std::string buffer;
};
std::atomic<int> g_created{0};

class ScratchFactory : public mrpc::DataFactory {
public:
    void* CreateData() const override {
        g_created.fetch_add(1);
        return new Scratch;
    }
    void DestroyData(void* d) const override { delete static_cast<Scratch*>(d); }
};

class ScratchEcho : public example::EchoService {
public:
    void Echo(mrpc::RpcController* c, const example::EchoRequest* req, example::EchoResponse* res,
              mrpc::Closure* done) override {
        mrpc::ClosureGuard g(done);
        auto* s = static_cast<Scratch*>(static_cast<mrpc::Controller*>(c)->session_local_data());
        if (!s) {
            static_cast<mrpc::Controller*>(c)->SetFailed("no session data");
            return;
        }
        ++s->uses;
        s->buffer.assign(req->message());
        res->set_message(s->buffer + " (scratch used " + std::to_string(s->uses) + "x)");
    }
};
}  // namespace

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    ScratchFactory factory;
    ScratchEcho svc;
    mrpc::Server server;
    server.AddService(&svc, mrpc::SERVER_DOESNT_OWN_SERVICE);
    mrpc::ServerOptions so;
    so.session_local_data_factory = &factory;
    if (server.Start("127.0.0.1:0", &so) != 0) return 1;
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.timeout_ms = 2000;
    if (ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &opt) != 0) return 1;
    example::EchoService_Stub stub(&ch);
    int ok = 0;
    for (int i = 0; i < 200; ++i) {
        mrpc::Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("s" + std::to_string(i));
        stub.Echo(&cntl, &req, &res, nullptr);
        ok += !cntl.Failed();
    }
    printf("200 calls, %d ok, %d scratch objects created\n", ok, g_created.load());
    return demo::Check(ok == 200 && g_created.load() < 50, "pooled session data");
}
