// HTTP server + client (reference example/http_c++): a pb service exposed
// through a RESTful mapping, called with JSON bodies over http/1.1, plus a
// raw-bytes handler reading the unresolved path and query.
#include "examples/common.h"
#include "http/http_header.h"

namespace {
class QueueService : public example::EchoService {
public:
    void Echo(mrpc::RpcController* c, const example::EchoRequest* req, example::EchoResponse* res,
              mrpc::Closure* done) override {
        mrpc::ClosureGuard g(done);
        mrpc::Controller* cntl = static_cast<mrpc::Controller*>(c);
        // restful: /v1/queue/<name>/echo  -> unresolved path = "<name>/echo"
        res->set_message(req->message() + " via " + cntl->http_request().unresolved_path());
    }
};
}  // namespace

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    QueueService svc;
    mrpc::Server server;
    if (server.AddService(&svc, mrpc::SERVER_DOESNT_OWN_SERVICE, "/v1/queue/* => Echo") != 0) return 1;
    if (server.Start("127.0.0.1:0", nullptr) != 0) return 1;
    const std::string addr = "127.0.0.1:" + std::to_string(server.listen_port());
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.protocol = "http";
    opt.timeout_ms = 2000;
    if (ch.Init(("http://" + addr).c_str(), &opt) != 0) return 1;
    int bad = 0;
    {  // JSON body -> pb request -> JSON response
        mrpc::Controller cntl;
        cntl.http_request().uri().set_path("/v1/queue/jobs/echo");
        cntl.http_request().set_method(mrpc::HTTP_METHOD_POST);
        cntl.request_attachment().append("{\"message\":\"hi\"}");
        ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        const std::string body = cntl.response_attachment().to_string();
        printf("POST /v1/queue/jobs/echo -> %d %s", cntl.http_response().status_code(), body.c_str());
        bad += cntl.Failed() || body.find("hi via jobs/echo") == std::string::npos;
    }
    {  // typed stub over http: the pb request travels as JSON
        example::EchoService_Stub stub(&ch);
        mrpc::Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("stub");
        stub.Echo(&cntl, &req, &res, nullptr);
        printf("stub over http -> %s\n", res.message().c_str());
        bad += cntl.Failed();
    }
    {  // builtin pages share the port
        mrpc::Controller cntl;
        cntl.http_request().uri().set_path("/health");
        ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        bad += cntl.Failed();
    }
    return demo::Check(bad == 0, "http + restful + json");
}
