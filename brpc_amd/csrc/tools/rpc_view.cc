// rpc_view: browse the builtin pages of a server that is not reachable from
// your browser (role of the reference's tools/rpc_view). Runs an http server
// on -port whose http_master_service fetches the same path + query from
// -target and relays status, content type and body; /rpc_view/health tells
// whether the target answers.
#include "base/flags.h"
#include "base/logging.h"
#include "http/http_client.h"
#include "http/http_header.h"
#include "mrpc/proto/tools.pb.h"
#include "rpc/controller.h"
#include "rpc/server.h"

DEFINE_int32(port, 8888, "port of the viewer");
DEFINE_string(target, "", "ip:port of the server to view");
DEFINE_int32(timeout_ms, 5000, "timeout of one relayed request");

using namespace mrpc;

namespace {

class ViewServiceImpl : public tools::ViewService {
public:
    void default_method(RpcController* c, const tools::ViewRequest*, tools::ViewResponse*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = static_cast<Controller*>(c);
        const HttpHeader& h = cntl->http_request();
        std::string path = "/" + h.unresolved_path();
        const std::string q = h.uri().query_string();
        std::string url = "http://" + FLAGS_target + path + (q.empty() ? "" : "?" + q);
        HttpSimpleResponse resp;
        if (HttpFetch("GET", url, "", &resp, FLAGS_timeout_ms) != 0 && resp.status == 0) {
            cntl->http_response().set_status_code(502);
            cntl->response_attachment().append("rpc_view: fail to reach " + FLAGS_target + "\n");
            return;
        }
        cntl->http_response().set_status_code(resp.status);
        auto ct = resp.headers.find("content-type");
        if (ct == resp.headers.end()) ct = resp.headers.find("Content-Type");
        if (ct != resp.headers.end()) cntl->http_response().set_content_type(ct->second);
        // rewrite absolute links so they stay on the viewer
        cntl->response_attachment().append(resp.body);
    }
};

}  // namespace

int main(int argc, char** argv) {
    ParseCommandLineFlags(&argc, &argv);
    if (FLAGS_target.empty()) {
        LOG(ERROR) << "-target=ip:port is required";
        return 1;
    }
    ViewServiceImpl view;
    Server server;
    ServerOptions opt;
    opt.http_master_service = &view;
    opt.has_builtin_services = false;  // every path belongs to the target
    if (server.Start(FLAGS_port, &opt) != 0) {
        LOG(ERROR) << "Fail to start rpc_view on port " << FLAGS_port;
        return 1;
    }
    LOG(INFO) << "Viewing " << FLAGS_target << " at http://0.0.0.0:" << FLAGS_port;
    server.RunUntilAskedToQuit();
    return 0;
}
