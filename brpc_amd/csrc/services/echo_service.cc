#include "services/echo_service.h"

#include "fiber/fiber.h"
#include "rpc/controller.h"
#include "rpc/errno.h"

namespace mrpc {

void (*EchoServiceImpl::device_hook)(RpcController* cntl, example::EchoResponse* response) = nullptr;

void EchoServiceImpl::Echo(RpcController* cntl_base, const example::EchoRequest* request,
                           example::EchoResponse* response, Closure* done) {
    ClosureGuard done_guard(done);
    Controller* cntl = static_cast<Controller*>(cntl_base);
    _ncalls.fetch_add(1, std::memory_order_relaxed);
    if (request->sleep_us() > 0) fiber::usleep((uint64_t)request->sleep_us());
    if (request->server_fail()) {
        cntl->SetFailed(request->code() ? request->code() : EINTERNAL, "server_fail requested");
        return;
    }
    if (request->close_fd()) {
        cntl->CloseConnection("close_fd requested");
        return;
    }
    response->set_message(request->message());
    response->set_device(-1);
    // zero-copy echo of the attachment (host or device blocks alike)
    cntl->response_attachment().append(cntl->request_attachment());
    if (device_hook && !cntl->request_attachment().empty()) device_hook(cntl, response);
}

}  // namespace mrpc
