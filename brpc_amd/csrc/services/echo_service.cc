#include "services/echo_service.h"

#include <cstdlib>
#include <cstring>

#include "fiber/fiber.h"
#include "gpu/device_handler.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/stream.h"

namespace mrpc {

namespace {
// Stream sink of the "stream:<round_bytes>" echo mode (streaming_echo /
// BASELINE config 3): counts received bytes and writes back the cumulative
// count (8 bytes, little endian) every round_bytes, so a sender can time
// rounds end to end. Deletes itself when the stream closes.
class StreamSink : public StreamInputHandler {
public:
    explicit StreamSink(int64_t round) : _round(round > 0 ? round : 1) {}
    int on_received_messages(StreamId id, Buf* const messages[], size_t n) override {
        for (size_t i = 0; i < n; ++i) _bytes += (int64_t)messages[i]->size();
        while (_bytes >= _acked + _round) {
            _acked += _round;
            Buf ack;
            ack.append(&_acked, sizeof(_acked));
            StreamWrite(id, ack);
        }
        return 0;
    }
    void on_closed(StreamId) override { delete this; }

private:
    int64_t _round;
    int64_t _bytes = 0;
    int64_t _acked = 0;
};
}  // namespace

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
    if (cntl->has_remote_stream() && request->message().compare(0, 7, "stream:") == 0) {
        StreamSink* sink = new StreamSink(strtoll(request->message().c_str() + 7, nullptr, 10));
        StreamOptions so;
        so.handler = sink;
        StreamId sid;
        if (StreamAccept(&sid, *cntl, &so) != 0) {
            delete sink;
            cntl->SetFailed(EINTERNAL, "fail to accept the stream");
            return;
        }
    }
    response->set_message(request->message());
    response->set_device(-1);
    if (request->gpu_process()) {
        if (_gpu_device < 0) {
            cntl->SetFailed(EREQUEST, "this server has no GPU for gpu_process");
            return;
        }
        uint32_t crc = 0;
        Buf dev;
        if (gpu::GatherToDeviceWithCrc(cntl->request_attachment(), &dev, &crc, _gpu_device) != 0) {
            cntl->SetFailed(EINTERNAL, "device processing of %zu bytes failed", cntl->request_attachment().size());
            return;
        }
        _gpu_calls.fetch_add(1, std::memory_order_relaxed);
        response->set_device(_gpu_device);
        response->set_crc32c(crc);
        cntl->response_attachment().append(std::move(dev));  // served from HBM
        return;
    }
    // zero-copy echo of the attachment (host or device blocks alike)
    cntl->response_attachment().append(cntl->request_attachment());
}

}  // namespace mrpc
