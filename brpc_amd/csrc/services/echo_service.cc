#include "services/echo_service.h"

#include <cstdlib>
#include <cstring>

#include "base/crc32c.h"
#include "base/time.h"
#include "fiber/fiber.h"
#include "gpu/device_handler.h"
#include "net/socket.h"
#include "policy/device_payload.h"
#include "rpc/channel.h"
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

// Stream relay of the "relay:<round_bytes>:<next>[,<next>...]" mode, the
// pipeline-parallel analog (SURVEY §2.10 PP: a stream chain across GPUs).
// The server opens a stream to the next hop (which relays further, or sinks
// with "stream:" at the end of the chain), forwards every chunk downstream
// in order — device chunks are re-lent to the next GPU over xGMI, never
// staged — and forwards the tail's acknowledgements back upstream, so the
// sender sees end-to-end completion. A full downstream window blocks the
// upstream consumer, which backpressures the sender through its window.
struct RelayState {
    Channel ch;  // to the next hop
    StreamId up = INVALID_STREAM_ID, down = INVALID_STREAM_ID;
};

class RelayUp : public StreamInputHandler {
public:
    explicit RelayUp(std::shared_ptr<RelayState> st) : _st(std::move(st)) {}
    int on_received_messages(StreamId, Buf* const messages[], size_t n) override {
        for (size_t i = 0; i < n; ++i) {
            for (;;) {
                const int rc = StreamWrite(_st->down, *messages[i]);
                if (rc == 0) break;
                if (rc != EAGAIN) return 0;  // downstream gone: on_closed follows
                timespec ts = realtime_after_us(10 * 1000000LL);
                if (StreamWait(_st->down, &ts) != 0) return 0;
            }
        }
        return 0;
    }
    void on_closed(StreamId) override {
        StreamClose(_st->down);
        delete this;
    }

private:
    std::shared_ptr<RelayState> _st;
};

class RelayDown : public StreamInputHandler {
public:
    explicit RelayDown(std::shared_ptr<RelayState> st) : _st(std::move(st)) {}
    int on_received_messages(StreamId, Buf* const messages[], size_t n) override {
        for (size_t i = 0; i < n; ++i) StreamWrite(_st->up, *messages[i]);  // acks: tiny
        return 0;
    }
    void on_closed(StreamId) override {
        StreamClose(_st->up);
        delete this;
    }

private:
    std::shared_ptr<RelayState> _st;
};

// Sets up the relay for `spec` = "<round>:<next>[,<rest>]"; 0 or -1 + *err.
int StartRelay(Controller* cntl, const std::string& spec, int gpu_device, std::string* err) {
    const size_t colon = spec.find(':');
    if (colon == std::string::npos || colon + 1 >= spec.size()) {
        *err = "relay spec must be <round>:<next>[,<next>...]";
        return -1;
    }
    const std::string round = spec.substr(0, colon);
    const std::string hops = spec.substr(colon + 1);
    const size_t comma = hops.find(',');
    const std::string next = hops.substr(0, comma);
    const std::string rest = comma == std::string::npos ? std::string() : hops.substr(comma + 1);
    auto st = std::make_shared<RelayState>();
    ChannelOptions co;
    co.timeout_ms = 10000;
    co.max_retry = 0;
    co.use_device_transport = gpu_device >= 0;
    co.gpu_device = gpu_device;
    co.connection_group = "relay";
    if (st->ch.Init(next.c_str(), &co) != 0) {
        *err = "relay: cannot reach " + next;
        return -1;
    }
    RelayDown* down_h = new RelayDown(st);
    Controller dc;
    StreamOptions dso;
    dso.handler = down_h;
    if (StreamCreate(&st->down, dc, &dso) != 0) {
        delete down_h;
        *err = "relay: StreamCreate failed";
        return -1;
    }
    example::EchoService_Stub stub(&st->ch);
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message(rest.empty() ? "stream:" + round : "relay:" + round + ":" + rest);
    stub.Echo(&dc, &req, &res, nullptr);
    if (dc.Failed()) {
        *err = "relay: next hop " + next + " refused: " + dc.ErrorText();
        return -1;  // the failed stream closes and frees down_h
    }
    RelayUp* up_h = new RelayUp(st);
    StreamOptions uso;
    uso.handler = up_h;
    if (StreamAccept(&st->up, *cntl, &uso) != 0) {
        delete up_h;
        StreamClose(st->down);
        *err = "relay: fail to accept the upstream";
        return -1;
    }
    return 0;
}
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
    if (cntl->has_remote_stream() && request->message().compare(0, 6, "relay:") == 0) {
        std::string err;
        if (StartRelay(cntl, request->message().substr(6), _gpu_device, &err) != 0) {
            cntl->SetFailed(EINTERNAL, "%s", err.c_str());
            return;
        }
    }
    response->set_message(request->message());
    if (request->ids_size()) *response->mutable_ids() = request->ids();
    response->set_device(-1);
    if (request->gpu_process()) {
        if (_gpu_device < 0) {
            cntl->SetFailed(EREQUEST, "this server has no GPU for gpu_process");
            return;
        }
        // The kernel reads the request bytes once and folds their CRC32C.
        // Its output goes where the response travels from: HBM when the
        // client is on a device transport (lent over xGMI), else pinned
        // host memory the socket sends from — one device round trip per
        // batch of requests instead of a gather plus a stage-out.
        bool device_peer = false;
        {
            SocketUniquePtr sock;
            device_peer = Socket::Address(cntl->_server_socket_id, &sock) == 0 && HasDeviceTransport(sock.get());
        }
        // asynchronous: the response is sent from the completion, so this
        // fiber (the connection's reader) goes back to reading at once
        Buf in;
        in.swap(cntl->request_attachment());
        const size_t nbytes = in.size();
        const int dev = _gpu_device;
        std::atomic<int64_t>* calls = &_gpu_calls;
        Closure* d = done_guard.release();
        gpu::ProcessWithCrcAsync(std::move(in), device_peer, dev,
                                 [cntl, response, d, dev, nbytes, calls](int rc, Buf out, uint32_t crc) {
                                     ClosureGuard g(d);
                                     if (rc != 0) {
                                         cntl->SetFailed(EINTERNAL, "device processing of %zu bytes failed (%d: %s)", nbytes, rc,
                                                         gpu::DeviceHandlerErrorText(rc));
                                         return;
                                     }
                                     calls->fetch_add(1, std::memory_order_relaxed);
                                     response->set_device(dev);
                                     response->set_crc32c(crc);
                                     cntl->response_attachment().append(std::move(out));
                                 });
        return;
    }
    if (request->cpu_process()) {
        // the GPU handler's work on the host: checksum, zero-copy echo
        const Buf& in = cntl->request_attachment();
        if (!in.all_host_accessible()) {
            cntl->SetFailed(EREQUEST, "cpu_process needs a host attachment");
            return;
        }
        uint32_t crc = 0;
        for (size_t i = 0; i < in.backing_block_num(); ++i) {
            crc = crc32c::Extend(crc, in.block_data(i), in.block_len(i));
        }
        response->set_device(-1);
        response->set_crc32c(crc);
    }
    // zero-copy echo of the attachment (host or device blocks alike); a
    // device payload goes back the way it came: encoded on the device again
    // if it arrived encoded, indexed by the client if it arrived indexed
    if (cntl->received_device_payload_compress_type() != COMPRESS_TYPE_NONE)
        cntl->set_device_payload_compress_type(cntl->received_device_payload_compress_type());
    if (cntl->device_payload_index().nfields >= 0) cntl->set_device_payload_scan(true);
    cntl->response_attachment().append(cntl->request_attachment());
}

}  // namespace mrpc
