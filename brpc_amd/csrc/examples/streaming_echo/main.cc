// Streaming echo (reference example/streaming_echo_c++): the client opens a
// stream alongside an RPC, writes -messages chunks of -chunk_size bytes with
// flow control (StreamWait on EAGAIN), the server's handler receives them in
// order in batches.
#include <atomic>
#include <mutex>
#include <vector>

#include "base/time.h"
#include "examples/common.h"
#include "rpc/stream.h"

DEFINE_int32(messages, 1000, "messages to stream");
DEFINE_int32(chunk_size, 65536, "bytes per message");

namespace {
class Receiver : public mrpc::StreamInputHandler {
public:
    int on_received_messages(mrpc::StreamId, mrpc::Buf* const msgs[], size_t n) override {
        for (size_t i = 0; i < n; ++i) {
            char head[16] = {0};
            msgs[i]->copy_to(head, 8);
            if (memcmp(head, &next, sizeof(next)) != 0) out_of_order = true;
            ++next;
            bytes += (int64_t)msgs[i]->size();
        }
        batches.fetch_add(1);
        return 0;
    }
    void on_closed(mrpc::StreamId) override { closed = true; }
    int64_t next = 0;
    std::atomic<int64_t> bytes{0};
    std::atomic<int> batches{0};
    std::atomic<bool> closed{false}, out_of_order{false};
};

class StreamingEcho : public example::EchoService {
public:
    void Echo(mrpc::RpcController* c, const example::EchoRequest* req, example::EchoResponse* res,
              mrpc::Closure* done) override {
        mrpc::ClosureGuard g(done);
        mrpc::Controller* cntl = static_cast<mrpc::Controller*>(c);
        mrpc::StreamOptions so;
        so.handler = &receiver;
        mrpc::StreamId sid;
        if (mrpc::StreamAccept(&sid, *cntl, &so) != 0) {
            cntl->SetFailed("fail to accept stream");
            return;
        }
        res->set_message(req->message());
    }
    Receiver receiver;
};
}  // namespace

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    StreamingEcho svc;
    mrpc::Server server;
    server.AddService(&svc, mrpc::SERVER_DOESNT_OWN_SERVICE);
    if (server.Start("127.0.0.1:0", nullptr) != 0) return 1;
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.timeout_ms = 5000;
    if (ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &opt) != 0) return 1;
    mrpc::Controller cntl;
    mrpc::StreamId sid;
    if (mrpc::StreamCreate(&sid, cntl, nullptr) != 0) return 1;
    example::EchoService_Stub stub(&ch);
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("open stream");
    stub.Echo(&cntl, &req, &res, nullptr);
    if (cntl.Failed()) return demo::Check(false, cntl.ErrorText().c_str());
    const int64_t t0 = mrpc::monotonic_us();
    std::string payload(FLAGS_chunk_size, 's');
    for (int64_t i = 0; i < FLAGS_messages; ++i) {
        memcpy(&payload[0], &i, sizeof(i));
        mrpc::Buf b;
        b.append(payload);
        while (mrpc::StreamWrite(sid, b) == EAGAIN) {
            timespec ts = mrpc::realtime_after_us(1000000);
            mrpc::StreamWait(sid, &ts);
        }
    }
    const int64_t want = (int64_t)FLAGS_messages * FLAGS_chunk_size;
    for (int i = 0; i < 1000 && svc.receiver.bytes.load() < want; ++i) usleep(2000);
    const double sec = (mrpc::monotonic_us() - t0) / 1e6;
    mrpc::StreamClose(sid);
    for (int i = 0; i < 200 && !svc.receiver.closed; ++i) usleep(5000);
    printf("streamed %lld bytes in %.3fs (%.2f GB/s) in %d batches\n", (long long)svc.receiver.bytes.load(), sec,
           svc.receiver.bytes.load() / sec / 1e9, svc.receiver.batches.load());
    return demo::Check(svc.receiver.bytes.load() == want && !svc.receiver.out_of_order && svc.receiver.closed,
                       "ordered, flow-controlled stream");
}
