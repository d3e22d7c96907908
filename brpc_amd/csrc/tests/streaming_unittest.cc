// Streaming RPC behaviour (spirit of the reference's
// test/brpc_streaming_rpc_unittest.cpp): bidirectional ping-pong, writer
// backpressure with the async StreamWait, idle timeouts, close from either
// side, streams ending with their host connection, an offer the server never
// accepts, order across many sizes, and data the server writes before its
// response leaves (reference test/brpc_streaming_rpc_unittest.cpp: sanity,
// received_in_order, server_send_data_before_run_done).
#include <unistd.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "base/time.h"
#include "fiber/fiber.h"
#include "mrpc/proto/echo.pb.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/server.h"
#include "rpc/stream.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

class Recorder : public StreamInputHandler {
public:
    int on_received_messages(StreamId id, Buf* const messages[], size_t size) override {
        if (sleep_per_batch_us) fiber::usleep(sleep_per_batch_us);
        std::vector<std::string> batch;
        for (size_t i = 0; i < size; ++i) batch.push_back(messages[i]->to_string());
        {
            std::lock_guard<std::mutex> g(mu);
            got.insert(got.end(), batch.begin(), batch.end());
        }
        if (pong) {
            for (const std::string& s : batch) {
                Buf b;
                b.append("pong:" + s);
                if (StreamWrite(id, b) != 0) write_errors.fetch_add(1);
            }
        }
        return 0;
    }
    void on_idle_timeout(StreamId) override { idle.fetch_add(1); }
    void on_closed(StreamId) override { closed.store(true); }
    size_t count() {
        std::lock_guard<std::mutex> g(mu);
        return got.size();
    }
    std::mutex mu;
    std::vector<std::string> got;
    std::atomic<bool> closed{false};
    std::atomic<int> idle{0}, write_errors{0};
    bool pong = false;
    int64_t sleep_per_batch_us = 0;
};

// The request message picks the server stream's behaviour.
class ModeService : public example::EchoService {
public:
    void Echo(RpcController* cb, const example::EchoRequest* req, example::EchoResponse* res, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = static_cast<Controller*>(cb);
        auto r = std::make_shared<Recorder>();
        StreamOptions so;
        so.handler = r.get();
        const std::string& mode = req->message();
        if (mode == "noaccept") {  // the stream the client offered is never accepted
            res->set_message(mode);
            return;
        }
        if (mode == "pong") r->pong = true;
        if (mode == "slow") {  // a reader that consumes one message per 20 ms
            r->sleep_per_batch_us = 20000;
            so.messages_in_batch = 1;
        }
        if (mode == "idle") so.idle_timeout_ms = 100;
        StreamId sid;
        if (StreamAccept(&sid, *cntl, &so) != 0) {
            cntl->SetFailed("fail to accept stream");
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            recorders.push_back(r);
            sids.push_back(sid);
        }
        if (mode == "early") {
            // data written before the response (done->Run) leaves: it must
            // reach the client after the stream is established, in order
            for (int i = 0; i < 3; ++i) {
                Buf b;
                b.append("early-" + std::to_string(i));
                if (StreamWrite(sid, b) != 0) r->write_errors.fetch_add(1);
            }
        }
        if (mode == "close") {
            fiber::start([sid] {
                fiber::usleep(50000);
                StreamClose(sid);
            });
        }
        res->set_message(mode);
    }
    std::shared_ptr<Recorder> last() {
        std::lock_guard<std::mutex> lk(mu);
        return recorders.empty() ? nullptr : recorders.back();
    }
    std::mutex mu;
    std::vector<std::shared_ptr<Recorder>> recorders;
    std::vector<StreamId> sids;
};

struct Fixture {
    Server server;
    ModeService svc;
    Channel ch;
    bool ok = false;
    Fixture() {
        server.AddService(&svc, SERVER_DOESNT_OWN_SERVICE);
        ServerOptions so;
        so.has_builtin_services = false;
        if (server.Start("127.0.0.1:0", &so) != 0) return;
        ChannelOptions opt;
        opt.timeout_ms = 3000;
        ok = ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &opt) == 0;
    }
    // The server-side handlers live in svc: their streams report on_closed
    // on a consumer fiber, so close them and wait for that before svc goes.
    ~Fixture() {
        std::vector<StreamId> ids;
        std::vector<std::shared_ptr<Recorder>> recs;
        {
            std::lock_guard<std::mutex> lk(svc.mu);
            ids = svc.sids;
            recs = svc.recorders;
        }
        for (StreamId id : ids) StreamClose(id);
        const int64_t deadline = monotonic_us() + 3000000;
        for (const auto& r : recs) {
            while (!r->closed.load() && monotonic_us() < deadline) fiber::usleep(2000);
        }
    }
    // Opens a stream in `mode`; the client side reports into `rec`.
    // `window`: the client's write window (a writer is bounded by its own
    // max_buf_size, as in the reference's StreamOptions).
    StreamId open(const std::string& mode, Recorder* rec, int64_t window = 0) {
        Controller cntl;
        StreamId sid = INVALID_STREAM_ID;
        StreamOptions copt;
        copt.handler = rec;
        if (window > 0) copt.min_buf_size = copt.max_buf_size = window;
        if (StreamCreate(&sid, cntl, &copt) != 0) return INVALID_STREAM_ID;
        example::EchoService_Stub stub(&ch);
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message(mode);
        stub.Echo(&cntl, &req, &res, nullptr);
        return cntl.Failed() ? INVALID_STREAM_ID : sid;
    }
};

template <typename F>
bool wait_until(F f, int64_t us = 3000000) {
    const int64_t deadline = monotonic_us() + us;
    while (!f()) {
        if (monotonic_us() > deadline) return false;
        fiber::usleep(2000);
    }
    return true;
}

struct WritableArg {
    std::atomic<int> fired{0};
    std::atomic<int> rc{-1};
};

void on_writable(StreamId, void* arg, int rc) {
    auto* a = static_cast<WritableArg*>(arg);
    a->rc.store(rc);
    a->fired.fetch_add(1);
}

}  // namespace

TEST(StreamingRpc, ping_pong_both_directions) {
    Fixture f;
    ASSERT_TRUE(f.ok);
    Recorder client;
    const StreamId sid = f.open("pong", &client);
    ASSERT_NE(sid, INVALID_STREAM_ID);
    const int N = 50;
    for (int i = 0; i < N; ++i) {
        Buf b;
        b.append("p" + std::to_string(i));
        ASSERT_EQ(StreamWrite(sid, b), 0);
    }
    ASSERT_TRUE(wait_until([&] { return client.count() == (size_t)N; }));
    {
        std::lock_guard<std::mutex> g(client.mu);
        for (int i = 0; i < N; ++i) EXPECT_EQ(client.got[i], "pong:p" + std::to_string(i));
    }
    EXPECT_EQ(f.svc.last()->write_errors.load(), 0);
    StreamClose(sid);
    // the handler lives on this frame: on_closed runs on the stream's
    // consumer fiber after StreamClose returns, so wait for it
    EXPECT_TRUE(wait_until([&] { return client.closed.load(); }));
    EXPECT_TRUE(wait_until([&] { return f.svc.last()->closed.load(); }));
}

TEST(StreamingRpc, writer_blocks_until_the_reader_consumes) {
    Fixture f;
    ASSERT_TRUE(f.ok);
    Recorder client;
    const StreamId sid = f.open("slow", &client, 8 * 1024);
    ASSERT_NE(sid, INVALID_STREAM_ID);
    Buf chunk;
    chunk.append(std::string(4096, 'w'));
    int written = 0;
    while (StreamWrite(sid, chunk) == 0) {
        ++written;
        ASSERT_LT(written, 64);  // an 8 KiB window must push back quickly
    }
    EXPECT_LE(written, 4);
    EXPECT_GT(StreamUnconsumedBytes(sid), 0);
    // asynchronous wait: fires once feedback reopens the window
    WritableArg arg;
    timespec due = realtime_after_us(3000000);
    StreamWait(sid, &due, on_writable, &arg);
    ASSERT_TRUE(wait_until([&] { return arg.fired.load() > 0; }));
    EXPECT_EQ(arg.rc.load(), 0);
    EXPECT_EQ(StreamWrite(sid, chunk), 0);
    int total = written + 1;
    // a synchronous wait that cannot succeed in time reports ETIMEDOUT
    while (StreamWrite(sid, chunk) == 0) ++total;
    timespec soon = realtime_after_us(1000);
    EXPECT_EQ(StreamWait(sid, &soon), ETIMEDOUT);
    // every accepted write arrives, and the window drains completely
    ASSERT_TRUE(wait_until([&] { return f.svc.last()->count() == (size_t)total; }));
    EXPECT_TRUE(wait_until([&] { return StreamUnconsumedBytes(sid) == 0; }));
    StreamClose(sid);
    // the handler lives on this frame: on_closed runs on the stream's
    // consumer fiber after StreamClose returns, so wait for it
    EXPECT_TRUE(wait_until([&] { return client.closed.load(); }));
}

TEST(StreamingRpc, idle_timeout_fires_without_traffic) {
    Fixture f;
    ASSERT_TRUE(f.ok);
    Recorder client;
    const StreamId sid = f.open("idle", &client);
    ASSERT_NE(sid, INVALID_STREAM_ID);
    ASSERT_TRUE(wait_until([&] { return f.svc.last() && f.svc.last()->idle.load() >= 2; }, 2000000));
    // traffic resets the idle clock; the stream stays usable
    Buf b;
    b.append("wake");
    EXPECT_EQ(StreamWrite(sid, b), 0);
    EXPECT_TRUE(wait_until([&] { return f.svc.last()->count() == 1; }));
    EXPECT_FALSE(f.svc.last()->closed.load());
    StreamClose(sid);
    // the handler lives on this frame: on_closed runs on the stream's
    // consumer fiber after StreamClose returns, so wait for it
    EXPECT_TRUE(wait_until([&] { return client.closed.load(); }));
}

TEST(StreamingRpc, server_close_reaches_the_client) {
    Fixture f;
    ASSERT_TRUE(f.ok);
    Recorder client;
    const StreamId sid = f.open("close", &client);
    ASSERT_NE(sid, INVALID_STREAM_ID);
    ASSERT_TRUE(wait_until([&] { return client.closed.load(); }));
    Buf b;
    b.append("late");
    EXPECT_EQ(StreamWrite(sid, b), EINVAL);
    EXPECT_FALSE(StreamIsConnected(sid));
    timespec due = realtime_after_us(100000);
    EXPECT_EQ(StreamWait(sid, &due), EINVAL);
}

TEST(StreamingRpc, streams_end_with_their_connection) {
    Recorder client;
    StreamId sid = INVALID_STREAM_ID;
    std::shared_ptr<Recorder> server_side;
    {
        Fixture f;
        ASSERT_TRUE(f.ok);
        sid = f.open("plain", &client);
        ASSERT_NE(sid, INVALID_STREAM_ID);
        server_side = f.svc.last();
        Buf b;
        b.append("x");
        ASSERT_EQ(StreamWrite(sid, b), 0);
        ASSERT_TRUE(wait_until([&] { return server_side->count() == 1; }));
        f.server.Stop(0);
        f.server.Join();
    }
    EXPECT_TRUE(wait_until([&] { return client.closed.load(); }));
    EXPECT_TRUE(wait_until([&] { return server_side->closed.load(); }));
    Buf b;
    b.append("after");
    EXPECT_NE(StreamWrite(sid, b), 0);
    StreamClose(sid);  // closing twice is harmless
}

TEST(StreamingRpc, sanity_stream_the_server_never_accepts_closes) {
    Fixture f;
    ASSERT_TRUE(f.ok);
    Recorder client;
    const StreamId sid = f.open("noaccept", &client);
    ASSERT_NE(sid, INVALID_STREAM_ID);  // the RPC itself succeeded
    EXPECT_TRUE(wait_until([&] { return client.closed.load(); }));
    EXPECT_FALSE(StreamIsConnected(sid));
    Buf b;
    b.append("nobody listens");
    EXPECT_NE(StreamWrite(sid, b), 0);
    StreamClose(sid);
}

TEST(StreamingRpc, received_in_order_across_sizes) {
    Fixture f;
    ASSERT_TRUE(f.ok);
    Recorder client;
    const StreamId sid = f.open("plain", &client);
    ASSERT_NE(sid, INVALID_STREAM_ID);
    // 600 messages of 1 B .. 20 KiB, written back to back (small ones get
    // batched, large ones span several Buf blocks): the reader sees exactly
    // the written sequence
    std::vector<std::string> sent;
    uint32_t x = 12345;
    for (int i = 0; i < 600; ++i) {
        x = x * 1103515245u + 12345u;
        const size_t len = 1 + (x >> 8) % (i % 50 == 0 ? 20000 : 300);
        std::string m = std::to_string(i) + ":" + std::string(len, (char)('a' + i % 26));
        Buf b;
        b.append(m);
        while (StreamWrite(sid, b) == EAGAIN) {
            timespec due = realtime_after_us(1000000);
            StreamWait(sid, &due);
        }
        sent.push_back(std::move(m));
    }
    auto srv = f.svc.last();
    ASSERT_TRUE(wait_until([&] { return srv->count() == sent.size(); }, 10000000));
    {
        std::lock_guard<std::mutex> g(srv->mu);
        for (size_t i = 0; i < sent.size(); ++i) {
            if (srv->got[i] != sent[i]) {
                EXPECT_EQ(srv->got[i].substr(0, 16), sent[i].substr(0, 16));
                break;
            }
        }
    }
    StreamClose(sid);
    EXPECT_TRUE(wait_until([&] { return client.closed.load(); }));
}

TEST(StreamingRpc, server_sends_data_before_its_response) {
    Fixture f;
    ASSERT_TRUE(f.ok);
    Recorder client;
    const StreamId sid = f.open("early", &client);
    ASSERT_NE(sid, INVALID_STREAM_ID);
    ASSERT_TRUE(wait_until([&] { return client.count() == 3; }));
    {
        std::lock_guard<std::mutex> g(client.mu);
        for (int i = 0; i < 3; ++i) EXPECT_EQ(client.got[i], "early-" + std::to_string(i));
    }
    EXPECT_EQ(f.svc.last()->write_errors.load(), 0);
    StreamClose(sid);
    EXPECT_TRUE(wait_until([&] { return client.closed.load(); }));
}
