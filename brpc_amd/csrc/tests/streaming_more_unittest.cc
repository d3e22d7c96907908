// More streaming RPC cases (rpc/stream.h), after the reference's
// test/brpc_streaming_rpc_unittest.cpp: writes to unknown and closed
// streams, a second stream on one controller, an offer whose RPC fails,
// StreamWait edges (writable now, deadline passed, closed while waiting),
// unconsumed-byte accounting that drains back to zero, several streams
// sharing one connection, batch limits on the receiving side, concurrent
// writers on one stream, empty messages, and close from the client side.
#include <unistd.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "base/time.h"
#include "fiber/fiber.h"
#include "fiber/sync.h"
#include "mrpc/proto/echo.pb.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/server.h"
#include "rpc/stream.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

class Sink : public StreamInputHandler {
public:
    int on_received_messages(StreamId, Buf* const messages[], size_t size) override {
        if (sleep_per_batch_us) fiber::usleep(sleep_per_batch_us);
        std::lock_guard<std::mutex> g(mu);
        batches.push_back(size);
        for (size_t i = 0; i < size; ++i) got.push_back(messages[i]->to_string());
        return 0;
    }
    void on_closed(StreamId) override { closed.store(true); }
    size_t count() {
        std::lock_guard<std::mutex> g(mu);
        return got.size();
    }
    std::mutex mu;
    std::vector<std::string> got;
    std::vector<size_t> batches;
    std::atomic<bool> closed{false};
    int64_t sleep_per_batch_us = 0;
};

template <typename F>
bool wait_for(F f, int64_t us = 3000000) {
    const int64_t deadline = monotonic_us() + us;
    while (!f()) {
        if (monotonic_us() > deadline) return false;
        fiber::usleep(2000);
    }
    return true;
}

// The request message names what the server stream does.
class Svc : public example::EchoService {
public:
    void Echo(RpcController* cb, const example::EchoRequest* req, example::EchoResponse* res, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = static_cast<Controller*>(cb);
        auto sink = std::make_shared<Sink>();
        StreamOptions so;
        so.handler = sink.get();
        const std::string& mode = req->message();
        if (mode == "slow") {
            sink->sleep_per_batch_us = 5000;
            so.messages_in_batch = 1;
        }
        if (mode == "batch4") so.messages_in_batch = 4;
        StreamId sid;
        if (StreamAccept(&sid, *cntl, &so) != 0) {
            cntl->SetFailed("accept failed");
            return;
        }
        // a second accept on the same call is refused
        StreamId again;
        if (StreamAccept(&again, *cntl, &so) == 0) second_accept_ok.store(true);
        {
            std::lock_guard<std::mutex> lk(mu);
            sinks.push_back(sink);
            sids.push_back(sid);
        }
        if (mode == "burst") {
            // 4 fibers write 50 messages each into the client's stream
            for (int f = 0; f < 4; ++f) {
                fiber::start([sid, f] {
                    for (int i = 0; i < 50; ++i) {
                        Buf b;
                        b.append(std::to_string(f) + ":" + std::to_string(i));
                        while (StreamWrite(sid, b) == EAGAIN) StreamWait(sid, nullptr);
                    }
                });
            }
        }
        res->set_message(mode);
    }
    std::shared_ptr<Sink> sink_at(size_t i) {
        std::lock_guard<std::mutex> lk(mu);
        return i < sinks.size() ? sinks[i] : nullptr;
    }
    StreamId sid_at(size_t i) {
        std::lock_guard<std::mutex> lk(mu);
        return i < sids.size() ? sids[i] : INVALID_STREAM_ID;
    }
    std::mutex mu;
    std::vector<std::shared_ptr<Sink>> sinks;
    std::vector<StreamId> sids;
    std::atomic<bool> second_accept_ok{false};
};

struct Env {
    Server server;
    Svc svc;
    Channel ch;
    bool ok = false;
    std::vector<StreamId> client_ids;
    std::vector<std::unique_ptr<Sink>> client_sinks;  // outlive the client streams
    Sink& new_sink() {
        client_sinks.emplace_back(new Sink);
        return *client_sinks.back();
    }
    Env() {
        server.AddService(&svc, SERVER_DOESNT_OWN_SERVICE);
        ServerOptions so;
        so.has_builtin_services = false;
        if (server.Start("127.0.0.1:0", &so) != 0) return;
        ChannelOptions opt;
        opt.timeout_ms = 3000;
        ok = ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &opt) == 0;
    }
    ~Env() {
        for (StreamId id : client_ids) StreamClose(id);
        std::vector<StreamId> ids;
        std::vector<std::shared_ptr<Sink>> sinks;
        {
            std::lock_guard<std::mutex> lk(svc.mu);
            ids = svc.sids;
            sinks = svc.sinks;
        }
        for (StreamId id : ids) StreamClose(id);
        for (auto& s : sinks) wait_for([&] { return s->closed.load(); });
        for (auto& s : client_sinks) wait_for([&] { return s->closed.load(); });
    }
    StreamId open(const std::string& mode, Sink* rec, int64_t window = 0) {
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
        if (cntl.Failed()) return INVALID_STREAM_ID;
        client_ids.push_back(sid);
        return sid;
    }
};

Buf msg(const std::string& s) {
    Buf b;
    b.append(s);
    return b;
}

}  // namespace

TEST(StreamingMore, unknown_stream_ids_are_refused) {
    EXPECT_EQ(StreamWrite(INVALID_STREAM_ID, msg("x")), EINVAL);
    EXPECT_EQ(StreamWait(INVALID_STREAM_ID, nullptr), EINVAL);
    EXPECT_EQ(StreamClose(INVALID_STREAM_ID), EINVAL);
    EXPECT_EQ(StreamUnconsumedBytes(INVALID_STREAM_ID), -1);
    EXPECT_FALSE(StreamIsConnected(INVALID_STREAM_ID));
}

TEST(StreamingMore, one_stream_per_controller_and_per_accept) {
    Env e;
    ASSERT_TRUE(e.ok);
    Controller cntl;
    StreamId a, b;
    StreamOptions o;
    ASSERT_EQ(StreamCreate(&a, cntl, &o), 0);
    EXPECT_NE(StreamCreate(&b, cntl, &o), 0);
    StreamClose(a);
    Sink& rec = e.new_sink();
    ASSERT_TRUE(e.open("plain", &rec) != INVALID_STREAM_ID);
    EXPECT_FALSE(e.svc.second_accept_ok.load());
}

TEST(StreamingMore, accept_without_an_offered_stream_fails) {
    Controller cntl;
    StreamId s;
    StreamOptions o;
    EXPECT_NE(StreamAccept(&s, cntl, &o), 0);
}

TEST(StreamingMore, offer_on_a_failed_rpc_is_closed) {
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 500;
    opt.max_retry = 0;
    ASSERT_EQ(ch.Init("127.0.0.1:1", &opt), 0);  // nothing listens there
    Sink rec;
    Controller cntl;
    StreamId sid;
    StreamOptions so;
    so.handler = &rec;
    ASSERT_EQ(StreamCreate(&sid, cntl, &so), 0);
    example::EchoService_Stub stub(&ch);
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("x");
    stub.Echo(&cntl, &req, &res, nullptr);
    EXPECT_TRUE(cntl.Failed());
    EXPECT_FALSE(StreamIsConnected(sid));
    EXPECT_EQ(StreamWrite(sid, msg("late")), EINVAL);
    EXPECT_TRUE(wait_for([&] { return rec.closed.load(); }));  // the handler learns it too
}

TEST(StreamingMore, write_after_close_is_refused_and_a_second_close_is_harmless) {
    Env e;
    ASSERT_TRUE(e.ok);
    Sink& rec = e.new_sink();
    StreamId sid = e.open("plain", &rec);
    ASSERT_TRUE(sid != INVALID_STREAM_ID);
    EXPECT_TRUE(StreamIsConnected(sid));
    EXPECT_EQ(StreamWrite(sid, msg("one")), 0);
    EXPECT_EQ(StreamClose(sid), 0);
    const int again = StreamClose(sid);  // 0 while the stream lingers, EINVAL once it is recycled
    EXPECT_TRUE(again == 0 || again == EINVAL);
    EXPECT_EQ(StreamWrite(sid, msg("two")), EINVAL);
    EXPECT_EQ(StreamWait(sid, nullptr), EINVAL);
    // the server side sees the message written before the close, then the close
    EXPECT_TRUE(wait_for([&] { return e.svc.sink_at(0) && e.svc.sink_at(0)->closed.load(); }));
    std::shared_ptr<Sink> srv = e.svc.sink_at(0);
    std::lock_guard<std::mutex> g(srv->mu);
    ASSERT_EQ(srv->got.size(), 1u);
    EXPECT_EQ(srv->got[0], "one");
}

TEST(StreamingMore, wait_on_a_writable_stream_returns_at_once) {
    Env e;
    ASSERT_TRUE(e.ok);
    Sink& rec = e.new_sink();
    StreamId sid = e.open("plain", &rec);
    ASSERT_TRUE(sid != INVALID_STREAM_ID);
    timespec due = realtime_after_us(1000);
    EXPECT_EQ(StreamWait(sid, &due), 0);
}

TEST(StreamingMore, wait_with_a_full_window_times_out) {
    Env e;
    ASSERT_TRUE(e.ok);
    Sink& rec = e.new_sink();
    StreamId sid = e.open("slow", &rec, 1024);
    ASSERT_TRUE(sid != INVALID_STREAM_ID);
    const std::string kb(1024, 'w');
    EXPECT_EQ(StreamWrite(sid, msg(kb)), 0);
    EXPECT_EQ(StreamWrite(sid, msg(kb)), EAGAIN);  // 1 KiB window, 1 KiB in flight
    // the slow reader's feedback arrives after ~5 ms; a deadline already
    // behind us cannot be met unless it already came
    timespec past = realtime_after_us(-1000);
    const int rc = StreamWait(sid, &past);
    EXPECT_TRUE(rc == ETIMEDOUT || rc == 0);
    timespec later = realtime_after_us(2000000);
    EXPECT_EQ(StreamWait(sid, &later), 0);
    EXPECT_EQ(StreamWrite(sid, msg(kb)), 0);
}

TEST(StreamingMore, close_wakes_a_blocked_waiter) {
    Env e;
    ASSERT_TRUE(e.ok);
    Sink& rec = e.new_sink();
    // a reader that never consumes: a window of 64 bytes fills at once
    StreamId sid = e.open("slow", &rec, 64);
    ASSERT_TRUE(sid != INVALID_STREAM_ID);
    EXPECT_EQ(StreamWrite(sid, msg(std::string(64, 'z'))), 0);
    std::atomic<int> rc{-100};
    fiber::CountdownEvent done(1);
    fiber::start([&] {
        // either the feedback arrives (0) or the close below wakes it (EINVAL)
        timespec due = realtime_after_us(3000000);
        int r = 0;
        while ((r = StreamWrite(sid, msg(std::string(64, 'y')))) == EAGAIN) {
            r = StreamWait(sid, &due);
            if (r != 0) break;
        }
        rc.store(r);
        done.signal();
    });
    fiber::usleep(1000);
    StreamClose(sid);
    done.wait();
    EXPECT_TRUE(rc.load() == 0 || rc.load() == EINVAL);
}

TEST(StreamingMore, unconsumed_bytes_drain_to_zero) {
    Env e;
    ASSERT_TRUE(e.ok);
    Sink& rec = e.new_sink();
    StreamId sid = e.open("plain", &rec);
    ASSERT_TRUE(sid != INVALID_STREAM_ID);
    for (int i = 0; i < 100; ++i) EXPECT_EQ(StreamWrite(sid, msg(std::string(1000, 'a'))), 0);
    EXPECT_TRUE(StreamUnconsumedBytes(sid) <= 100000);
    EXPECT_TRUE(wait_for([&] { return e.svc.sink_at(0) && e.svc.sink_at(0)->count() == 100; }));
    EXPECT_TRUE(wait_for([&] { return StreamUnconsumedBytes(sid) == 0; }));
}

TEST(StreamingMore, several_streams_share_one_connection_in_order) {
    Env e;
    ASSERT_TRUE(e.ok);
    const int kStreams = 4, kMsgs = 200;
    std::vector<StreamId> ids;
    for (int s = 0; s < kStreams; ++s) {
        StreamId id = e.open("plain", &e.new_sink());
        ASSERT_TRUE(id != INVALID_STREAM_ID);
        ids.push_back(id);
    }
    for (int i = 0; i < kMsgs; ++i) {
        for (int s = 0; s < kStreams; ++s) {
            Buf b = msg(std::to_string(s) + "/" + std::to_string(i));
            while (StreamWrite(ids[s], b) == EAGAIN) StreamWait(ids[s], nullptr);
        }
    }
    for (int s = 0; s < kStreams; ++s) {
        ASSERT_TRUE(wait_for([&] { return e.svc.sink_at(s) && e.svc.sink_at(s)->count() == (size_t)kMsgs; }));
    }
    // each server stream got exactly its own client's messages, in order
    for (int s = 0; s < kStreams; ++s) {
        std::shared_ptr<Sink> srv = e.svc.sink_at(s);
        std::lock_guard<std::mutex> g(srv->mu);
        const std::string prefix = srv->got[0].substr(0, srv->got[0].find('/') + 1);
        for (int i = 0; i < kMsgs; ++i) EXPECT_EQ(srv->got[i], prefix + std::to_string(i));
    }
}

TEST(StreamingMore, receiver_batches_respect_messages_in_batch) {
    Env e;
    ASSERT_TRUE(e.ok);
    Sink& rec = e.new_sink();
    StreamId sid = e.open("batch4", &rec);
    ASSERT_TRUE(sid != INVALID_STREAM_ID);
    for (int i = 0; i < 300; ++i) EXPECT_EQ(StreamWrite(sid, msg("m" + std::to_string(i))), 0);
    ASSERT_TRUE(wait_for([&] { return e.svc.sink_at(0) && e.svc.sink_at(0)->count() == 300; }));
    std::shared_ptr<Sink> srv = e.svc.sink_at(0);
    std::lock_guard<std::mutex> g(srv->mu);
    for (size_t b : srv->batches) EXPECT_LE(b, 4u);
    for (int i = 0; i < 300; ++i) EXPECT_EQ(srv->got[i], "m" + std::to_string(i));
}

TEST(StreamingMore, concurrent_server_writers_keep_per_writer_order) {
    Env e;
    ASSERT_TRUE(e.ok);
    Sink& rec = e.new_sink();
    StreamId sid = e.open("burst", &rec);
    ASSERT_TRUE(sid != INVALID_STREAM_ID);
    ASSERT_TRUE(wait_for([&] { return rec.count() == 200; }));
    std::map<int, int> next;
    std::lock_guard<std::mutex> g(rec.mu);
    for (const std::string& s : rec.got) {
        const int f = std::stoi(s.substr(0, s.find(':')));
        const int i = std::stoi(s.substr(s.find(':') + 1));
        EXPECT_EQ(i, next[f]);
        next[f] = i + 1;
    }
    EXPECT_EQ(next.size(), 4u);
}

TEST(StreamingMore, empty_and_large_messages_arrive_intact) {
    Env e;
    ASSERT_TRUE(e.ok);
    Sink& rec = e.new_sink();
    StreamId sid = e.open("plain", &rec);
    ASSERT_TRUE(sid != INVALID_STREAM_ID);
    std::string big(3 * 1024 * 1024 + 7, '\0');
    for (size_t i = 0; i < big.size(); ++i) big[i] = (char)(i * 131 + 7);
    EXPECT_EQ(StreamWrite(sid, msg("")), 0);
    EXPECT_EQ(StreamWrite(sid, msg(big)), 0);  // larger than the 2 MiB window: allowed while nothing is in flight
    int rc;
    while ((rc = StreamWrite(sid, msg("tail"))) == EAGAIN) EXPECT_EQ(StreamWait(sid, nullptr), 0);
    EXPECT_EQ(rc, 0);
    ASSERT_TRUE(wait_for([&] { return e.svc.sink_at(0) && e.svc.sink_at(0)->count() == 3; }));
    std::shared_ptr<Sink> srv = e.svc.sink_at(0);
    std::lock_guard<std::mutex> g(srv->mu);
    EXPECT_TRUE(srv->got[0].empty());
    EXPECT_TRUE(srv->got[1] == big);
    EXPECT_EQ(srv->got[2], "tail");
}

TEST(StreamingMore, server_close_is_seen_and_refuses_client_writes) {
    Env e;
    ASSERT_TRUE(e.ok);
    Sink& rec = e.new_sink();
    StreamId sid = e.open("plain", &rec);
    ASSERT_TRUE(sid != INVALID_STREAM_ID);
    StreamClose(e.svc.sid_at(0));
    ASSERT_TRUE(wait_for([&] { return rec.closed.load(); }));
    EXPECT_TRUE(wait_for([&] { return StreamWrite(sid, msg("after")) == EINVAL; }));
}
