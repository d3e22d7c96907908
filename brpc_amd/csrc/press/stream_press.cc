#include "press/stream_press.h"

#include <cstring>

#include "base/time.h"
#include "mrpc/proto/echo.pb.h"
#include "rpc/controller.h"

namespace mrpc {
namespace press {

StreamPress::~StreamPress() {
    if (_sid != INVALID_STREAM_ID) {
        StreamClose(_sid);
        std::unique_lock<std::mutex> g(_mu);
        _cv.wait_for(g, std::chrono::seconds(2), [this] { return _closed; });
    }
}

int StreamPress::Init(const StreamPressOptions& opt, std::string* err) {
    _opt = opt;
    ChannelOptions co;
    co.timeout_ms = opt.timeout_ms;
    co.max_retry = 0;
    if (_ch.Init(opt.server.c_str(), &co) != 0) {
        *err = "fail to init channel to " + opt.server;
        return -1;
    }
    Controller cntl;
    StreamOptions so;
    so.handler = this;
    so.max_buf_size = opt.max_buf_size;
    so.min_buf_size = std::min<int64_t>(opt.max_buf_size, 1024 * 1024);
    if (StreamCreate(&_sid, cntl, &so) != 0) {
        *err = "StreamCreate failed";
        return -1;
    }
    example::EchoService_Stub stub(&_ch);
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("stream:" + std::to_string((int64_t)opt.chunk_size * opt.chunks_per_step));
    stub.Echo(&cntl, &req, &res, nullptr);
    if (cntl.Failed()) {
        *err = "stream handshake failed: " + cntl.ErrorText();
        _sid = INVALID_STREAM_ID;
        return -1;
    }
    _chunk.assign((size_t)opt.chunk_size, '\0');
    for (size_t i = 0; i < _chunk.size(); ++i) _chunk[i] = (char)(i * 131 + 7);
    return 0;
}

int StreamPress::RunSteps(int steps, std::string* err) {
    const int64_t round = (int64_t)_opt.chunk_size * _opt.chunks_per_step;
    for (int s = 0; s < steps; ++s) {
        for (int c = 0; c < _opt.chunks_per_step; ++c) {
            Buf b;
            b.append(_chunk);
            for (;;) {
                const int rc = StreamWrite(_sid, b);
                if (rc == 0) break;
                if (rc != EAGAIN) {
                    *err = "StreamWrite failed: " + std::string(strerror(rc));
                    return -1;
                }
                timespec ts = realtime_after_us((int64_t)_opt.timeout_ms * 1000);
                if (StreamWait(_sid, &ts) != 0) {
                    *err = "stream window never reopened";
                    return -1;
                }
            }
            _sent += _opt.chunk_size;
        }
        std::unique_lock<std::mutex> g(_mu);
        const int64_t want = (_steps + 1) * round;
        if (!_cv.wait_for(g, std::chrono::milliseconds(_opt.timeout_ms), [&] { return _acked >= want || _closed; }) ||
            _acked < want) {
            *err = _closed ? "stream closed by the server" : "timed out waiting for the round's ack";
            return -1;
        }
        ++_steps;
    }
    return 0;
}

int64_t StreamPress::bytes_acked() {
    std::lock_guard<std::mutex> g(_mu);
    return _acked;
}

int StreamPress::on_received_messages(StreamId, Buf* const messages[], size_t size) {
    int64_t latest = -1;
    for (size_t i = 0; i < size; ++i) {
        if (messages[i]->size() >= sizeof(int64_t)) messages[i]->copy_to(&latest, sizeof(latest));
    }
    if (latest >= 0) {
        std::lock_guard<std::mutex> g(_mu);
        if (latest > _acked) _acked = latest;
        _cv.notify_all();
    }
    return 0;
}

void StreamPress::on_closed(StreamId) {
    std::lock_guard<std::mutex> g(_mu);
    _closed = true;
    _cv.notify_all();
}

}  // namespace press
}  // namespace mrpc
