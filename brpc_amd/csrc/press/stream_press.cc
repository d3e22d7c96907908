#include "press/stream_press.h"

#include <algorithm>
#include <cstring>

#include "base/time.h"
#include "base/util.h"
#include "gpu/gpu.h"
#include "gpu/hbm_pool.h"
#include "mrpc/proto/echo.pb.h"
#include "rpc/controller.h"

namespace mrpc {
namespace press {

StreamPress::~StreamPress() {
    for (auto& p : _peers) {
        if (p->sid != INVALID_STREAM_ID) StreamClose(p->sid);
    }
    std::unique_lock<std::mutex> g(_mu);
    _cv.wait_for(g, std::chrono::seconds(2), [this] {
        for (auto& p : _peers) {
            if (p->sid != INVALID_STREAM_ID && !p->closed) return false;
        }
        return true;
    });
}

int StreamPress::Init(const StreamPressOptions& opt, std::string* err) {
    _opt = opt;
    std::vector<std::string> servers;
    for (const std::string& s : split_string(opt.server, ',')) {
        if (!s.empty()) servers.push_back(s);
    }
    if (servers.empty()) {
        *err = "no server";
        return -1;
    }
    // the chunk, built once
    std::string bytes((size_t)opt.chunk_size, '\0');
    for (size_t i = 0; i < bytes.size(); ++i) bytes[i] = (char)(i * 131 + 7);
    if (opt.device_chunks) {
        if (gpu::Init(opt.gpu_device, err) != 0) return -1;
        void* d = gpu::AppendNewDeviceBlock(&_chunk, bytes.size(), opt.gpu_device);
        if (!d || gpu::CopyHostToDevice(d, bytes.data(), bytes.size(), opt.gpu_device) != 0) {
            *err = "fail to stage the chunk in HBM";
            return -1;
        }
    } else {
        _chunk.append(bytes);
    }
    for (const std::string& server : servers) {
        std::unique_ptr<Peer> p(new Peer);
        p->owner = this;
        ChannelOptions co;
        co.timeout_ms = opt.timeout_ms;
        co.max_retry = 0;
        co.use_device_transport = opt.device_chunks;
        co.gpu_device = opt.gpu_device;
        // one connection per peer server (distinct groups never share)
        co.connection_group = "stream_press";
        if (p->ch.Init(server.c_str(), &co) != 0) {
            *err = "fail to init channel to " + server;
            return -1;
        }
        Controller cntl;
        StreamOptions so;
        so.handler = p.get();
        so.max_buf_size = opt.max_buf_size;
        so.min_buf_size = std::min<int64_t>(opt.max_buf_size, 1024 * 1024);
        if (StreamCreate(&p->sid, cntl, &so) != 0) {
            *err = "StreamCreate failed";
            return -1;
        }
        example::EchoService_Stub stub(&p->ch);
        example::EchoRequest req;
        example::EchoResponse res;
        const std::string round = std::to_string((int64_t)opt.chunk_size * opt.chunks_per_step);
        req.set_message(opt.relay_chain.empty() ? "stream:" + round : "relay:" + round + ":" + opt.relay_chain);
        stub.Echo(&cntl, &req, &res, nullptr);
        if (cntl.Failed()) {
            *err = "stream handshake with " + server + " failed: " + cntl.ErrorText();
            p->sid = INVALID_STREAM_ID;
            return -1;
        }
        _peers.push_back(std::move(p));
    }
    return 0;
}

int StreamPress::write_chunk(Peer* p, std::string* err) {
    for (;;) {
        const int rc = StreamWrite(p->sid, _chunk);  // shares the chunk's block
        if (rc == 0) return 0;
        if (rc != EAGAIN) {
            *err = "StreamWrite failed: " + std::string(strerror(rc));
            return -1;
        }
        timespec ts = realtime_after_us((int64_t)_opt.timeout_ms * 1000);
        if (StreamWait(p->sid, &ts) != 0) {
            *err = "stream window never reopened";
            return -1;
        }
    }
}

int StreamPress::RunSteps(int steps, std::string* err, int64_t deadline_us, int* done) {
    if (done) *done = 0;
    const int64_t round = (int64_t)_opt.chunk_size * _opt.chunks_per_step;
    const int depth = std::max(1, _opt.pipeline_rounds);
    // every peer acknowledged `rounds` complete rounds (cumulative acks)
    auto wait_acked = [&](int64_t rounds) -> int {
        const int64_t want = rounds * round;
        std::unique_lock<std::mutex> g(_mu);
        const bool ok = _cv.wait_for(g, std::chrono::milliseconds(_opt.timeout_ms), [&] {
            for (auto& p : _peers) {
                if (p->closed || p->acked < want) return p->closed;
            }
            return true;
        });
        for (auto& p : _peers) {
            if (!ok || p->acked < want) {
                *err = p->closed ? "stream closed by the server" : "timed out waiting for the round's ack";
                return -1;
            }
        }
        return 0;
    };
    const int64_t first = _steps;
    for (int s = 0; s < steps; ++s) {
        if (deadline_us && monotonic_us() >= deadline_us) {
            steps = s;  // no step starts after the deadline
            break;
        }
        for (int c = 0; c < _opt.chunks_per_step; ++c) {
            for (auto& p : _peers) {
                if (write_chunk(p.get(), err) != 0) return -1;
                _sent += _opt.chunk_size;
            }
        }
        // round first+s+1 is written; keep at most depth-1 rounds unacked
        const int64_t must = first + s + 1 - (depth - 1);
        if (must > first && wait_acked(must) != 0) return -1;
    }
    if (steps > 0 && wait_acked(first + steps) != 0) return -1;
    _steps = first + steps;
    if (done) *done = steps;
    return 0;
}

int64_t StreamPress::bytes_acked() {
    std::lock_guard<std::mutex> g(_mu);
    int64_t t = 0;
    for (auto& p : _peers) t += p->acked;
    return t;
}

int StreamPress::Peer::on_received_messages(StreamId, Buf* const messages[], size_t size) {
    int64_t latest = -1;
    for (size_t i = 0; i < size; ++i) {
        if (messages[i]->size() >= sizeof(int64_t)) messages[i]->copy_to(&latest, sizeof(latest));
    }
    if (latest >= 0) {
        std::lock_guard<std::mutex> g(owner->_mu);
        if (latest > acked) acked = latest;
        owner->_cv.notify_all();
    }
    return 0;
}

void StreamPress::Peer::on_closed(StreamId) {
    std::lock_guard<std::mutex> g(owner->_mu);
    closed = true;
    owner->_cv.notify_all();
}

}  // namespace press
}  // namespace mrpc
