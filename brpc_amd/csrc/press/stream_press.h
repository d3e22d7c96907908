// Streaming-RPC load generator (BASELINE config 3, the reference's
// example/streaming_echo_c++ shape): one stream per server, each to an echo
// server started in "stream:<round_bytes>" mode. A step pushes
// chunks_per_step chunks of chunk_size bytes through EVERY stream (writes
// interleave across the streams, so all peers receive concurrently — the
// 64 KiB-chunk fan-out of config 3) and ends when every server acknowledged
// the round's bytes on the reverse direction.
//
// The chunk is built once: each write appends a reference to the same block
// (zero copy). With device_chunks the chunk lives in HBM (arena block) and
// the frames lend it over the xGMI transport: the peers pull it straight
// from this GPU's HBM.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "rpc/channel.h"
#include "rpc/stream.h"

namespace mrpc {
namespace press {

struct StreamPressOptions {
    std::string server = "127.0.0.1:8002";  // one server, or a comma-separated fan-out list
    int chunk_size = 65536;
    int chunks_per_step = 64;
    int timeout_ms = 10000;
    int64_t max_buf_size = 2 * 1024 * 1024;  // stream window (StreamOptions)
    // Rounds in flight: the next round is written while up to this many
    // earlier rounds still wait for their acks (1 = write, wait, repeat).
    // RunSteps drains every ack before it returns either way.
    int pipeline_rounds = 1;
    bool device_chunks = false;              // chunks in HBM, moved over xGMI
    int gpu_device = -1;
    // Pipeline (PP analog): the servers in `server` relay every chunk on
    // through these comma-separated hops before the last one acknowledges.
    std::string relay_chain;
};

class StreamPress {
public:
    StreamPress() = default;
    ~StreamPress();
    int Init(const StreamPressOptions& opt, std::string* err);
    // 0, or -1 with *err (timeout, stream failure). With a deadline
    // (monotonic us, 0: none) no step starts after it; *done (optional)
    // gets the steps completed by this call.
    int RunSteps(int steps, std::string* err, int64_t deadline_us = 0, int* done = nullptr);
    int64_t bytes_sent() const { return _sent; }
    int64_t bytes_acked();
    int64_t steps_done() const { return _steps; }
    int num_streams() const { return (int)_peers.size(); }

private:
    // One stream to one server; receives the cumulative acks.
    struct Peer : public StreamInputHandler {
        StreamPress* owner = nullptr;
        Channel ch;
        StreamId sid = INVALID_STREAM_ID;
        int64_t acked = 0;
        bool closed = false;
        int on_received_messages(StreamId id, Buf* const messages[], size_t size) override;
        void on_closed(StreamId id) override;
    };
    int write_chunk(Peer* p, std::string* err);

    StreamPressOptions _opt;
    std::vector<std::unique_ptr<Peer>> _peers;
    Buf _chunk;  // built once, appended by reference
    int64_t _sent = 0, _steps = 0;
    std::mutex _mu;
    std::condition_variable _cv;
};

}  // namespace press
}  // namespace mrpc
