// Streaming-RPC load generator (BASELINE config 3, the reference's
// example/streaming_echo_c++ shape): one stream to an echo server started in
// "stream:<round_bytes>" mode; a step pushes chunks_per_step chunks of
// chunk_size bytes through the flow-controlled stream and ends when the
// server acknowledges the round's bytes on the reverse direction.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>

#include "rpc/channel.h"
#include "rpc/stream.h"

namespace mrpc {
namespace press {

struct StreamPressOptions {
    std::string server = "127.0.0.1:8002";
    int chunk_size = 65536;
    int chunks_per_step = 64;
    int timeout_ms = 10000;
    int64_t max_buf_size = 2 * 1024 * 1024;  // stream window (StreamOptions)
};

class StreamPress : public StreamInputHandler {
public:
    StreamPress() = default;
    ~StreamPress() override;
    int Init(const StreamPressOptions& opt, std::string* err);
    // 0, or -1 with *err (timeout, stream failure).
    int RunSteps(int steps, std::string* err);
    int64_t bytes_sent() const { return _sent; }
    int64_t bytes_acked();
    int64_t steps_done() const { return _steps; }

    // StreamInputHandler (acks from the server)
    int on_received_messages(StreamId id, Buf* const messages[], size_t size) override;
    void on_closed(StreamId id) override;

private:
    StreamPressOptions _opt;
    Channel _ch;
    StreamId _sid = INVALID_STREAM_ID;
    std::string _chunk;
    int64_t _sent = 0, _steps = 0;
    std::mutex _mu;
    std::condition_variable _cv;
    int64_t _acked = 0;
    bool _closed = false;
};

}  // namespace press
}  // namespace mrpc
