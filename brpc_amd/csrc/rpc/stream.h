// Streaming RPC (role of src/brpc/stream.h:50-88, stream.cpp:274-756):
// ordered, flow-controlled, bidirectional message streams multiplexed on the
// host connection of an RPC. The writer is blocked when produced >=
// remote_consumed + window; the receiver consumes in batches (<=
// messages_in_batch) through an ExecutionQueue and reports consumption with
// FEEDBACK frames. MI355X usage: chunked tensor streams (64 KB chunks fanned
// out to peer GPUs, BASELINE config 3) — chunks may be DEVICE Bufs which are
// moved by the host socket's device transport.
#pragma once

#include <time.h>

#include <cstddef>
#include <cstdint>

#include "base/buf.h"

namespace mrpc {

class Controller;
typedef uint64_t StreamId;
const StreamId INVALID_STREAM_ID = 0;

class StreamInputHandler {
public:
    virtual ~StreamInputHandler() {}
    virtual int on_received_messages(StreamId id, Buf* const messages[], size_t size) = 0;
    virtual void on_idle_timeout(StreamId id) { (void)id; }
    virtual void on_closed(StreamId id) = 0;
};

struct StreamOptions {
    // Flow-control window grows from min to max buffer size.
    int64_t min_buf_size = 1024 * 1024;
    int64_t max_buf_size = 2 * 1024 * 1024;
    int64_t idle_timeout_ms = -1;
    size_t messages_in_batch = 128;
    StreamInputHandler* handler = nullptr;
};

struct StreamWriteOptions {
    bool write_in_background = false;
};

int StreamCreate(StreamId* request_stream, Controller& cntl, const StreamOptions* options);
int StreamAccept(StreamId* response_stream, Controller& cntl, const StreamOptions* options);
// 0 on success; EAGAIN when the window is full; EINVAL when closed.
int StreamWrite(StreamId stream_id, const Buf& message, const StreamWriteOptions* options = nullptr);
// Wait until writable (or due_time). 0 / ETIMEDOUT / EINVAL.
int StreamWait(StreamId stream_id, const timespec* due_time);
void StreamWait(StreamId stream_id, const timespec* due_time, void (*on_writable)(StreamId, void*, int), void* arg);
int StreamClose(StreamId stream_id);
// Introspection (for tests / /streams)
int64_t StreamUnconsumedBytes(StreamId id);
bool StreamIsConnected(StreamId id);

}  // namespace mrpc
