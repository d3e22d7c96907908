// Progressive (streamed) HTTP bodies: the server side writes a response body
// piece by piece after the RPC completed (ProgressiveAttachment, role of
// src/brpc/progressive_attachment.h:32), the client side consumes a large
// response as it arrives (ProgressiveReader, src/brpc/progressive_reader.h).
// Bodies go out with chunked transfer coding.
#pragma once

#include <atomic>
#include <memory>
#include <mutex>

#include "base/buf.h"
#include "base/endpoint.h"
#include "base/util.h"
#include "net/socket.h"
#include "pb/service.h"

namespace mrpc {

class ProgressiveReader {
public:
    virtual ~ProgressiveReader() {}
    // Called for each piece of the body; a non-OK status stops reading.
    virtual Status OnReadOnePart(const void* data, size_t length) = 0;
    // Called once at the end (OK, or the error that cut the body short).
    virtual void OnEndOfMessage(const Status& status) = 0;
};

class ProgressiveAttachment {
public:
    ProgressiveAttachment(SocketId sid, bool before_http_1_1);
    ~ProgressiveAttachment();
    // Append a piece of the body. Before the response header went out the
    // data is buffered; afterwards each call is one chunk on the wire.
    // Returns 0, or -1 with errno (the connection is gone).
    int Write(const Buf& data);
    int Write(const void* data, size_t n);
    int Write(const std::string& s) { return Write(s.data(), s.size()); }
    EndPoint remote_side() const;
    // `done` runs when the body is finished or the connection broke.
    void NotifyOnStopped(Closure* done);

    // protocol internal: the header was sent (or the RPC failed)
    void MarkRPCAsDone(bool rpc_failed);
    // The response said "Connection: close": half-close after the last chunk.
    void set_shutdown_after_end() { _shutdown_after_end = true; }

private:
    int write_chunk(Buf* frame);
    SocketId _sid;
    bool _before_http_1_1;
    bool _shutdown_after_end = false;
    std::mutex _mu;
    bool _header_sent = false;
    bool _rpc_failed = false;
    Buf _saved;
    Closure* _notify = nullptr;
};

}  // namespace mrpc
