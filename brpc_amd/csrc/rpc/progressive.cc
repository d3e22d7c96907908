#include "rpc/progressive.h"

#include <cerrno>
#include <cstdio>

#include "rpc/errno.h"

namespace mrpc {

ProgressiveAttachment::ProgressiveAttachment(SocketId sid, bool before_http_1_1)
    : _sid(sid), _before_http_1_1(before_http_1_1) {}

ProgressiveAttachment::~ProgressiveAttachment() {
    bool send_end = false;
    Closure* notify;
    {
        std::lock_guard<std::mutex> g(_mu);
        send_end = _header_sent && !_rpc_failed;
        notify = _notify;
        _notify = nullptr;
    }
    SocketUniquePtr s;
    if (send_end && Socket::Address(_sid, &s) == 0) {
        // HTTP/1.0: the body ends where the connection does, so half-close
        // it once everything queued is written; HTTP/1.1: the last chunk
        // (then the same half-close for "Connection: close")
        Buf end;
        if (!_before_http_1_1) end.append("0\r\n\r\n", 5);
        WriteOptions opt;
        opt.ignore_eovercrowded = true;
        opt.shutdown_write_after = _before_http_1_1 || _shutdown_after_end;
        s->Write(&end, &opt);
    }
    if (notify) notify->Run();
}

int ProgressiveAttachment::write_chunk(Buf* payload) {
    SocketUniquePtr s;
    if (Socket::Address(_sid, &s) != 0) {
        errno = ECONNRESET;
        return -1;
    }
    Buf frame;
    if (!_before_http_1_1) {
        char head[32];
        const int n = snprintf(head, sizeof(head), "%zx\r\n", payload->size());
        frame.append(head, n);
        frame.append(std::move(*payload));
        frame.append("\r\n", 2);
    } else {
        frame.append(std::move(*payload));
    }
    WriteOptions opt;
    opt.ignore_eovercrowded = false;
    return s->Write(&frame, &opt);
}

int ProgressiveAttachment::Write(const Buf& data) {
    if (data.empty()) return 0;
    std::unique_lock<std::mutex> g(_mu);
    if (_rpc_failed) {
        errno = ECANCELED;
        return -1;
    }
    if (!_header_sent) {
        _saved.append(data);
        return 0;
    }
    g.unlock();
    Buf copy(data);
    return write_chunk(&copy);
}

int ProgressiveAttachment::Write(const void* data, size_t n) {
    Buf b;
    b.append(data, n);
    return Write(b);
}

EndPoint ProgressiveAttachment::remote_side() const {
    SocketUniquePtr s;
    if (Socket::AddressFailedAsWell(_sid, &s) != 0) return EndPoint();
    return s->remote_side();
}

void ProgressiveAttachment::NotifyOnStopped(Closure* done) {
    if (!done) return;
    {
        std::lock_guard<std::mutex> g(_mu);
        if (!_rpc_failed) {
            if (_notify) _notify->Run();
            _notify = done;
            // also fire when the connection breaks
            SocketUniquePtr s;
            if (Socket::Address(_sid, &s) == 0) {
                ProgressiveAttachment* self = this;
                (void)self;
            }
            return;
        }
    }
    done->Run();
}

void ProgressiveAttachment::MarkRPCAsDone(bool rpc_failed) {
    Buf saved;
    {
        std::lock_guard<std::mutex> g(_mu);
        _header_sent = !rpc_failed;
        _rpc_failed = rpc_failed;
        saved.swap(_saved);
    }
    if (!rpc_failed && !saved.empty()) write_chunk(&saved);
}

}  // namespace mrpc
