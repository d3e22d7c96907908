// In-order response writer for protocols without correlation ids on the
// server side (nshead, framed thrift): requests of one connection get a
// sequence number when parsed, handlers may finish in any order, and
// Deliver() writes every response whose predecessors were all delivered.
// This is what lets clients pipeline such calls on a single connection.
#pragma once

#include <cstdint>
#include <map>
#include <mutex>

#include "base/buf.h"
#include "fiber/sync.h"

namespace mrpc {

class Socket;

class OrderedResponseWriter {
public:
    uint64_t NextSeq() { return _next_assign++; }  // parse side (one reader per socket)
    // An empty packet (one-way request) just advances the sequence.
    void Deliver(uint64_t seq, Buf* packet, Socket* sock);

private:
    uint64_t _next_assign = 0;
    fiber::Mutex _mu;  // fiber-aware: held across Socket::Write
    uint64_t _next_send = 0;
    std::map<uint64_t, Buf> _ready;
};

}  // namespace mrpc
