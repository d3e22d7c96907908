// InputMessenger: per-socket read loop, message cutting by protocol
// sniffing, dispatch of every message but the last into its own fiber (role
// of src/brpc/input_messenger.cpp:60-398). Adaptive read size:
// clamp(avg_msg_size * 16, 4KB, 512KB).
#pragma once

#include <string>
#include <vector>

#include "rpc/protocol.h"

namespace mrpc {

struct InputMessageHandler {
    ParseResult (*parse)(Buf* source, Socket* socket, bool read_eof, const void* arg) = nullptr;
    void (*process)(InputMessageBase* msg) = nullptr;
    bool (*verify)(const InputMessageBase* msg) = nullptr;
    const void* arg = nullptr;
    const char* name = nullptr;
};

class InputMessenger {
public:
    explicit InputMessenger(size_t capacity = 128);
    ~InputMessenger();
    int AddHandler(const InputMessageHandler& h);
    int AddNonProtocolHandler(const InputMessageHandler& h);
    // Socket callback (on_edge_triggered_events).
    static void OnNewMessages(Socket* m);
    // Create a socket whose reads are handled by this messenger.
    int Create(const SocketOptions& options, SocketId* id);
    size_t handler_count() const { return _handlers.size(); }
    const InputMessageHandler& handler(size_t i) const { return _handlers[i]; }

private:
    ParseResult CutInputMessage(Socket* m, size_t* index, bool read_eof);
    std::vector<InputMessageHandler> _handlers;
    size_t _capacity;
};

// Messenger handling responses for all client sockets.
InputMessenger* get_client_side_messenger();
// Read up to this many bytes per read() call at most.
void QueueOrProcessMessage(InputMessageBase* msg, bool in_place);

}  // namespace mrpc
