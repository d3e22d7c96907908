// SocketMap: shares one client connection per (endpoint, signature) across
// Channels (role of src/brpc/socket_map.cpp:89-213). Sockets are created
// lazily-connecting, health-checked, and released when the last user leaves.
#pragma once

#include <string>

#include "base/endpoint.h"
#include "net/socket.h"

namespace mrpc {

struct SocketMapKey {
    EndPoint peer;
    std::string signature;  // e.g. protocol/ssl/auth specific tag
    bool operator<(const SocketMapKey& o) const {
        if (peer != o.peer) return peer < o.peer;
        return signature < o.signature;
    }
};

// Returns 0 and the shared SocketId (creating it if needed); increments the
// reference count of the entry.
int SocketMapInsert(const SocketMapKey& key, SocketId* id);
// Decrements; releases the socket when the count drops to zero.
void SocketMapRemove(const SocketMapKey& key);
int SocketMapFind(const SocketMapKey& key, SocketId* id);
size_t SocketMapSize();

}  // namespace mrpc
