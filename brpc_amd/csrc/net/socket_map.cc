#include "net/socket_map.h"

#include <map>
#include <mutex>

#include "base/flags.h"
#include "base/logging.h"
#include "net/input_messenger.h"

DEFINE_int32(health_check_interval, 3, "seconds between health checks of failed client connections (<=0 disables)");
DEFINE_int32(idle_timeout_second, 30, "client connections without users for this long are closed");

namespace mrpc {

namespace {
struct Entry {
    SocketId id;
    int ref;
};
struct Map {
    std::mutex mu;
    std::map<SocketMapKey, Entry> m;
};
Map& socket_map() {
    static Map* m = new Map;
    return *m;
}
}  // namespace

int SocketMapInsert(const SocketMapKey& key, SocketId* id) {
    Map& sm = socket_map();
    std::lock_guard<std::mutex> g(sm.mu);
    auto it = sm.m.find(key);
    if (it != sm.m.end()) {
        SocketUniquePtr p;
        if (Socket::AddressFailedAsWell(it->second.id, &p) >= 0) {
            ++it->second.ref;
            *id = it->second.id;
            return 0;
        }
        sm.m.erase(it);  // recycled: create a new one
    }
    SocketOptions opt;
    opt.remote_side = key.peer;
    opt.connect_lazily = true;
    opt.health_check_interval_s = FLAGS_health_check_interval;
    const size_t ssl_at = key.signature.find("|ssl:");
    if (ssl_at != std::string::npos) {
        const size_t b = ssl_at + 5;
        const size_t e = key.signature.find('|', b);
        opt.ssl_sni = key.signature.substr(b, e == std::string::npos ? std::string::npos : e - b);
        opt.ssl_ctx = SslContext::DefaultClient();
        if (!opt.ssl_ctx) return -1;
    }
    if (key.signature.find("|rdma") != std::string::npos) opt.rdma = SocketOptions::RDMA_CLIENT;
    SocketId sid;
    if (get_client_side_messenger()->Create(opt, &sid) != 0) return -1;
    sm.m[key] = Entry{sid, 1};
    *id = sid;
    return 0;
}

void SocketMapRemove(const SocketMapKey& key) {
    Map& sm = socket_map();
    SocketId to_release = INVALID_SOCKET_ID;
    {
        std::lock_guard<std::mutex> g(sm.mu);
        auto it = sm.m.find(key);
        if (it == sm.m.end()) return;
        if (--it->second.ref > 0) return;
        to_release = it->second.id;
        sm.m.erase(it);
    }
    SocketUniquePtr p;
    if (Socket::AddressFailedAsWell(to_release, &p) >= 0) p->ReleaseAdditionalReference();
}

int SocketMapFind(const SocketMapKey& key, SocketId* id) {
    Map& sm = socket_map();
    std::lock_guard<std::mutex> g(sm.mu);
    auto it = sm.m.find(key);
    if (it == sm.m.end()) return -1;
    *id = it->second.id;
    return 0;
}

size_t SocketMapSize() {
    Map& sm = socket_map();
    std::lock_guard<std::mutex> g(sm.mu);
    return sm.m.size();
}

}  // namespace mrpc
