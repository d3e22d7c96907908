// Load balancing interfaces (role of src/brpc/load_balancer.h,
// excluded_servers.h, server_id.h). Implementations live in
// cluster/load_balancers.cc: rr, wrr, random, wr, la (locality-aware),
// c_murmurhash / c_md5 / c_ketama (consistent hashing), _dynpart.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <ostream>
#include <string>
#include <vector>

#include "net/socket.h"

namespace mrpc {

class Controller;

struct ServerId {
    SocketId id = INVALID_SOCKET_ID;
    std::string tag;
    ServerId() {}
    explicit ServerId(SocketId i) : id(i) {}
    ServerId(SocketId i, const std::string& t) : id(i), tag(t) {}
    bool operator==(const ServerId& o) const { return id == o.id && tag == o.tag; }
    bool operator<(const ServerId& o) const { return id != o.id ? id < o.id : tag < o.tag; }
};

// Servers tried by previous attempts of one RPC (retries avoid them).
class ExcludedServers {
public:
    explicit ExcludedServers(int cap = 4) : _cap(cap) {}
    void Add(SocketId id) {
        if (IsExcluded(id)) return;
        if ((int)_ids.size() >= _cap) _ids.erase(_ids.begin());
        _ids.push_back(id);
    }
    bool IsExcluded(SocketId id) const {
        for (SocketId x : _ids) {
            if (x == id) return true;
        }
        return false;
    }
    size_t size() const { return _ids.size(); }
private:
    int _cap;
    std::vector<SocketId> _ids;
};

class LoadBalancer {
public:
    struct SelectIn {
        int64_t begin_time_us = 0;
        bool changable_weights = true;
        bool has_request_code = false;
        uint64_t request_code = 0;
        const ExcludedServers* excluded = nullptr;
    };
    struct SelectOut {
        SocketUniquePtr* ptr = nullptr;
        bool need_feedback = false;
    };
    struct CallInfo {
        int64_t begin_time_us = 0;
        SocketId server_id = INVALID_SOCKET_ID;
        int error_code = 0;
        const Controller* controller = nullptr;
    };
    virtual ~LoadBalancer() {}
    virtual bool AddServer(const ServerId& server) = 0;
    virtual bool RemoveServer(const ServerId& server) = 0;
    virtual size_t AddServersInBatch(const std::vector<ServerId>& servers);
    virtual size_t RemoveServersInBatch(const std::vector<ServerId>& servers);
    // 0 and a referenced socket in *out->ptr; EHOSTDOWN if no server.
    virtual int SelectServer(const SelectIn& in, SelectOut* out) = 0;
    virtual void Feedback(const CallInfo&) {}
    virtual LoadBalancer* New(const std::string& params) const = 0;
    virtual void Describe(std::ostream& os) const { os << "LoadBalancer"; }
    virtual size_t ServerCount() const = 0;
};

// Registry of LB prototypes by name ("rr", "la", ...)
void RegisterLoadBalancer(const std::string& name, const LoadBalancer* prototype);
// "rr" or "c_murmurhash:replicas=100" -> new instance
LoadBalancer* CreateLoadBalancer(const std::string& lb_name_with_params);
void RegisterBuiltinLoadBalancers();
std::vector<std::string> ListLoadBalancers();

// Returns true if the socket is usable by the LB (alive and not
// isolated by its circuit breaker).
bool IsServerAvailable(SocketId id, SocketUniquePtr* out);

}  // namespace mrpc
