#include "cluster/lb_with_naming.h"

#include <algorithm>
#include <set>
#include <sstream>

#include "base/logging.h"
#include "base/time.h"
#include "net/socket_map.h"

namespace mrpc {

LoadBalancerWithNaming::LoadBalancerWithNaming() {}

LoadBalancerWithNaming::~LoadBalancerWithNaming() {
    if (_ns_tid) {
        fiber::stop(_ns_tid);
        fiber::join(_ns_tid);
    }
    std::map<ServerNode, SocketId> cur;
    {
        std::lock_guard<std::mutex> g(_mu);
        cur.swap(_current);
    }
    for (auto& kv : cur) {
        if (_lb) _lb->RemoveServer(ServerId(kv.second, kv.first.tag));
        SocketMapRemove(SocketMapKey{kv.first.addr, _opt.socket_signature});
    }
}

int LoadBalancerWithNaming::Init(const char* ns_url, const char* lb_name, const Options& opt) {
    _opt = opt;
    _ns_url = ns_url;
    _lb_name = lb_name;
    std::string url = ns_url;
    size_t p = url.find("://");
    if (p == std::string::npos) {
        LOG(ERROR) << "Invalid naming service url `" << url << "'";
        return -1;
    }
    const std::string scheme = url.substr(0, p);
    _service_name = url.substr(p + 3);
    _ns.reset(CreateNamingService(scheme));
    if (!_ns) {
        LOG(ERROR) << "Unknown naming service scheme `" << scheme << "'";
        return -1;
    }
    _lb.reset(CreateLoadBalancer(lb_name));
    if (!_lb) {
        LOG(ERROR) << "Unknown load balancer `" << lb_name << "'";
        return -1;
    }
    if (_ns->RunNamingServiceReturnsQuickly()) {
        _ns->RunNamingService(_service_name.c_str(), this);
        return 0;
    }
    if (fiber::start_background(&_ns_tid, &fiber::ATTR_NORMAL, RunNS, this) != 0) return -1;
    // Wait (bounded) for the first batch of servers like the reference does.
    timespec ts = realtime_after_us(5000000);
    _first_batch.timed_wait(&ts);
    return 0;
}

void* LoadBalancerWithNaming::RunNS(void* arg) {
    LoadBalancerWithNaming* self = static_cast<LoadBalancerWithNaming*>(arg);
    self->_ns->RunNamingService(self->_service_name.c_str(), self);
    return nullptr;
}

void LoadBalancerWithNaming::ResetServers(const std::vector<ServerNode>& servers0) {
    std::vector<ServerNode> servers;
    std::set<ServerNode> seen;
    for (const ServerNode& s : servers0) {
        if (_opt.ns_filter && !_opt.ns_filter->Accept(s)) continue;
        if (seen.insert(s).second) servers.push_back(s);
    }
    std::vector<ServerId> to_add, to_remove;
    std::vector<ServerNode> removed_nodes;
    {
        std::lock_guard<std::mutex> g(_mu);
        std::map<ServerNode, SocketId> next;
        for (const ServerNode& s : servers) {
            auto it = _current.find(s);
            if (it != _current.end()) {
                next[s] = it->second;
                continue;
            }
            SocketId sid;
            if (SocketMapInsert(SocketMapKey{s.addr, _opt.socket_signature}, &sid) != 0) {
                LOG(ERROR) << "Fail to create socket for " << s.addr;
                continue;
            }
            next[s] = sid;
            to_add.emplace_back(sid, s.tag);
        }
        for (auto& kv : _current) {
            if (!next.count(kv.first)) {
                to_remove.emplace_back(kv.second, kv.first.tag);
                removed_nodes.push_back(kv.first);
            }
        }
        _current.swap(next);
    }
    if (!to_add.empty()) _lb->AddServersInBatch(to_add);
    if (!to_remove.empty()) _lb->RemoveServersInBatch(to_remove);
    for (const ServerNode& n : removed_nodes) SocketMapRemove(SocketMapKey{n.addr, _opt.socket_signature});
    if (!_first_done) {
        _first_done = true;
        _first_batch.signal();
    }
}

std::vector<ServerNode> LoadBalancerWithNaming::servers() const {
    std::lock_guard<std::mutex> g(_mu);
    std::vector<ServerNode> out;
    for (auto& kv : _current) out.push_back(kv.first);
    return out;
}

std::string LoadBalancerWithNaming::Describe() const {
    std::ostringstream os;
    os << _lb_name << " over " << _ns_url << " (" << ServerCount() << " servers)";
    return os.str();
}

}  // namespace mrpc
