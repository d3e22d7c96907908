// Glue between a naming service thread and a load balancer (role of
// src/brpc/details/load_balancer_with_naming.cpp and
// details/naming_service_thread.cpp:92-415): the NS fiber diffs server lists,
// creates/reuses sockets through SocketMap and adds/removes them in the LB.
#pragma once

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "cluster/load_balancer.h"
#include "cluster/naming_service.h"
#include "fiber/sync.h"

namespace mrpc {

class LoadBalancerWithNaming : public NamingServiceActions {
public:
    struct Options {
        std::string socket_signature;
        const NamingServiceFilter* ns_filter = nullptr;
        bool enable_circuit_breaker = false;
    };
    LoadBalancerWithNaming();
    ~LoadBalancerWithNaming() override;
    int Init(const char* ns_url, const char* lb_name, const Options& opt);
    void ResetServers(const std::vector<ServerNode>& servers) override;
    LoadBalancer* lb() const { return _lb.get(); }
    size_t ServerCount() const { return _lb ? _lb->ServerCount() : 0; }
    std::string Describe() const;
    std::vector<ServerNode> servers() const;

private:
    static void* RunNS(void* arg);
    std::unique_ptr<LoadBalancer> _lb;
    std::unique_ptr<NamingService> _ns;
    std::string _ns_url, _service_name, _lb_name;
    Options _opt;
    mutable std::mutex _mu;
    std::map<ServerNode, SocketId> _current;
    fiber::fiber_t _ns_tid = 0;
    fiber::CountdownEvent _first_batch{1};
    bool _first_done = false;
};

}  // namespace mrpc
