// Cluster recovery throttling (role of the reference's
// src/brpc/cluster_recover_policy.h/.cpp): when every server of a cluster
// went down and servers come back one by one, the first revived server
// would otherwise receive the traffic of the whole cluster. While
// "recovering", a request is accepted with probability usable/min_working
// and rejected (EREJECT) otherwise; recovery ends once the usable count has
// been stable for hold_seconds.
#pragma once

#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "cluster/load_balancer.h"

namespace mrpc {

class ClusterRecoverPolicy {
public:
    virtual ~ClusterRecoverPolicy() {}
    // Every server is unavailable: start recovering.
    virtual void StartRecover() = 0;
    // True if this request should be rejected to protect revived servers.
    virtual bool DoReject(const std::vector<ServerId>& servers) = 0;
    // Leaves the recovering state when its condition holds; returns true
    // while still recovering.
    virtual bool StopRecoverIfNecessary() = 0;
};

class DefaultClusterRecoverPolicy : public ClusterRecoverPolicy {
public:
    DefaultClusterRecoverPolicy(int64_t min_working_instances, int64_t hold_seconds);
    void StartRecover() override;
    bool DoReject(const std::vector<ServerId>& servers) override;
    bool StopRecoverIfNecessary() override;
    bool recovering() const { return _recovering; }

private:
    uint64_t UsableCount(int64_t now_ms, const std::vector<ServerId>& servers);
    bool _recovering = false;
    const int64_t _min_working;
    const int64_t _hold_seconds;
    std::mutex _mu;
    uint64_t _last_usable = 0;
    int64_t _last_usable_change_ms = 0;
    uint64_t _usable_cache = 0;
    int64_t _usable_cache_ms = 0;
};

// "min_working_instances=N hold_seconds=S" (both needed) -> policy; an
// empty string gives no policy. False on malformed parameters.
bool GetRecoverPolicyByParams(const std::string& params, std::shared_ptr<ClusterRecoverPolicy>* out);

}  // namespace mrpc
