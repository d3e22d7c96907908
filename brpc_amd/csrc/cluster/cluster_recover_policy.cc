#include "cluster/cluster_recover_policy.h"

#include <cstdlib>

#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"

namespace mrpc {

DefaultClusterRecoverPolicy::DefaultClusterRecoverPolicy(int64_t min_working_instances, int64_t hold_seconds)
    : _min_working(min_working_instances), _hold_seconds(hold_seconds) {}

void DefaultClusterRecoverPolicy::StartRecover() {
    std::lock_guard<std::mutex> g(_mu);
    _recovering = true;
}

uint64_t DefaultClusterRecoverPolicy::UsableCount(int64_t now_ms, const std::vector<ServerId>& servers) {
    // Probing every socket per request is too costly: cache for 100 ms.
    if (now_ms - _usable_cache_ms <= 100) return _usable_cache;
    uint64_t usable = 0;
    for (const ServerId& s : servers) {
        SocketUniquePtr p;
        if (IsServerAvailable(s.id, &p)) ++usable;
    }
    std::lock_guard<std::mutex> g(_mu);
    _usable_cache = usable;
    _usable_cache_ms = now_ms;
    return usable;
}

bool DefaultClusterRecoverPolicy::StopRecoverIfNecessary() {
    if (!_recovering) return false;
    const int64_t now_ms = monotonic_us() / 1000;
    std::lock_guard<std::mutex> g(_mu);
    if (_last_usable_change_ms != 0 && now_ms - _last_usable_change_ms > _hold_seconds * 1000) {
        _recovering = false;
        _last_usable = 0;
        _last_usable_change_ms = 0;
        return false;
    }
    return true;
}

bool DefaultClusterRecoverPolicy::DoReject(const std::vector<ServerId>& servers) {
    if (!_recovering) return false;
    const int64_t now_ms = monotonic_us() / 1000;
    const uint64_t usable = UsableCount(now_ms, servers);
    {
        std::lock_guard<std::mutex> g(_mu);
        if (usable != _last_usable) {
            _last_usable = usable;
            _last_usable_change_ms = now_ms;
        }
    }
    if (_min_working <= 0) return false;
    // accept with probability usable / min_working
    return (int64_t)(fast_rand() % (uint64_t)_min_working) >= (int64_t)usable;
}

bool GetRecoverPolicyByParams(const std::string& params, std::shared_ptr<ClusterRecoverPolicy>* out) {
    out->reset();
    int64_t min_working = -1, hold = -1;
    bool any = false;
    for (const std::string& kv : split_string(params, ' ')) {
        if (kv.empty()) continue;
        const size_t eq = kv.find('=');
        if (eq == std::string::npos) return false;
        const std::string k = kv.substr(0, eq);
        char* end = nullptr;
        const long long v = strtoll(kv.c_str() + eq + 1, &end, 10);
        if (*end != '\0' || v < 0) return false;
        if (k == "min_working_instances") {
            min_working = v;
            any = true;
        } else if (k == "hold_seconds") {
            hold = v;
            any = true;
        }
        // other keys belong to the load balancer itself
    }
    if (!any) return true;
    if (min_working <= 0 || hold < 0) {
        LOG(ERROR) << "cluster recover policy needs min_working_instances>0 and hold_seconds>=0: " << params;
        return false;
    }
    out->reset(new DefaultClusterRecoverPolicy(min_working, hold));
    return true;
}

}  // namespace mrpc
