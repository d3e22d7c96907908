// Built-in load balancers (role of src/brpc/policy/*_load_balancer.cpp):
// rr, random, wrr, wr, la (locality-aware: weight ~ 1 / (latency * (1 +
// inflight)), reference docs/cn/lalb.md), c_murmurhash / c_md5 / c_ketama
// (consistent hashing on request_code). Server lists live in
// DoublyBufferedData so selection never blocks on membership changes.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <map>
#include <mutex>
#include <sstream>
#include <unordered_map>

#include "base/containers.h"
#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"
#include "cluster/circuit_breaker.h"
#include "cluster/cluster_recover_policy.h"
#include "cluster/load_balancer.h"
#include "rpc/controller.h"
#include "rpc/errno.h"

namespace mrpc {

size_t LoadBalancer::AddServersInBatch(const std::vector<ServerId>& servers) {
    size_t n = 0;
    for (auto& s : servers) n += AddServer(s) ? 1 : 0;
    return n;
}

size_t LoadBalancer::RemoveServersInBatch(const std::vector<ServerId>& servers) {
    size_t n = 0;
    for (auto& s : servers) n += RemoveServer(s) ? 1 : 0;
    return n;
}

bool IsServerAvailable(SocketId id, SocketUniquePtr* out) {
    if (Socket::Address(id, out) != 0) return false;
    if (IsIsolatedByCircuitBreaker(id)) {
        out->reset();
        return false;
    }
    return true;
}

namespace {

int weight_of(const std::string& tag) {
    int64_t w;
    if (!tag.empty() && parse_int64(tag, &w) && w > 0) return (int)w;
    return 1;
}

// ------------------------------------------------------------------ list based
struct ServerList {
    std::vector<ServerId> servers;
};

class ListLB : public LoadBalancer {
public:
    bool AddServer(const ServerId& s) override {
        return _db.Modify([&s](ServerList& l) -> size_t {
            for (auto& x : l.servers) {
                if (x.id == s.id) return 0;
            }
            l.servers.push_back(s);
            return 1;
        }) > 0;
    }
    bool RemoveServer(const ServerId& s) override {
        return _db.Modify([&s](ServerList& l) -> size_t {
            for (size_t i = 0; i < l.servers.size(); ++i) {
                if (l.servers[i].id == s.id) {
                    l.servers[i] = l.servers.back();
                    l.servers.pop_back();
                    return 1;
                }
            }
            return 0;
        }) > 0;
    }
    size_t ServerCount() const override {
        DoublyBufferedData<ServerList>::ScopedPtr p;
        const_cast<DoublyBufferedData<ServerList>&>(_db).Read(&p);
        return p->servers.size();
    }

protected:
    // pick among servers starting at `start`, stepping by 1
    int pick_from(const ServerList& l, size_t start, const SelectIn& in, SelectOut* out) {
        const size_t n = l.servers.size();
        if (n == 0) return EHOSTDOWN;
        if (_recover && _recover->StopRecoverIfNecessary() && _recover->DoReject(l.servers)) return EREJECT;
        for (size_t i = 0; i < n; ++i) {
            const ServerId& s = l.servers[(start + i) % n];
            if (in.excluded && in.excluded->IsExcluded(s.id)) continue;
            if (IsServerAvailable(s.id, out->ptr)) return 0;
        }
        // all excluded or down: try excluded ones too (better than failing)
        for (size_t i = 0; i < n; ++i) {
            const ServerId& s = l.servers[(start + i) % n];
            if (IsServerAvailable(s.id, out->ptr)) return 0;
        }
        if (_recover) _recover->StartRecover();
        return EHOSTDOWN;
    }
    // "min_working_instances=N hold_seconds=S" enables cluster recovery throttling.
    template <typename T>
    static LoadBalancer* NewWithRecover(const std::string& params) {
        T* lb = new T;
        if (!GetRecoverPolicyByParams(params, &lb->_recover)) {
            delete lb;
            return nullptr;
        }
        return lb;
    }
    DoublyBufferedData<ServerList> _db;
    std::shared_ptr<ClusterRecoverPolicy> _recover;
};

class RoundRobinLB : public ListLB {
public:
    int SelectServer(const SelectIn& in, SelectOut* out) override {
        DoublyBufferedData<ServerList>::ScopedPtr p;
        _db.Read(&p);
        static thread_local uint64_t offset = fast_rand();
        return pick_from(*p, (size_t)(offset++), in, out);
    }
    LoadBalancer* New(const std::string& params) const override { return NewWithRecover<RoundRobinLB>(params); }
    void Describe(std::ostream& os) const override { os << "rr"; }
};

class RandomLB : public ListLB {
public:
    int SelectServer(const SelectIn& in, SelectOut* out) override {
        DoublyBufferedData<ServerList>::ScopedPtr p;
        _db.Read(&p);
        return pick_from(*p, (size_t)fast_rand(), in, out);
    }
    LoadBalancer* New(const std::string& params) const override { return NewWithRecover<RandomLB>(params); }
    void Describe(std::ostream& os) const override { os << "random"; }
};

// ------------------------------------------------------------------ weighted
struct WeightedList {
    std::vector<ServerId> servers;
    std::vector<uint32_t> schedule;   // wrr: server index per slot (weights / gcd)
    std::vector<uint64_t> prefix;     // wr: prefix sums of weights
};

class WeightedLBBase : public LoadBalancer {
public:
    bool AddServer(const ServerId& s) override {
        return _db.Modify([&s](WeightedList& l) -> size_t {
            for (auto& x : l.servers) {
                if (x.id == s.id) return 0;
            }
            l.servers.push_back(s);
            rebuild(l);
            return 1;
        }) > 0;
    }
    bool RemoveServer(const ServerId& s) override {
        return _db.Modify([&s](WeightedList& l) -> size_t {
            for (size_t i = 0; i < l.servers.size(); ++i) {
                if (l.servers[i].id == s.id) {
                    l.servers.erase(l.servers.begin() + i);
                    rebuild(l);
                    return 1;
                }
            }
            return 0;
        }) > 0;
    }
    size_t ServerCount() const override {
        DoublyBufferedData<WeightedList>::ScopedPtr p;
        const_cast<DoublyBufferedData<WeightedList>&>(_db).Read(&p);
        return p->servers.size();
    }

protected:
    static void rebuild(WeightedList& l) {
        l.prefix.clear();
        l.schedule.clear();
        uint64_t sum = 0;
        uint64_t g = 0;
        for (auto& s : l.servers) {
            const int w = weight_of(s.tag);
            sum += w;
            l.prefix.push_back(sum);
            g = g == 0 ? (uint64_t)w : std::__gcd(g, (uint64_t)w);
        }
        if (g == 0) return;
        // Interleaved (smooth) schedule: repeatedly pick the server with the
        // largest current weight (nginx smooth WRR), capped in length.
        std::vector<int64_t> cur(l.servers.size(), 0);
        const uint64_t slots = std::min<uint64_t>(sum / g, 65536);
        for (uint64_t k = 0; k < slots; ++k) {
            size_t best = 0;
            for (size_t i = 0; i < l.servers.size(); ++i) {
                cur[i] += weight_of(l.servers[i].tag) / (int64_t)g;
                if (cur[i] > cur[best]) best = i;
            }
            cur[best] -= (int64_t)(sum / g);
            l.schedule.push_back((uint32_t)best);
        }
    }
    int pick_index_order(const WeightedList& l, size_t first, const SelectIn& in, SelectOut* out) {
        const size_t n = l.servers.size();
        if (n == 0) return EHOSTDOWN;
        for (size_t i = 0; i < n; ++i) {
            const ServerId& s = l.servers[(first + i) % n];
            if (in.excluded && in.excluded->IsExcluded(s.id) && i + 1 < n) continue;
            if (IsServerAvailable(s.id, out->ptr)) return 0;
        }
        return EHOSTDOWN;
    }
    DoublyBufferedData<WeightedList> _db;
};

class WeightedRoundRobinLB : public WeightedLBBase {
public:
    int SelectServer(const SelectIn& in, SelectOut* out) override {
        DoublyBufferedData<WeightedList>::ScopedPtr p;
        _db.Read(&p);
        if (p->schedule.empty()) return EHOSTDOWN;
        static thread_local uint64_t pos = fast_rand();
        const size_t first = p->schedule[(pos++) % p->schedule.size()];
        return pick_index_order(*p, first, in, out);
    }
    LoadBalancer* New(const std::string&) const override { return new WeightedRoundRobinLB; }
    void Describe(std::ostream& os) const override { os << "wrr"; }
};

class WeightedRandomLB : public WeightedLBBase {
public:
    int SelectServer(const SelectIn& in, SelectOut* out) override {
        DoublyBufferedData<WeightedList>::ScopedPtr p;
        _db.Read(&p);
        if (p->prefix.empty()) return EHOSTDOWN;
        const uint64_t r = fast_rand_less_than(p->prefix.back());
        const size_t first = std::upper_bound(p->prefix.begin(), p->prefix.end(), r) - p->prefix.begin();
        return pick_index_order(*p, first, in, out);
    }
    LoadBalancer* New(const std::string&) const override { return new WeightedRandomLB; }
    void Describe(std::ostream& os) const override { os << "wr"; }
};

// ------------------------------------------------------------------ locality aware
struct LAStat {
    std::atomic<int64_t> ema_latency_us{0};
    std::atomic<int64_t> inflight{0};
    std::atomic<int64_t> errors{0};
};

struct LAList {
    std::vector<ServerId> servers;
    std::vector<std::shared_ptr<LAStat>> stats;
};

class LocalityAwareLB : public LoadBalancer {
public:
    bool AddServer(const ServerId& s) override {
        auto st = get_stat(s.id);
        return _db.Modify([&](LAList& l) -> size_t {
            for (auto& x : l.servers) {
                if (x.id == s.id) return 0;
            }
            l.servers.push_back(s);
            l.stats.push_back(st);
            return 1;
        }) > 0;
    }
    bool RemoveServer(const ServerId& s) override {
        const bool r = _db.Modify([&s](LAList& l) -> size_t {
            for (size_t i = 0; i < l.servers.size(); ++i) {
                if (l.servers[i].id == s.id) {
                    l.servers.erase(l.servers.begin() + i);
                    l.stats.erase(l.stats.begin() + i);
                    return 1;
                }
            }
            return 0;
        }) > 0;
        return r;
    }
    size_t ServerCount() const override {
        DoublyBufferedData<LAList>::ScopedPtr p;
        const_cast<DoublyBufferedData<LAList>&>(_db).Read(&p);
        return p->servers.size();
    }
    int SelectServer(const SelectIn& in, SelectOut* out) override {
        DoublyBufferedData<LAList>::ScopedPtr p;
        _db.Read(&p);
        const size_t n = p->servers.size();
        if (n == 0) return EHOSTDOWN;
        // weight = 1e9 / (latency * (inflight + 1)); servers without samples
        // get the average weight so that they are explored.
        double total = 0;
        std::vector<double> w(n);
        int64_t known = 0, sum_lat = 0;
        for (size_t i = 0; i < n; ++i) {
            const int64_t l = p->stats[i]->ema_latency_us.load(std::memory_order_relaxed);
            if (l > 0) {
                sum_lat += l;
                ++known;
            }
        }
        const int64_t avg = known ? sum_lat / known : 1000;
        for (size_t i = 0; i < n; ++i) {
            if (in.excluded && in.excluded->IsExcluded(p->servers[i].id)) {
                w[i] = 0;
                continue;
            }
            int64_t l = p->stats[i]->ema_latency_us.load(std::memory_order_relaxed);
            if (l <= 0) l = avg;
            const int64_t inflight = p->stats[i]->inflight.load(std::memory_order_relaxed);
            w[i] = 1e9 / ((double)std::max<int64_t>(l, 1) * (double)(inflight + 1));
            total += w[i];
        }
        for (int attempt = 0; attempt < (int)n + 1; ++attempt) {
            size_t idx;
            if (total > 0) {
                double r = fast_rand_double() * total;
                idx = 0;
                while (idx + 1 < n && r >= w[idx]) {
                    r -= w[idx];
                    ++idx;
                }
            } else {
                idx = fast_rand_less_than(n);
            }
            if (IsServerAvailable(p->servers[idx].id, out->ptr)) {
                p->stats[idx]->inflight.fetch_add(1, std::memory_order_relaxed);
                out->need_feedback = true;
                return 0;
            }
            total -= w[idx];
            w[idx] = 0;
        }
        return EHOSTDOWN;
    }
    void Feedback(const CallInfo& info) override {
        auto st = find_stat(info.server_id);
        if (!st) return;
        st->inflight.fetch_sub(1, std::memory_order_relaxed);
        int64_t lat = monotonic_us() - info.begin_time_us;
        if (info.error_code) {
            // punish errors: count them as slow calls
            st->errors.fetch_add(1, std::memory_order_relaxed);
            lat = std::max<int64_t>(lat, 2 * std::max<int64_t>(st->ema_latency_us.load(), 1000));
        }
        int64_t old = st->ema_latency_us.load(std::memory_order_relaxed);
        st->ema_latency_us.store(old == 0 ? lat : (old * 7 + lat) / 8, std::memory_order_relaxed);
    }
    LoadBalancer* New(const std::string&) const override { return new LocalityAwareLB; }
    void Describe(std::ostream& os) const override { os << "la"; }

private:
    std::shared_ptr<LAStat> get_stat(SocketId id) {
        std::lock_guard<std::mutex> g(_mu);
        auto& s = _stats[id];
        if (!s) s = std::make_shared<LAStat>();
        return s;
    }
    std::shared_ptr<LAStat> find_stat(SocketId id) {
        std::lock_guard<std::mutex> g(_mu);
        auto it = _stats.find(id);
        return it == _stats.end() ? nullptr : it->second;
    }
    DoublyBufferedData<LAList> _db;
    std::mutex _mu;
    std::unordered_map<SocketId, std::shared_ptr<LAStat>> _stats;
};

// ------------------------------------------------------------------ consistent hashing
enum HashKind { HASH_MURMUR, HASH_MD5, HASH_KETAMA };

struct Ring {
    std::vector<std::pair<uint32_t, ServerId>> nodes;  // sorted by hash
    std::vector<ServerId> servers;
};

class ConsistentHashLB : public LoadBalancer {
public:
    ConsistentHashLB(HashKind k, int replicas) : _kind(k), _replicas(replicas) {}
    bool AddServer(const ServerId& s) override {
        return _db.Modify([&](Ring& r) -> size_t {
            for (auto& x : r.servers) {
                if (x.id == s.id) return 0;
            }
            r.servers.push_back(s);
            rebuild(r);
            return 1;
        }) > 0;
    }
    bool RemoveServer(const ServerId& s) override {
        return _db.Modify([&](Ring& r) -> size_t {
            for (size_t i = 0; i < r.servers.size(); ++i) {
                if (r.servers[i].id == s.id) {
                    r.servers.erase(r.servers.begin() + i);
                    rebuild(r);
                    return 1;
                }
            }
            return 0;
        }) > 0;
    }
    size_t ServerCount() const override {
        DoublyBufferedData<Ring>::ScopedPtr p;
        const_cast<DoublyBufferedData<Ring>&>(_db).Read(&p);
        return p->servers.size();
    }
    int SelectServer(const SelectIn& in, SelectOut* out) override {
        if (!in.has_request_code) {
            LOG_EVERY_SECOND(ERROR) << "consistent hashing LB requires Controller::set_request_code()";
            return EINVAL;
        }
        DoublyBufferedData<Ring>::ScopedPtr p;
        _db.Read(&p);
        if (p->nodes.empty()) return EHOSTDOWN;
        const uint32_t h = (uint32_t)in.request_code;
        auto it = std::lower_bound(p->nodes.begin(), p->nodes.end(), std::make_pair(h, ServerId()),
                                   [](const std::pair<uint32_t, ServerId>& a, const std::pair<uint32_t, ServerId>& b) {
                                       return a.first < b.first;
                                   });
        for (size_t i = 0; i < p->nodes.size(); ++i) {
            if (it == p->nodes.end()) it = p->nodes.begin();
            if (!(in.excluded && in.excluded->IsExcluded(it->second.id)) && IsServerAvailable(it->second.id, out->ptr)) {
                return 0;
            }
            ++it;
        }
        return EHOSTDOWN;
    }
    LoadBalancer* New(const std::string& params) const override {
        int rep = _replicas;
        for (const std::string& kv : split_string(params, ' ')) {
            if (starts_with(kv, "replicas=")) rep = atoi(kv.c_str() + 9);
        }
        return new ConsistentHashLB(_kind, rep > 0 ? rep : _replicas);
    }
    void Describe(std::ostream& os) const override {
        os << (_kind == HASH_MURMUR ? "c_murmurhash" : _kind == HASH_MD5 ? "c_md5" : "c_ketama");
    }

private:
    void rebuild(Ring& r) {
        r.nodes.clear();
        for (auto& s : r.servers) {
            SocketUniquePtr sock;
            std::string addr;
            if (Socket::AddressFailedAsWell(s.id, &sock) >= 0) addr = sock->remote_side().to_string();
            else addr = std::to_string(s.id);
            if (_kind == HASH_KETAMA) {
                for (int i = 0; i < _replicas / 4 + 1; ++i) {
                    unsigned char d[16];
                    std::string key = addr + "-" + std::to_string(i);
                    md5(key.data(), key.size(), d);
                    for (int k = 0; k < 4; ++k) {
                        uint32_t h = ((uint32_t)d[3 + 4 * k] << 24) | ((uint32_t)d[2 + 4 * k] << 16) |
                                     ((uint32_t)d[1 + 4 * k] << 8) | d[4 * k];
                        r.nodes.emplace_back(h, s);
                    }
                }
            } else {
                for (int i = 0; i < _replicas; ++i) {
                    std::string key = addr + "-" + std::to_string(i);
                    uint32_t h = _kind == HASH_MURMUR ? murmurhash3_32(key.data(), key.size(), 0)
                                                       : md5_hash32(key.data(), key.size());
                    r.nodes.emplace_back(h, s);
                }
            }
        }
        std::sort(r.nodes.begin(), r.nodes.end(),
                  [](const std::pair<uint32_t, ServerId>& a, const std::pair<uint32_t, ServerId>& b) {
                      return a.first < b.first;
                  });
    }
    HashKind _kind;
    int _replicas;
    DoublyBufferedData<Ring> _db;
};

struct LBRegistry {
    std::mutex mu;
    std::map<std::string, const LoadBalancer*> m;
};
LBRegistry& lbs() {
    static LBRegistry* r = new LBRegistry;
    return *r;
}
}  // namespace

void RegisterLoadBalancer(const std::string& name, const LoadBalancer* prototype) {
    std::lock_guard<std::mutex> g(lbs().mu);
    lbs().m[name] = prototype;
}

void RegisterBuiltinLoadBalancers() {
    static std::once_flag once;
    std::call_once(once, [] {
        RegisterLoadBalancer("rr", new RoundRobinLB);
        RegisterLoadBalancer("random", new RandomLB);
        RegisterLoadBalancer("wrr", new WeightedRoundRobinLB);
        RegisterLoadBalancer("wr", new WeightedRandomLB);
        RegisterLoadBalancer("la", new LocalityAwareLB);
        RegisterLoadBalancer("c_murmurhash", new ConsistentHashLB(HASH_MURMUR, 100));
        RegisterLoadBalancer("c_md5", new ConsistentHashLB(HASH_MD5, 100));
        RegisterLoadBalancer("c_ketama", new ConsistentHashLB(HASH_KETAMA, 160));
    });
}

LoadBalancer* CreateLoadBalancer(const std::string& spec) {
    RegisterBuiltinLoadBalancers();
    std::string name = spec, params;
    size_t colon = spec.find(':');
    if (colon != std::string::npos) {
        name = spec.substr(0, colon);
        params = spec.substr(colon + 1);
    }
    std::lock_guard<std::mutex> g(lbs().mu);
    auto it = lbs().m.find(name);
    if (it == lbs().m.end()) return nullptr;
    return it->second->New(params);
}

std::vector<std::string> ListLoadBalancers() {
    RegisterBuiltinLoadBalancers();
    std::lock_guard<std::mutex> g(lbs().mu);
    std::vector<std::string> out;
    for (auto& kv : lbs().m) out.push_back(kv.first);
    return out;
}

}  // namespace mrpc
