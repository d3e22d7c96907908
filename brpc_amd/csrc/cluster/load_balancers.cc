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
// Locality-aware LB (reference src/brpc/policy/locality_aware_load_balancer.h
// :41-216, docs/cn/lalb.md): a server's weight is proportional to its
// throughput capacity, kLAWeightScale / avg_latency, and is punished while
// its in-flight calls are older than its average latency (weight *=
// avg_latency / inflight_delay), so a server that suddenly stalls sheds
// traffic before its calls even complete.
//
// Selection is O(log n) and lock-free: the weights sit in a Fenwick tree
// (an implicit complete binary tree of prefix sums) of atomics inside the
// DoublyBufferedData copy; a select draws r in [0, total) and descends the
// tree with atomic loads. Feedback and selection re-weight one server and
// push the difference up its Fenwick path with fetch_add. Each tree copy
// keeps its own leaf values, so a copy rebuilt concurrently with an update
// converges at that server's next update instead of drifting. The only lock
// is a per-server mutex around that server's latency statistics.
const int64_t kLAWeightScale = (int64_t)1 << 40;
const int64_t kLAMinWeight = 1000;  // never starve a server completely

struct LAServerStats {
    std::mutex mu;
    int64_t avg_latency_us = 0;  // EMA; 0 = no sample yet
    int64_t inflight = 0;
    int64_t inflight_begin_sum_us = 0;
    int64_t samples = 0;
    std::atomic<int64_t> weight{0};  // last computed weight
    std::atomic<int64_t> errors{0};

    // Weight from the statistics (caller holds mu).
    int64_t compute_locked(int64_t now_us, int64_t default_latency) const {
        const int64_t lat = std::max<int64_t>(avg_latency_us > 0 ? avg_latency_us : default_latency, 1);
        int64_t w = kLAWeightScale / lat;
        if (inflight > 0) {
            const int64_t delay = now_us - inflight_begin_sum_us / inflight;
            if (delay > lat) w = (int64_t)((double)w * (double)lat / (double)delay);
        }
        return std::max(w, kLAMinWeight);
    }
};

struct LATree {
    std::vector<ServerId> servers;
    std::vector<std::shared_ptr<LAServerStats>> stats;
    std::unique_ptr<std::atomic<int64_t>[]> fen;   // 1-based Fenwick tree
    std::unique_ptr<std::atomic<int64_t>[]> leaf;  // this copy's value of each leaf
    std::unordered_map<SocketId, size_t> index;     // server -> leaf (read-only between rebuilds)
    size_t n = 0;

    void rebuild() {
        n = servers.size();
        index.clear();
        for (size_t i = 0; i < n; ++i) index[servers[i].id] = i;
        fen.reset(new std::atomic<int64_t>[n + 1]);
        leaf.reset(new std::atomic<int64_t>[n]);
        std::vector<int64_t> f(n + 1, 0);
        for (size_t i = 0; i < n; ++i) {
            const int64_t w = std::max(stats[i]->weight.load(std::memory_order_relaxed), kLAMinWeight);
            leaf[i].store(w, std::memory_order_relaxed);
            f[i + 1] += w;
            const size_t parent = (i + 1) + ((i + 1) & (~(i + 1) + 1));
            if (parent <= n) f[parent] += f[i + 1];
        }
        for (size_t i = 0; i <= n; ++i) fen[i].store(f[i], std::memory_order_relaxed);
    }
    int64_t total() const {
        int64_t t = 0;
        for (size_t i = n; i > 0; i -= i & (~i + 1)) t += fen[i].load(std::memory_order_relaxed);
        return t;
    }
    // Set leaf i to w (lock-free; concurrent setters of one leaf serialise
    // through the exchange).
    void set(size_t i, int64_t w) const {
        const int64_t old = leaf[i].exchange(w, std::memory_order_relaxed);
        const int64_t diff = w - old;
        if (!diff) return;
        for (size_t k = i + 1; k <= n; k += k & (~k + 1)) fen[k].fetch_add(diff, std::memory_order_relaxed);
    }
    // Index whose cumulative range contains r (0 <= r < total).
    size_t find(int64_t r) const {
        size_t pos = 0;
        size_t step = 1;
        while (step * 2 <= n) step *= 2;
        for (; step; step >>= 1) {
            if (pos + step <= n) {
                const int64_t v = fen[pos + step].load(std::memory_order_relaxed);
                if (v <= r) {
                    pos += step;
                    r -= v;
                }
            }
        }
        return pos < n ? pos : n - 1;
    }
};

class LocalityAwareLB : public LoadBalancer {
public:
    bool AddServer(const ServerId& s) override {
        auto st = std::make_shared<LAServerStats>();
        // a newcomer starts at the average weight of the cluster, so it is
        // explored without being flooded
        st->weight.store(average_weight(), std::memory_order_relaxed);
        return _db.Modify([&](LATree& t) -> size_t {
            for (auto& x : t.servers) {
                if (x.id == s.id) return 0;
            }
            t.servers.push_back(s);
            t.stats.push_back(st);
            t.rebuild();
            return 1;
        }) > 0;
    }
    bool RemoveServer(const ServerId& s) override {
        return _db.Modify([&s](LATree& t) -> size_t {
            for (size_t i = 0; i < t.servers.size(); ++i) {
                if (t.servers[i].id == s.id) {
                    t.servers.erase(t.servers.begin() + i);
                    t.stats.erase(t.stats.begin() + i);
                    t.rebuild();
                    return 1;
                }
            }
            return 0;
        }) > 0;
    }
    size_t ServerCount() const override {
        DoublyBufferedData<LATree>::ScopedPtr p;
        const_cast<DoublyBufferedData<LATree>&>(_db).Read(&p);
        return p->n;
    }
    int SelectServer(const SelectIn& in, SelectOut* out) override {
        DoublyBufferedData<LATree>::ScopedPtr p;
        _db.Read(&p);
        const LATree& t = *p;
        if (t.n == 0) return EHOSTDOWN;
        const int64_t now = in.begin_time_us ? in.begin_time_us : monotonic_us();
        // weighted draws first; if they keep hitting excluded or unavailable
        // servers, scan from a random start for any usable one (excluded
        // servers last, as the other LBs do)
        size_t chosen = t.n;
        for (size_t attempt = 0; attempt < t.n + 2 && chosen == t.n; ++attempt) {
            const int64_t total = t.total();
            const size_t i = total > 0 ? t.find((int64_t)fast_rand_less_than((uint64_t)total))
                                       : (size_t)fast_rand_less_than(t.n);
            if (in.excluded && in.excluded->IsExcluded(t.servers[i].id)) continue;
            if (IsServerAvailable(t.servers[i].id, out->ptr)) chosen = i;
        }
        for (int pass = 0; pass < 2 && chosen == t.n; ++pass) {
            const size_t start = (size_t)fast_rand_less_than(t.n);
            for (size_t k = 0; k < t.n; ++k) {
                const size_t i = (start + k) % t.n;
                if (pass == 0 && in.excluded && in.excluded->IsExcluded(t.servers[i].id)) continue;
                if (IsServerAvailable(t.servers[i].id, out->ptr)) {
                    chosen = i;
                    break;
                }
            }
        }
        if (chosen == t.n) return EHOSTDOWN;
        LAServerStats& st = *t.stats[chosen];
        int64_t w;
        {
            std::lock_guard<std::mutex> g(st.mu);
            ++st.inflight;
            st.inflight_begin_sum_us += now;
            w = st.compute_locked(now, _default_latency.load(std::memory_order_relaxed));
        }
        st.weight.store(w, std::memory_order_relaxed);
        t.set(chosen, w);
        out->need_feedback = true;
        return 0;
    }
    void Feedback(const CallInfo& info) override {
        DoublyBufferedData<LATree>::ScopedPtr p;
        _db.Read(&p);
        const LATree& t = *p;
        auto it = t.index.find(info.server_id);
        if (it == t.index.end()) return;  // removed meanwhile
        const size_t i = it->second;
        LAServerStats& st = *t.stats[i];
        const int64_t now = monotonic_us();
        int64_t lat = now - info.begin_time_us;
        int64_t w;
        {
            std::lock_guard<std::mutex> g(st.mu);
            if (st.inflight > 0) {
                --st.inflight;
                st.inflight_begin_sum_us -= info.begin_time_us;
            }
            if (info.error_code) {
                // an error costs like a slow call (reference: punish_error_ratio)
                st.errors.fetch_add(1, std::memory_order_relaxed);
                lat = std::max<int64_t>(lat, 2 * std::max<int64_t>(st.avg_latency_us, 1000));
            }
            lat = std::max<int64_t>(lat, 1);
            // EMA that converges fast for the first samples
            const int64_t k = std::min<int64_t>(st.samples + 1, 8);
            st.avg_latency_us = st.samples == 0 ? lat : (st.avg_latency_us * (k - 1) + lat) / k;
            ++st.samples;
            w = st.compute_locked(now, _default_latency.load(std::memory_order_relaxed));
        }
        st.weight.store(w, std::memory_order_relaxed);
        t.set(i, w);
        int64_t d = _default_latency.load(std::memory_order_relaxed);
        _default_latency.store(d == 0 ? lat : (d * 15 + lat) / 16, std::memory_order_relaxed);
    }
    LoadBalancer* New(const std::string&) const override { return new LocalityAwareLB; }
    void Describe(std::ostream& os) const override {
        os << "la";
        DoublyBufferedData<LATree>::ScopedPtr p;
        const_cast<DoublyBufferedData<LATree>&>(_db).Read(&p);
        os << "{n=" << p->n << " total=" << p->total() << "}";
    }

private:
    int64_t average_weight() {
        DoublyBufferedData<LATree>::ScopedPtr p;
        _db.Read(&p);
        return p->n ? std::max(p->total() / (int64_t)p->n, kLAMinWeight) : kLAWeightScale / 1000;
    }
    DoublyBufferedData<LATree> _db;
    std::atomic<int64_t> _default_latency{0};
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
