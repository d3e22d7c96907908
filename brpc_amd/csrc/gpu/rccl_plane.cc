#include "gpu/rccl_plane.h"

#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "fiber/butex.h"
#include "gpu/gpu.h"
#include "gpu/hbm_pool.h"
#include "var/var.h"

DEFINE_int32(rccl_timeout_ms, 10000,
             "abort the RCCL plane when its oldest group made no progress for this long");
DEFINE_int32(rccl_max_group_ops, 256, "most sends/receives issued as one ncclGroupStart/End group");

namespace mrpc {
namespace gpu {
namespace rccl {

namespace {

// The entry points we use, resolved from the RCCL the process already has
// (torch's) or from ROCm's.
struct Api {
    decltype(&::ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&::ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&::ncclCommAbort) comm_abort = nullptr;
    decltype(&::ncclCommGetAsyncError) async_error = nullptr;
    decltype(&::ncclSend) send = nullptr;
    decltype(&::ncclRecv) recv = nullptr;
    decltype(&::ncclGroupStart) group_start = nullptr;
    decltype(&::ncclGroupEnd) group_end = nullptr;
    decltype(&::ncclGetErrorString) error_string = nullptr;
};

bool load_api(Api* a, std::string* err) {
    static std::once_flag once;
    static void* lib = nullptr;
    std::call_once(once, [] {
        for (const char* n : {"librccl.so", "librccl.so.1"}) {
            lib = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
            if (lib) return;
        }
        for (const char* n : {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so"}) {
            lib = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
            if (lib) return;
        }
    });
    if (!lib) {
        if (err) *err = "librccl.so not found";
        return false;
    }
#define MRPC_RCCL_SYM(field, name)                                       \
    a->field = reinterpret_cast<decltype(a->field)>(dlsym(lib, name));   \
    if (!a->field) {                                                     \
        if (err) *err = std::string("librccl.so lacks ") + name;         \
        return false;                                                    \
    }
    MRPC_RCCL_SYM(get_unique_id, "ncclGetUniqueId");
    MRPC_RCCL_SYM(comm_init_rank, "ncclCommInitRank");
    MRPC_RCCL_SYM(comm_abort, "ncclCommAbort");
    MRPC_RCCL_SYM(async_error, "ncclCommGetAsyncError");
    MRPC_RCCL_SYM(send, "ncclSend");
    MRPC_RCCL_SYM(recv, "ncclRecv");
    MRPC_RCCL_SYM(group_start, "ncclGroupStart");
    MRPC_RCCL_SYM(group_end, "ncclGroupEnd");
    MRPC_RCCL_SYM(error_string, "ncclGetErrorString");
#undef MRPC_RCCL_SYM
    return true;
}

// Fibers receiving several payloads park on one butex: 0 pending, 1 done,
// -1 failed.
struct Waiter {
    std::atomic<int>* butex = nullptr;
    std::atomic<int> left{0};
    std::atomic<bool> failed{false};
};

void finish(Waiter* w, bool ok) {
    if (!w) return;
    if (!ok) w->failed.store(true, std::memory_order_relaxed);
    if (w->left.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        // the waiter may return (and its Waiter die) as soon as the store
        // lands; butexes are pooled, so waking through the copy is safe
        std::atomic<int>* b = w->butex;
        b->store(w->failed.load(std::memory_order_relaxed) ? -1 : 1, std::memory_order_release);
        fiber::butex_wake_all(b);
    }
}

struct Op {
    bool is_send = false;
    int peer = 0;
    uint64_t seq = 0;
    void* ptr = nullptr;
    size_t len = 0;
    Buf hold;               // send: the payload; discard: the scratch block
    Waiter* waiter = nullptr;
    int64_t queued_us = 0;  // receives: when the reorder buffer took it
};

struct Inflight {
    hipEvent_t ev = nullptr;
    std::vector<Op> ops;
    int64_t issued_us = 0;
};

std::atomic<int64_t> g_sent{0}, g_sent_bytes{0}, g_recv{0}, g_recv_bytes{0}, g_discarded{0}, g_groups{0},
    g_aborts{0}, g_reorder{0};

class Plane {
public:
    Api api;
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    int device = -1, rank = 0, world = 0;
    uint64_t id = 0;

    std::mutex mu;
    std::condition_variable cv;
    std::vector<Op> ready;                       // issue in this order
    std::vector<uint64_t> next_send, next_recv;  // per peer / per source
    std::vector<std::map<uint64_t, Op>> held;    // per source: receives waiting for an earlier seq
    std::map<uint64_t, Op> self_sends;           // self payloads waiting for their receive
    bool dead = false, stop = false;
    std::atomic<bool> dead_flag{false};
    std::vector<uint64_t> skipped_self;  // cancelled self payloads (never announced)
    std::thread poster;

    int64_t send(int peer, const void* p, size_t len, Buf&& hold) {
        std::lock_guard<std::mutex> g(mu);
        if (dead || peer < 0 || peer >= world) return -1;
        Op op;
        op.is_send = true;
        op.peer = peer;
        op.seq = next_send[peer]++;
        op.ptr = const_cast<void*>(p);
        op.len = len;
        op.hold = std::move(hold);
        const int64_t seq = (int64_t)op.seq;
        if (peer == rank) {
            self_sends.emplace(op.seq, std::move(op));
        } else {
            ready.push_back(std::move(op));
            cv.notify_one();
        }
        return seq;
    }

    // Queue receives (under mu); drains every source into `ready` in order.
    bool add_recvs(std::vector<Op>* ops) {
        std::lock_guard<std::mutex> g(mu);
        if (dead) return false;
        for (Op& op : *ops) {
            if (op.seq < next_recv[op.peer] || held[op.peer].count(op.seq)) {
                // a payload announced twice: the pair is out of sync
                LOG(ERROR) << "rccl: duplicate receive of seq " << op.seq << " from rank " << op.peer;
                finish(op.waiter, false);
                continue;
            }
            const int src = op.peer;
            const uint64_t seq = op.seq;
            op.queued_us = monotonic_us();
            held[src].emplace(seq, std::move(op));
            if (seq != next_recv[src]) g_reorder.fetch_add(1, std::memory_order_relaxed);
            auto& h = held[src];
            for (auto it = h.find(next_recv[src]); it != h.end(); it = h.find(next_recv[src])) {
                if (src == rank) {
                    auto s = self_sends.find(it->first);
                    if (s == self_sends.end()) break;  // cannot happen: sends are queued first
                    ready.push_back(std::move(s->second));
                    self_sends.erase(s);
                }
                ready.push_back(std::move(it->second));
                h.erase(it);
                ++next_recv[src];
                if (src == rank) skip_cancelled_self();
            }
        }
        cv.notify_one();
        return true;
    }

    // (mu held) step over self payloads that were queued but never announced
    void skip_cancelled_self() {
        for (auto it = std::find(skipped_self.begin(), skipped_self.end(), next_recv[rank]); it != skipped_self.end();
             it = std::find(skipped_self.begin(), skipped_self.end(), next_recv[rank])) {
            skipped_self.erase(it);
            ++next_recv[rank];
        }
    }

    void cancel_self(uint64_t seq) {
        std::vector<Op> drop;
        {
            std::lock_guard<std::mutex> g(mu);
            auto s = self_sends.find(seq);
            if (s == self_sends.end()) return;
            drop.push_back(std::move(s->second));
            self_sends.erase(s);
            skipped_self.push_back(seq);
            skip_cancelled_self();
            // receives that waited behind the cancelled one can go now
            auto& h = held[rank];
            for (auto it = h.find(next_recv[rank]); it != h.end(); it = h.find(next_recv[rank])) {
                auto ss = self_sends.find(it->first);
                if (ss == self_sends.end()) break;
                ready.push_back(std::move(ss->second));
                self_sends.erase(ss);
                ready.push_back(std::move(it->second));
                h.erase(it);
                ++next_recv[rank];
                skip_cancelled_self();
            }
            cv.notify_one();
        }
        fail_ops(&drop);
    }

    // (mu held) a receive waited in the reorder buffer for too long: the
    // payload it waits behind was never announced
    bool reorder_stalled(int64_t now) const {
        for (const auto& h : held) {
            for (const auto& kv : h) {
                if (now - kv.second.queued_us > (int64_t)FLAGS_rccl_timeout_ms * 1000) return true;
            }
        }
        return false;
    }

    bool any_held() const {
        for (const auto& h : held)
            if (!h.empty()) return true;
        return false;
    }

    void fail_ops(std::vector<Op>* ops) {
        for (Op& op : *ops) {
            op.hold.clear();
            finish(op.waiter, false);
        }
        ops->clear();
    }

    // Called by the poster with mu NOT held.
    void abort(std::deque<Inflight>* inflight, const char* why) {
        LOG(ERROR) << "rccl plane aborted: " << why << " (payloads fall back to xGMI lending)";
        g_aborts.fetch_add(1, std::memory_order_relaxed);
        if (comm) api.comm_abort(comm);
        comm = nullptr;
        std::vector<Op> pending;
        {
            std::lock_guard<std::mutex> g(mu);
            dead = true;
            dead_flag.store(true, std::memory_order_release);
            pending.swap(ready);
            for (auto& h : held)
                for (auto& kv : h) pending.push_back(std::move(kv.second));
            for (auto& kv : self_sends) pending.push_back(std::move(kv.second));
            held.assign(held.size(), {});
            self_sends.clear();
        }
        fail_ops(&pending);
        for (Inflight& f : *inflight) {
            fail_ops(&f.ops);
            if (f.ev) ReleaseEvent(f.ev);
        }
        inflight->clear();
    }

    void complete(Inflight* f) {
        for (Op& op : f->ops) {
            if (op.is_send) {
                g_sent.fetch_add(1, std::memory_order_relaxed);
                g_sent_bytes.fetch_add((int64_t)op.len, std::memory_order_relaxed);
            } else if (op.waiter) {
                g_recv.fetch_add(1, std::memory_order_relaxed);
                g_recv_bytes.fetch_add((int64_t)op.len, std::memory_order_relaxed);
            } else {
                g_discarded.fetch_add(1, std::memory_order_relaxed);
            }
            op.hold.clear();
            finish(op.waiter, true);
        }
        ReleaseEvent(f->ev);
    }

    void run() {
        hipSetDevice(device);
        std::deque<Inflight> inflight;
        std::vector<Op> batch;
        for (;;) {
            bool stalled = false;
            {
                std::unique_lock<std::mutex> lk(mu);
                if (inflight.empty() && !any_held()) {
                    cv.wait(lk, [&] { return stop || !ready.empty(); });
                } else if (ready.empty()) {
                    const auto nap = inflight.empty() ? std::chrono::microseconds(5000) : std::chrono::microseconds(20);
                    cv.wait_for(lk, nap, [&] { return stop || !ready.empty(); });
                }
                if (stop) break;
                stalled = !dead && reorder_stalled(monotonic_us());
                const size_t n = std::min(ready.size(), (size_t)std::max(1, FLAGS_rccl_max_group_ops));
                // never split a self pair (send directly followed by its receive)
                size_t cut = n;
                if (cut < ready.size() && cut > 0 && ready[cut - 1].is_send && ready[cut - 1].peer == rank) ++cut;
                batch.assign(std::make_move_iterator(ready.begin()), std::make_move_iterator(ready.begin() + cut));
                ready.erase(ready.begin(), ready.begin() + cut);
            }
            if (stalled) {
                abort(&inflight, "a receive waited -rccl_timeout_ms for an earlier payload that never came");
                continue;
            }
            if (!batch.empty() && comm) {
                ncclResult_t r = api.group_start();
                for (const Op& op : batch) {
                    if (r != ncclSuccess) break;
                    r = op.is_send ? api.send(op.ptr, op.len, ncclUint8, op.peer, comm, stream)
                                   : api.recv(op.ptr, op.len, ncclUint8, op.peer, comm, stream);
                }
                const ncclResult_t e = api.group_end();
                if (r == ncclSuccess) r = e;
                Inflight f;
                f.ev = AcquireEvent();
                f.ops.swap(batch);
                f.issued_us = monotonic_us();
                const bool rec_ok = f.ev && hipEventRecord(f.ev, stream) == hipSuccess;
                inflight.push_back(std::move(f));
                g_groups.fetch_add(1, std::memory_order_relaxed);
                if (r != ncclSuccess || !rec_ok) {
                    abort(&inflight, r != ncclSuccess ? api.error_string(r) : "event record failed");
                    continue;
                }
            } else if (!batch.empty()) {
                fail_ops(&batch);
            }
            while (!inflight.empty()) {
                const hipError_t q = hipEventQuery(inflight.front().ev);
                if (q == hipErrorNotReady) break;
                if (q != hipSuccess) {
                    abort(&inflight, hipGetErrorString(q));
                    break;
                }
                complete(&inflight.front());
                inflight.pop_front();
            }
            if (!inflight.empty() && comm) {
                ncclResult_t ae = ncclSuccess;
                api.async_error(comm, &ae);
                if (ae != ncclSuccess && ae != ncclInProgress) {
                    abort(&inflight, api.error_string(ae));
                } else if (monotonic_us() - inflight.front().issued_us > (int64_t)FLAGS_rccl_timeout_ms * 1000) {
                    abort(&inflight, "no progress within -rccl_timeout_ms");
                }
            }
        }
        abort(&inflight, "shutdown");
    }
};

std::mutex g_mu;
Plane* g_plane = nullptr;
std::atomic<bool> g_active{false};

uint64_t fnv1a(const std::string& s) {
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    return h | 1;  // never 0: 0 means "no plane" in the hello
}

}  // namespace

std::string UniqueId(std::string* error) {
    Api a;
    if (!load_api(&a, error)) return std::string();
    ncclUniqueId id;
    const ncclResult_t r = a.get_unique_id(&id);
    if (r != ncclSuccess) {
        if (error) *error = a.error_string(r);
        return std::string();
    }
    return std::string(id.internal, sizeof(id.internal));
}

int Init(int rank, int world, const std::string& unique_id, int device, std::string* error) {
    std::lock_guard<std::mutex> g(g_mu);
    if (g_plane) {
        if (g_plane->id == fnv1a(unique_id) && g_plane->rank == rank) return 0;
        if (error) *error = "another RCCL plane is active";
        return -1;
    }
    if (world <= 0 || rank < 0 || rank >= world || unique_id.size() != sizeof(ncclUniqueId)) {
        if (error) *error = "bad rank/world/unique id";
        return -1;
    }
    if (device < 0) device = CurrentDevice();
    if (gpu::Init(device, error) != 0 || InitHbmPool(device, error) != 0) return -1;
    std::unique_ptr<Plane> p(new Plane);
    if (!load_api(&p->api, error)) return -1;
    p->device = device;
    p->rank = rank;
    p->world = world;
    p->id = fnv1a(unique_id);
    int prev = 0;
    hipGetDevice(&prev);
    hipSetDevice(device);
    ncclUniqueId id;
    memcpy(id.internal, unique_id.data(), sizeof(id.internal));
    ncclResult_t r = p->api.comm_init_rank(&p->comm, world, id, rank);
    if (r != ncclSuccess) {
        hipSetDevice(prev);
        if (error) *error = std::string("ncclCommInitRank: ") + p->api.error_string(r);
        return -1;
    }
    if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess) {
        p->api.comm_abort(p->comm);
        hipSetDevice(prev);
        if (error) *error = "hipStreamCreate failed";
        return -1;
    }
    // Connect every pair now (RCCL connects p2p peers lazily inside
    // ncclGroupEnd, which would block the poster on a peer that has not yet
    // posted anything to us): one byte to and from every rank, collectively.
    void* warm = nullptr;
    if (hipMalloc(&warm, 2 * (size_t)world) != hipSuccess) warm = nullptr;
    r = warm ? p->api.group_start() : ncclInternalError;
    for (int q = 0; q < world && r == ncclSuccess; ++q) {
        r = p->api.send(static_cast<char*>(warm) + q, 1, ncclUint8, q, p->comm, p->stream);
        if (r == ncclSuccess) r = p->api.recv(static_cast<char*>(warm) + world + q, 1, ncclUint8, q, p->comm, p->stream);
    }
    if (warm) {
        const ncclResult_t e = p->api.group_end();
        if (r == ncclSuccess) r = e;
    }
    const bool synced = warm && r == ncclSuccess && hipStreamSynchronize(p->stream) == hipSuccess;
    if (warm) hipFree(warm);
    hipSetDevice(prev);
    if (!synced) {
        p->api.comm_abort(p->comm);
        hipStreamDestroy(p->stream);
        if (error) *error = std::string("rccl warm-up exchange failed: ") + p->api.error_string(r);
        return -1;
    }
    p->next_send.assign(world, 0);
    p->next_recv.assign(world, 0);
    p->held.assign(world, {});
    Plane* raw = p.release();
    raw->poster = std::thread([raw] { raw->run(); });
    g_plane = raw;
    g_active.store(true, std::memory_order_release);
    static var::PassiveStatus<int64_t> v1("rccl_sent_bytes", [] { return g_sent_bytes.load(); });
    static var::PassiveStatus<int64_t> v2("rccl_recv_bytes", [] { return g_recv_bytes.load(); });
    static var::PassiveStatus<int64_t> v3("rccl_groups", [] { return g_groups.load(); });
    static var::PassiveStatus<int64_t> v4("rccl_aborts", [] { return g_aborts.load(); });
    LOG(INFO) << "rccl plane up: rank " << rank << "/" << world << " on device " << device;
    return 0;
}

bool Active() {
    return g_active.load(std::memory_order_acquire) && !g_plane->dead_flag.load(std::memory_order_acquire);
}
int Rank() { return g_active.load(std::memory_order_acquire) ? g_plane->rank : -1; }
int World() { return g_active.load(std::memory_order_acquire) ? g_plane->world : 0; }
uint64_t PlaneId() { return g_active.load(std::memory_order_acquire) ? g_plane->id : 0; }

void Shutdown() {
    std::lock_guard<std::mutex> g(g_mu);
    if (!g_plane) return;
    {
        std::lock_guard<std::mutex> lk(g_plane->mu);
        g_plane->stop = true;
        g_plane->cv.notify_one();
    }
    if (g_plane->poster.joinable()) g_plane->poster.join();
    // the plane object stays (Active() is false from now on): late callers
    // may still hold a pointer to it
}

int64_t Send(int peer, const void* p, size_t len, Buf&& hold) {
    if (!g_active.load(std::memory_order_acquire) || len == 0) return -1;
    return g_plane->send(peer, p, len, std::move(hold));
}

int Recv(int n, const int* src, const uint64_t* seq, const size_t* len, Buf* outs) {
    if (n <= 0) return 0;
    if (!g_active.load(std::memory_order_acquire)) return -1;
    Plane* pl = g_plane;
    Waiter w;
    w.butex = fiber::butex_create();
    w.butex->store(0, std::memory_order_relaxed);
    w.left.store(n, std::memory_order_relaxed);
    std::vector<Op> ops(n);
    bool ok = true;
    for (int i = 0; i < n; ++i) {
        ops[i].peer = src[i];
        ops[i].seq = seq[i];
        ops[i].len = len[i];
        ops[i].waiter = &w;
        if (src[i] < 0 || src[i] >= pl->world || len[i] == 0) ok = false;
        else if (!(ops[i].ptr = AppendNewDeviceBlock(&outs[i], len[i], pl->device))) ok = false;
    }
    if (!ok) {
        // on a bad descriptor the good ones still drain the peer's sends
        for (Op& op : ops) {
            if (op.peer >= 0 && op.peer < pl->world && op.len > 0) Discard(op.peer, op.seq, op.len);
        }
        for (int i = 0; i < n; ++i) outs[i].clear();
        fiber::butex_destroy(w.butex);
        return -1;
    }
    if (!pl->add_recvs(&ops)) {  // plane dead: nothing was queued
        for (int i = 0; i < n; ++i) outs[i].clear();
        fiber::butex_destroy(w.butex);
        return -1;
    }
    while (w.butex->load(std::memory_order_acquire) == 0) fiber::butex_wait(w.butex, 0);
    const int rc = w.butex->load(std::memory_order_acquire) == 1 ? 0 : -1;
    fiber::butex_destroy(w.butex);
    if (rc != 0)
        for (int i = 0; i < n; ++i) outs[i].clear();
    return rc;
}

void Discard(int src, uint64_t seq, size_t len) {
    if (!g_active.load(std::memory_order_acquire)) return;
    Plane* pl = g_plane;
    if (src < 0 || src >= pl->world || len == 0) return;
    std::vector<Op> ops(1);
    ops[0].peer = src;
    ops[0].seq = seq;
    ops[0].len = len;
    ops[0].ptr = AppendNewDeviceBlock(&ops[0].hold, len, pl->device);
    if (!ops[0].ptr) {
        LOG(ERROR) << "rccl: no HBM to drain payload " << seq << " from rank " << src;
        return;  // the watchdog will abort the stalled pair
    }
    pl->add_recvs(&ops);
}

void Cancelled(int peer, uint64_t seq) {
    if (!g_active.load(std::memory_order_acquire)) return;
    if (peer == g_plane->rank) {
        g_plane->cancel_self(seq);  // never issued: just skip its number
        return;
    }
    LOG(ERROR) << "rccl: payload " << seq << " to rank " << peer
               << " was queued but never announced; the pair cannot resynchronise";
    // the poster's watchdog aborts the plane once the orphaned send stalls
}

Stats GetStats() {
    Stats s;
    s.sent_payloads = g_sent.load();
    s.sent_bytes = g_sent_bytes.load();
    s.recv_payloads = g_recv.load();
    s.recv_bytes = g_recv_bytes.load();
    s.discarded = g_discarded.load();
    s.groups = g_groups.load();
    s.aborts = g_aborts.load();
    s.reorder_waits = g_reorder.load();
    return s;
}

}  // namespace rccl
}  // namespace gpu
}  // namespace mrpc
