#include "gpu/rccl_plane.h"

#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <linux/futex.h>
#include <rccl/rccl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "fiber/butex.h"
#include "gpu/gpu.h"
#include "gpu/hbm_pool.h"
#include "gpu/kernels.h"
#include "mrpc/proto/device_payload.pb.h"
#include "var/var.h"

DEFINE_int32(rccl_timeout_ms, 10000,
             "abort the plane when a group made no progress for this long (and fail Recv waits older than this)");
DEFINE_string(rccl_library, "",
              "RCCL library the plane dlopens (empty: the librccl.so the process has, else ROCm's); "
              "the stub build/lib/libfake_rccl.so runs the plane on CPU hosts");
DEFINE_int64(rccl_window_bytes, int64_t(256) << 20,
             "landing credit per source rank: payload bytes a peer may send beyond what this rank consumed");
DEFINE_int32(rccl_round_payloads, 64, "most payloads moved to one peer per pair round");
DEFINE_int64(rccl_round_bytes, int64_t(64) << 20, "most payload bytes moved to one peer per pair round");
DEFINE_int32(rccl_stash_ttl_ms, 30000, "received payloads nobody claims are dropped after this long");
DEFINE_int32(rccl_idle_spin_us, 0, "an idle plane poster watches its wake word this long before sleeping");
DEFINE_bool(rccl_self_copy, true,
            "payloads a rank sends to itself move with one batched copy kernel on the plane stream instead of "
            "ncclSend/ncclRecv pairs to self (RCCL's per-op overhead for what is a device-local copy)");
DEFINE_int32(rccl_self_pipeline, 0,
             "groups of only self payloads (-rccl_self_copy) the poster keeps in flight on its stream before "
             "it waits for the oldest (0: wait for each, like peer groups; 2-3 measured a worse N=1 tail, "
             "p99 351-367 vs 319 us: smaller groups, more of them)");
DEFINE_bool(rccl_defer_busy_peers, true,
            "do not offer a new pair round to a peer whose group is in flight (it could not fire before its "
            "group ends; the offer would mostly be withdrawn); offer when it rings back after the group");
DEFINE_int32(rccl_fire_grace_us, 40,
             "once a pair round fired, wait up to this long for the other pairs this rank is ready with to fire "
             "too before building the group (each ready bit cleared unfired is a withdrawal: its payloads go "
             "back to the queue for a later round)");
DEFINE_int32(rccl_poll_spin_us, 0,
             "the poster polls its in-flight group's completion with pause loops this long before it yields "
             "the core between polls");
DEFINE_int32(rccl_test_poster_delay_us, 0,
             "test only: the poster sleeps this long after every group (a slow or preempted rank)");

namespace mrpc {
namespace gpu {
namespace rccl {

namespace {

// ------------------------------------------------------------------ library
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
    // stub only (tests/stub/fake_rccl.cc): stream stand-ins
    void* (*fake_stream_create)() = nullptr;
    uint64_t (*fake_stream_record)(void*) = nullptr;
    int (*fake_stream_query)(void*, uint64_t) = nullptr;
    bool fake() const { return fake_stream_create != nullptr; }
};

bool load_api(Api* a, std::string* err) {
    static std::once_flag once;
    static void* lib = nullptr;
    static std::string load_err;
    std::call_once(once, [] {
        if (!FLAGS_rccl_library.empty()) {
            lib = dlopen(FLAGS_rccl_library.c_str(), RTLD_NOW | RTLD_LOCAL);
            if (!lib) load_err = std::string("dlopen ") + FLAGS_rccl_library + ": " + dlerror();
            return;
        }
        for (const char* n : {"librccl.so", "librccl.so.1"}) {
            lib = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
            if (lib) return;
        }
        for (const char* n : {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so"}) {
            lib = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
            if (lib) return;
        }
        load_err = "librccl.so not found";
    });
    if (!lib) {
        if (err) *err = load_err;
        return false;
    }
#define MRPC_RCCL_SYM(field, name)                                       \
    a->field = reinterpret_cast<decltype(a->field)>(dlsym(lib, name));   \
    if (!a->field) {                                                     \
        if (err) *err = std::string("rccl library lacks ") + name;       \
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
    if (dlsym(lib, "mrpcfake_abi_version")) {
        a->fake_stream_create = reinterpret_cast<void* (*)()>(dlsym(lib, "mrpcfake_stream_create"));
        a->fake_stream_record = reinterpret_cast<uint64_t (*)(void*)>(dlsym(lib, "mrpcfake_stream_record"));
        a->fake_stream_query = reinterpret_cast<int (*)(void*, uint64_t)>(dlsym(lib, "mrpcfake_stream_query"));
        if (!a->fake_stream_create || !a->fake_stream_record || !a->fake_stream_query) {
            if (err) *err = "stub rccl library lacks its mrpcfake_stream_* functions";
            return false;
        }
    }
    return true;
}

// ------------------------------------------------------------------ streams
// The plane's one stream: groups, then a completion marker. A HIP stream
// and events on MI355X; the stub's executor on CPU hosts.
class StreamOps {
public:
    virtual ~StreamOps() {}
    virtual int init(int device, std::string* err) = 0;
    virtual void* stream() = 0;
    virtual int record(uint64_t* marker) = 0;
    // 1 complete, 0 pending, -1 failed
    virtual int query(uint64_t marker) = 0;
    virtual void release(uint64_t marker) = 0;
    virtual void* alloc(size_t len, Buf* out) = 0;
    virtual bool accepts(const BufBlock* b) const = 0;
    virtual bool host_memory() const = 0;
    // queue copies on the stream (self payloads: rank to itself)
    virtual int copy(const std::vector<Segment>& segs) = 0;
};

class HipOps : public StreamOps {
public:
    int init(int device, std::string* err) override {
        _device = device;
        hipSetDevice(device);
        if (hipStreamCreateWithFlags(&_stream, hipStreamNonBlocking) != hipSuccess) {
            if (err) *err = "hipStreamCreate failed";
            return -1;
        }
        return 0;
    }
    void* stream() override { return _stream; }
    int record(uint64_t* marker) override {
        hipEvent_t ev = AcquireEvent();
        if (!ev || hipEventRecord(ev, _stream) != hipSuccess) {
            if (ev) ReleaseEvent(ev);
            return -1;
        }
        *marker = reinterpret_cast<uint64_t>(ev);
        return 0;
    }
    int query(uint64_t marker) override {
        const hipError_t q = hipEventQuery(reinterpret_cast<hipEvent_t>(marker));
        if (q == hipSuccess) return 1;
        if (q == hipErrorNotReady) return 0;
        return -1;
    }
    void release(uint64_t marker) override { ReleaseEvent(reinterpret_cast<hipEvent_t>(marker)); }
    void* alloc(size_t len, Buf* out) override { return AppendNewDeviceBlock(out, len, _device); }
    bool accepts(const BufBlock* b) const override { return b->kind == MemKind::DEVICE && b->device == _device; }
    bool host_memory() const override { return false; }
    int copy(const std::vector<Segment>& segs) override {
        for (size_t i = 0; i < segs.size(); i += kInlineSegments) {
            const int n = (int)std::min<size_t>(kInlineSegments, segs.size() - i);
            if (LaunchBatchedCopy(segs.data() + i, n, _stream) != 0) return -1;
        }
        return 0;
    }

private:
    int _device = -1;
    hipStream_t _stream = nullptr;
};

void free_host(void* p, void*) { free(p); }

class StubOps : public StreamOps {
public:
    explicit StubOps(const Api& a) : _api(a) {}
    int init(int, std::string* err) override {
        _stream = _api.fake_stream_create();
        if (!_stream) {
            if (err) *err = "stub stream creation failed";
            return -1;
        }
        return 0;
    }
    void* stream() override { return _stream; }
    int record(uint64_t* marker) override {
        *marker = _api.fake_stream_record(_stream);
        return 0;
    }
    int query(uint64_t marker) override { return _api.fake_stream_query(_stream, marker); }
    void release(uint64_t) override {}
    void* alloc(size_t len, Buf* out) override {
        void* p = malloc(std::max<size_t>(len, 1));
        if (!p) return nullptr;
        out->append_user_data(p, len, free_host);
        return p;
    }
    bool accepts(const BufBlock* b) const override { return IsHostAccessible(b->kind); }
    bool host_memory() const override { return true; }
    int copy(const std::vector<Segment>& segs) override {
        // the stub's stream runs groups synchronously at group end, and the
        // marker recorded after this completes after it
        for (const Segment& g : segs) memcpy(g.dst, g.src, g.len);
        return 0;
    }

private:
    const Api& _api;
    void* _stream = nullptr;
};

// ------------------------------------------------------------------ node shm
// Everything the ranks of a node tell each other goes through one POSIX shm
// segment, never through RCCL: per unordered pair of ranks a round word and
// the two sides' payload lists, landing credit and cancel rings; per rank a
// futex wake word; the node's abort flag.
const int kMaxRanks = 16;  // ranks of one node's plane
const int kListMax = 64;   // payloads one side moves in one pair round
const int kCancelRing = 64;

struct Entry {
    uint64_t seq;
    uint64_t len;
};
struct PairList {
    uint32_t n;
    uint32_t pad;
    Entry e[kListMax];
};
struct CancelRing {  // single producer (the sender), single consumer (the receiver)
    std::atomic<uint64_t> head;
    std::atomic<uint64_t> tail;
    uint64_t seq[kCancelRing];
};
// A pair's rounds: word = round << 2 | ready(low rank) | ready(high rank) << 1.
// A side publishes its list for the open round, then sets its ready bit; the
// side that finds the other bit already set fires the round by moving the
// word to (round + 1, no bits). Both sides then issue that round's sends and
// receives. A side clears its bit (withdraws) with a CAS; a failed CAS means
// the peer fired meanwhile and the round must be issued.
struct alignas(64) PairSlot {
    std::atomic<uint64_t> word;
    char pad0[56];
    std::atomic<uint64_t> consumed[2];  // [direction]: bytes the receiver consumed (0: low -> high)
    std::atomic<uint32_t> stalled[2];   // [direction]: the sender waits for credit
    char pad1[40];
    PairList list[2][2];                // [round % 2][side]
    CancelRing cancels[2];              // [direction]: sequences the receiver must drop
};
const int kMaxPairs = kMaxRanks * (kMaxRanks - 1) / 2;

const uint64_t kBellMagic = 0x4d52504342454c33ull;  // "MRPCBEL3"
struct Doorbell {
    uint64_t magic;
    std::atomic<uint32_t> seq;     // bumped on abort (futex word of no one in particular)
    std::atomic<uint32_t> claim;   // the first aborting rank claims the reason slot
    std::atomic<uint32_t> abort;   // 0, or 1 + the rank that aborted first
    char reason[200];
    std::atomic<int32_t> pid[kMaxRanks];
    std::atomic<uint32_t> wake[kMaxRanks];  // futex word per rank: bumped by whoever has news for it
    std::atomic<uint32_t> busy[kMaxRanks];  // 1 while the rank has a group in flight
    PairSlot pairs[kMaxPairs];
};

long futex(std::atomic<uint32_t>* w, int op, uint32_t val, const timespec* ts) {
    return syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), op, val, ts, nullptr, 0);
}

uint64_t fnv1a(const std::string& s) {
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    return h | 1;  // never 0: 0 means "no plane" in the hello
}

int pair_index(int a, int b) {
    if (a > b) std::swap(a, b);
    return a * (2 * kMaxRanks - a - 1) / 2 + (b - a - 1);
}

// ------------------------------------------------------------------ state
struct Payload {
    uint64_t seq = 0;
    void* ptr = nullptr;
    size_t len = 0;
    Buf hold;  // send: the bytes; receive: the landing block
};

struct Waiter {
    std::atomic<int>* butex = nullptr;
    int left = 0;  // under Plane::mu
    bool failed = false;
};

struct WaitSlot {
    Waiter* w = nullptr;
    Buf* out = nullptr;
};

struct Stashed {
    Buf buf;
    size_t len = 0;
    int64_t since_us = 0;
};

typedef std::pair<int, uint64_t> Key;  // (source rank, sequence)

struct PeerState {
    std::deque<Payload> queued;        // not listed yet
    std::vector<Payload> listed;       // in our list of the pair's open round
    uint64_t next_seq = 0;
    uint64_t announced_bytes = 0;      // cumulative bytes listed to this peer (credit)
    uint64_t consumed = 0;             // cumulative bytes from this peer claimed/dropped
    uint64_t round = 0;                // the pair's open round, as this side knows it
    bool ready = false;                // our ready bit is set for `round`
    std::vector<uint64_t> cancels;     // moved (or listed) to this peer, then cancelled
};

std::atomic<int64_t> g_sent{0}, g_sent_bytes{0}, g_recv{0}, g_recv_bytes{0}, g_discarded{0}, g_rounds{0},
    g_payload_rounds{0}, g_aborts{0}, g_credit_stalls{0}, g_expired{0}, g_recv_timeouts{0}, g_doorbells{0},
    g_withdrawn{0}, g_pair_rounds{0}, g_withdrawals{0}, g_group_us{0};

void finish_locked(Waiter* w, bool ok) {
    if (!ok) w->failed = true;
    if (--w->left == 0) {
        std::atomic<int>* b = w->butex;
        b->store(w->failed ? -1 : 1, std::memory_order_release);
        fiber::butex_wake_all(b);
    }
}

class Plane {
public:
    Api api;
    ncclComm_t comm = nullptr;
    std::unique_ptr<StreamOps> ops;
    int device = -1, rank = 0, world = 0;
    uint64_t id = 0;
    Doorbell* bell = nullptr;
    std::string bell_name;

    std::mutex mu;
    std::vector<PeerState> peers;
    std::vector<char> in_last_group;  // [peer]: a pair round with it was in our latest group
    std::deque<Payload> self_q;
    std::map<Key, Stashed> stash;
    std::map<Key, WaitSlot> waiting;
    std::map<Key, int64_t> discards;
    std::map<Key, int64_t> lost;   // self payloads that found no memory to land in: their Recv fails
    uint64_t self_moved = 0;       // cumulative self bytes landed (credit: vs peers[rank].consumed)
    bool idle = false, dead = false, stop = false;
    std::atomic<bool> dead_flag{false};
    std::thread poster;
    int64_t last_expire_us = 0, last_liveness_us = 0;

    // the group in flight (poster only)
    std::vector<std::vector<Payload>> moving_send, moving_recv;
    std::vector<Payload> self_send, self_recv;
    struct SelfFlight {  // a self-only group on the stream, not waited for yet (poster only)
        uint64_t marker = 0;
        std::vector<Payload> send, recv;
    };
    std::deque<SelfFlight> self_flight;
    uint64_t marker = 0;
    bool marker_live = false;
    std::vector<Buf> graveyard;  // blocks RCCL may still touch after an abort

    // ---------------------------------------------------------------- shm
    PairSlot* slot(int peer) const { return &bell->pairs[pair_index(rank, peer)]; }
    int side_with(int peer) const { return rank < peer ? 0 : 1; }
    // direction index of payloads from `src` to `dst`
    static int dir(int src, int dst) { return src < dst ? 0 : 1; }

    void ring(int r) {
        bell->wake[r].fetch_add(1, std::memory_order_acq_rel);
        futex(&bell->wake[r], FUTEX_WAKE, INT_MAX, nullptr);
    }

    // ---------------------------------------------------------------- API
    int64_t send(int peer, const void* p, size_t len, Buf&& hold) {
        std::lock_guard<std::mutex> g(mu);
        if (dead || stop || peer < 0 || peer >= world) return -1;
        Payload pl;
        pl.seq = peers[peer].next_seq++;
        pl.ptr = const_cast<void*>(p);
        pl.len = len;
        pl.hold = std::move(hold);
        const int64_t seq = (int64_t)pl.seq;
        if (peer == rank) self_q.push_back(std::move(pl));
        else peers[peer].queued.push_back(std::move(pl));
        if (idle) {
            idle = false;
            g_doorbells.fetch_add(1, std::memory_order_relaxed);
            ring(rank);
        }
        return seq;
    }

    int recv(int n, const int* src, const uint64_t* seq, const size_t* len, Buf* outs) {
        Waiter w;
        w.butex = fiber::butex_create();
        w.butex->store(0, std::memory_order_relaxed);
        std::vector<Key> mine;
        {
            std::lock_guard<std::mutex> g(mu);
            if (dead) {
                fiber::butex_destroy(w.butex);
                return -1;
            }
            for (int i = 0; i < n; ++i) {
                const Key k(src[i], seq[i]);
                if (src[i] < 0 || src[i] >= world) {
                    w.failed = true;
                    continue;
                }
                auto l = lost.find(k);
                if (l != lost.end()) {
                    lost.erase(l);
                    w.failed = true;
                    continue;
                }
                auto s = stash.find(k);
                if (s != stash.end()) {
                    if (s->second.len != len[i]) w.failed = true;
                    outs[i] = std::move(s->second.buf);
                    consume_locked(src[i], s->second.len);
                    stash.erase(s);
                    continue;
                }
                if (waiting.count(k)) {
                    w.failed = true;
                    continue;
                }
                waiting[k] = WaitSlot{&w, &outs[i]};
                mine.push_back(k);
                ++w.left;
            }
            if (w.left == 0) w.butex->store(w.failed ? -1 : 1, std::memory_order_relaxed);
        }
        const int64_t deadline = monotonic_us() + (int64_t)FLAGS_rccl_timeout_ms * 1000;
        while (w.butex->load(std::memory_order_acquire) == 0) {
            const int64_t now = monotonic_us();
            if (now >= deadline) break;
            timespec ts = abstime_after_us(deadline - now);
            fiber::butex_wait(w.butex, 0, &ts);
        }
        int rc;
        {
            std::lock_guard<std::mutex> g(mu);
            rc = w.butex->load(std::memory_order_acquire);
            if (rc == 0) {  // timed out: withdraw what is still pending
                for (const Key& k : mine) {
                    auto it = waiting.find(k);
                    if (it != waiting.end() && it->second.w == &w) {
                        waiting.erase(it);
                        discards[k] = monotonic_us();
                    }
                }
                g_recv_timeouts.fetch_add(1, std::memory_order_relaxed);
                rc = -1;
            }
        }
        fiber::butex_destroy(w.butex);
        if (rc != 1) {
            for (int i = 0; i < n; ++i) outs[i].clear();
            return -1;
        }
        return 0;
    }

    static timespec abstime_after_us(int64_t us) {
        timespec ts;
        clock_gettime(CLOCK_REALTIME, &ts);
        const int64_t ns = ts.tv_nsec + (us % 1000000) * 1000;
        ts.tv_sec += us / 1000000 + ns / 1000000000;
        ts.tv_nsec = ns % 1000000000;
        return ts;
    }

    // (mu held) bytes from `src` were claimed or dropped: return the credit,
    // and wake the sender if it waits for it
    void consume_locked(int src, size_t len) {
        PeerState& ps = peers[src];
        ps.consumed += len;
        if (src == rank) return;
        PairSlot* s = slot(src);
        const int d = dir(src, rank);
        s->consumed[d].store(ps.consumed, std::memory_order_release);
        if (s->stalled[d].load(std::memory_order_acquire) && s->stalled[d].exchange(0)) ring(src);
    }

    void discard(int src, uint64_t seq, size_t len) {
        (void)len;
        Buf drop;  // released after the lock
        std::lock_guard<std::mutex> g(mu);
        discard_locked(src, seq, &drop);
    }

    // (mu held) drop payload (src, seq) now if it landed, else when it does
    void discard_locked(int src, uint64_t seq, Buf* drop) {
        if (src < 0 || src >= world) return;
        const Key k(src, seq);
        auto s = stash.find(k);
        if (s != stash.end()) {
            consume_locked(src, s->second.len);
            drop->append(std::move(s->second.buf));
            stash.erase(s);
            g_discarded.fetch_add(1, std::memory_order_relaxed);
            return;
        }
        discards[k] = monotonic_us();
    }

    void cancelled(int peer, uint64_t seq) {
        Buf drop;
        std::lock_guard<std::mutex> g(mu);
        if (peer < 0 || peer >= world) return;
        std::deque<Payload>& q = peer == rank ? self_q : peers[peer].queued;
        for (auto it = q.begin(); it != q.end(); ++it) {
            if (it->seq == seq) {
                drop = std::move(it->hold);
                q.erase(it);
                g_withdrawn.fetch_add(1, std::memory_order_relaxed);
                return;
            }
        }
        // listed or already moved. To ourselves: drop it here (now or when
        // it lands). To a peer: its cancel ring tells it to.
        if (peer == rank) {
            Buf dropped;
            discard_locked(rank, seq, &dropped);
            drop.append(std::move(dropped));
        } else {
            peers[peer].cancels.push_back(seq);
            if (idle) ring(rank);
        }
        g_withdrawn.fetch_add(1, std::memory_order_relaxed);
    }

    // ---------------------------------------------------------------- poster
    // One pass: issue nothing that a peer is not also about to issue. A pair
    // round fires only when both sides are ready for it, and every fired
    // round this rank takes part in goes into ONE group, the only group the
    // plane has in flight. A group therefore waits only for peers that
    // already committed to the matching group, never for a rank that is
    // busy elsewhere or slow: pairs with traffic move independently, idle
    // pairs exchange nothing.
    //
    // Why groups of different ranks cannot wait on each other in a cycle:
    //  * a rank sets ready bits only while it has no group in flight, and
    //    before it builds a group it clears every bit that did not fire (a
    //    failed clear means the pair fired: it joins the group). So while a
    //    group is in flight the rank has no bit set, nobody can fire a pair
    //    with it, and every pair-round in ANY rank's in-flight group is in
    //    the in-flight (or the next-built) group of its other endpoint too;
    //  * each group issues its pairs in ascending peer order, which is the
    //    same as ascending (low rank, high rank) pair order on every rank.
    //    Even a library that ran a group's peers strictly one after another
    //    then makes progress: the globally smallest pending pair is the
    //    first pending one at both of its endpoints. (RCCL runs a group's
    //    peers on parallel channels in its own delta-ordered schedule,
    //    which is deadlock-free on consistent groups as well.)
    // The stub library (one in-order queue per process, blocking sends) is
    // the serial worst case, and runs the plane at 2, 3 and 8 ranks.
    void run() {
        if (!ops->host_memory()) hipSetDevice(device);
        for (;;) {
            std::vector<int> fired;
            bool leave = false;
            {
                std::unique_lock<std::mutex> lk(mu);
                for (;;) {
                    if (dead || bell->abort.load(std::memory_order_acquire)) break;
                    const uint32_t s = bell->wake[rank].load(std::memory_order_acquire);
                    drain_cancels_locked();
                    // a leaving rank offers nothing new, but still issues
                    // rounds a peer fired with it (else that peer's group
                    // never completes)
                    offer_locked(&fired, /*offer_new=*/!stop);
                    if (stop) {
                        withdraw_all_locked(&fired);
                        leave = fired.empty();
                        break;
                    }
                    const bool self_room = (int)self_flight.size() < std::max(1, FLAGS_rccl_self_pipeline);
                    if (!fired.empty() || (self_room && self_ready_locked())) break;
                    if (!self_flight.empty()) {
                        // copies of self groups in flight: poll them, do not sleep
                        lk.unlock();
                        if (reap_self(/*block=*/false) != 0) {
                            lk.lock();
                            break;
                        }
                        if (!self_flight.empty()) {
                            for (int i = 0; i < 64; ++i) __builtin_ia32_pause();
                        }
                        lk.lock();
                        continue;
                    }
                    idle = true;
                    housekeeping_locked();
                    lk.unlock();
                    // watch the wake word a little while before sleeping: the
                    // next payload of a busy stream is usually close behind
                    const int64_t until = monotonic_us() + std::max(0, FLAGS_rccl_idle_spin_us);
                    while (bell->wake[rank].load(std::memory_order_acquire) == s && monotonic_us() < until) {
                        for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
                    }
                    timespec ts{0, 50 * 1000 * 1000};
                    futex(&bell->wake[rank], FUTEX_WAIT, s, &ts);
                    lk.lock();
                    idle = false;
                    if (check_liveness()) break;
                }
                idle = false;
                if (!leave && !stop && !fired.empty()) grace_locked(lk, &fired);
                if (!leave && !dead && !bell->abort.load(std::memory_order_acquire)) {
                    withdraw_all_locked(&fired);
                    build_group_locked(fired, /*with_self=*/!stop);
                }
            }
            if (leave) {
                reap_self(/*block=*/true);  // copies already on the stream land before the rank leaves
                break;
            }
            if (bell->abort.load(std::memory_order_acquire)) {
                abort(remote_reason(), false, !remote_is_shutdown());
                break;
            }
            if (dead) break;
            if (!stop && FLAGS_rccl_self_copy && FLAGS_rccl_self_pipeline > 0 && fired.empty() && !self_send.empty()) {
                if (issue_self() != 0) break;
                continue;
            }
            bell->busy[rank].store(1, std::memory_order_release);
            const int grc = run_group();
            // the stream is in order: self groups issued before this group
            // are done once it is
            const int src = grc == 0 ? reap_self(/*block=*/true) : 0;
            // every exit path clears busy and rings the peers:
            // a peer may have deferred offers to us whatever our own flag
            // says, and a stale busy word would keep deferring them
            bell->busy[rank].store(0, std::memory_order_release);
            for (int p = 0; p < world; ++p) {
                if (p != rank) ring(p);  // peers that deferred offers to us
            }
            if (grc != 0 || src != 0) break;
            if (!stop && FLAGS_rccl_test_poster_delay_us > 0) usleep((useconds_t)FLAGS_rccl_test_poster_delay_us);
        }
        if (!dead) abort("rank shut down", true, /*is_error=*/false);
    }

    // (mu held) peers' cancel rings: drop what they gave up
    void drain_cancels_locked() {
        for (int p = 0; p < world; ++p) {
            if (p == rank) continue;
            CancelRing& r = slot(p)->cancels[dir(p, rank)];
            uint64_t t = r.tail.load(std::memory_order_relaxed);
            const uint64_t h = r.head.load(std::memory_order_acquire);
            if (t == h) continue;
            Buf drop;
            for (; t < h; ++t) discard_locked(p, r.seq[t % kCancelRing], &drop);
            r.tail.store(t, std::memory_order_release);
        }
    }

    // (mu held) our cancels of payloads listed/moved to `p`, into its ring
    void publish_cancels_locked(int p) {
        PeerState& ps = peers[p];
        if (ps.cancels.empty()) return;
        CancelRing& r = slot(p)->cancels[dir(rank, p)];
        uint64_t h = r.head.load(std::memory_order_relaxed);
        const uint64_t t = r.tail.load(std::memory_order_acquire);
        size_t i = 0;
        for (; i < ps.cancels.size() && h - t < (uint64_t)kCancelRing; ++i, ++h) r.seq[h % kCancelRing] = ps.cancels[i];
        r.head.store(h, std::memory_order_release);
        // a full ring drops the rest: the receiver's stash expires those
        ps.cancels.clear();
        ring(p);
    }

    // (mu held) whether payload `len` fits the landing credit `p` granted
    bool fits_credit_locked(int p, size_t len) {
        PeerState& ps = peers[p];
        PairSlot* s = slot(p);
        const uint64_t window = (uint64_t)std::max<int64_t>(FLAGS_rccl_window_bytes, 1);
        const uint64_t consumed = s->consumed[dir(rank, p)].load(std::memory_order_acquire);
        // within credit, or the peer consumed everything we sent (a payload
        // larger than the window then goes alone)
        return ps.announced_bytes + len <= consumed + window || ps.announced_bytes <= consumed;
    }

    // (mu held) publish our list for the pair's open round: queued payloads
    // within credit and the per-round bounds
    void write_list_locked(int p, bool* stalled) {
        PeerState& ps = peers[p];
        PairList& l = slot(p)->list[ps.round % 2][side_with(p)];
        uint32_t n = 0;
        uint64_t bytes = 0;
        const int max_n = std::max(1, std::min(FLAGS_rccl_round_payloads, kListMax));
        while (!ps.queued.empty() && (int)n < max_n) {
            const Payload& q = ps.queued.front();
            if (n > 0 && bytes + q.len > (uint64_t)FLAGS_rccl_round_bytes) break;
            if (!fits_credit_locked(p, q.len)) {
                // ask for a wake-up when credit returns, then look once more
                // (the receiver may have consumed in between)
                PairSlot* s = slot(p);
                s->stalled[dir(rank, p)].store(1, std::memory_order_release);
                if (!fits_credit_locked(p, q.len)) {
                    *stalled = true;
                    break;
                }
            }
            l.e[n].seq = q.seq;
            l.e[n].len = q.len;
            ++n;
            bytes += q.len;
            ps.announced_bytes += q.len;
            ps.listed.push_back(std::move(ps.queued.front()));
            ps.queued.pop_front();
        }
        l.n = n;
    }

    // (mu held) the listed payloads go back to the front of the queue
    void unlist_locked(int p) {
        PeerState& ps = peers[p];
        for (auto it = ps.listed.rbegin(); it != ps.listed.rend(); ++it) {
            ps.announced_bytes -= it->len;
            ps.queued.push_front(std::move(*it));
        }
        ps.listed.clear();
    }

    // (mu held) every pair: notice fired rounds we were ready for, fire the
    // ones whose peer is ready, offer the ones with payloads within credit
    void offer_locked(std::vector<int>* fired, bool offer_new) {
        bool stalled = false;
        for (int p = 0; p < world; ++p) {
            if (p == rank) continue;
            PeerState& ps = peers[p];
            PairSlot* s = slot(p);
            const uint64_t mine = 1ull << side_with(p), other = 1ull << (1 - side_with(p));
            if (offer_new) publish_cancels_locked(p);
            uint64_t w = s->word.load(std::memory_order_acquire);
            if (ps.ready) {
                if ((w >> 2) != ps.round) fired->push_back(p);  // the peer fired it
                continue;
            }
            if (!offer_new) continue;
            const bool peer_ready = (w & other) != 0;
            // a peer with a group in flight cannot fire a round before that
            // group ends, and our bit would most likely be withdrawn (its
            // payloads re-queued) once some other pair fires first: offer to
            // it when it is back (it rings every peer after each group)
            // (a peer that shared our latest group is only finishing that
            // same group: announce now, it fires as soon as it is back)
            if (!peer_ready && FLAGS_rccl_defer_busy_peers && bell->busy[p].load(std::memory_order_acquire) &&
                !((size_t)p < in_last_group.size() && in_last_group[p])) {
                continue;
            }
            bool have = !ps.queued.empty() && (fits_credit_locked(p, ps.queued.front().len) || [&] {
                            s->stalled[dir(rank, p)].store(1, std::memory_order_release);
                            if (fits_credit_locked(p, ps.queued.front().len)) return true;
                            stalled = true;
                            return false;
                        }());
            if (!peer_ready && !have) continue;
            // (not ready: nothing of ours may be listed; a stale list would
            // be appended to and go out of step with the shm list)
            if (!ps.listed.empty()) unlist_locked(p);
            write_list_locked(p, &stalled);
            // what was actually listed decides: credit may have returned
            // since `have` was computed, and a list we publish without our
            // ready bit set would never be withdrawn
            have = !ps.listed.empty();
            for (;;) {
                if (w & other) {
                    // both ready: fire (the round moves on, both bits clear)
                    if (s->word.compare_exchange_weak(w, (ps.round + 1) << 2, std::memory_order_acq_rel)) {
                        ps.ready = true;
                        fired->push_back(p);
                        ring(p);
                        break;
                    }
                } else if (!have) {
                    break;  // the peer withdrew and we have nothing for it
                } else if (s->word.compare_exchange_weak(w, w | mine, std::memory_order_acq_rel)) {
                    ps.ready = true;
                    ring(p);  // it may be asleep with payloads for us, or none
                    break;
                }
            }
        }
        if (stalled) g_credit_stalls.fetch_add(1, std::memory_order_relaxed);
    }

    // (mu held, may drop it) a round fired: give the other pairs we are
    // ready with a short while to fire as well, so one group carries them
    // instead of withdrawing them now and offering them again next pass.
    // No group is in flight meanwhile, exactly as in the idle wait, so the
    // deadlock argument above is unchanged.
    void grace_locked(std::unique_lock<std::mutex>& lk, std::vector<int>* fired) {
        if (FLAGS_rccl_fire_grace_us <= 0) return;
        const int64_t until = monotonic_us() + FLAGS_rccl_fire_grace_us;
        for (;;) {
            int pending = 0;
            for (int p = 0; p < world; ++p) {
                if (p == rank || !peers[p].ready) continue;
                if (std::find(fired->begin(), fired->end(), p) != fired->end()) continue;
                if ((slot(p)->word.load(std::memory_order_acquire) >> 2) != peers[p].round) {
                    fired->push_back(p);  // the peer fired it
                } else {
                    ++pending;
                }
            }
            if (pending == 0 || monotonic_us() >= until || dead || bell->abort.load(std::memory_order_acquire)) {
                return;
            }
            lk.unlock();
            for (int i = 0; i < 64; ++i) __builtin_ia32_pause();
            lk.lock();
        }
    }

    // (mu held) clear our ready bit everywhere nothing fired; a failed clear
    // means the peer fired the round meanwhile, so it joins the group
    void withdraw_all_locked(std::vector<int>* fired) {
        for (int p = 0; p < world; ++p) {
            if (p == rank) continue;
            PeerState& ps = peers[p];
            if (!ps.ready || std::find(fired->begin(), fired->end(), p) != fired->end()) continue;
            PairSlot* s = slot(p);
            const uint64_t mine = 1ull << side_with(p);
            uint64_t w = s->word.load(std::memory_order_acquire);
            for (;;) {
                if ((w >> 2) != ps.round) {
                    fired->push_back(p);
                    break;
                }
                if (s->word.compare_exchange_weak(w, w & ~mine, std::memory_order_acq_rel)) {
                    ps.ready = false;
                    unlist_locked(p);
                    g_withdrawals.fetch_add(1, std::memory_order_relaxed);
                    break;
                }
            }
        }
    }

    // (mu held) self payloads that may land now (the same window a peer
    // grants: landed-but-unclaimed self bytes stay under -rccl_window_bytes)
    bool self_ready_locked() {
        if (self_q.empty()) return false;
        const uint64_t window = (uint64_t)std::max<int64_t>(FLAGS_rccl_window_bytes, 1);
        const uint64_t unclaimed = self_moved - peers[rank].consumed;
        return unclaimed == 0 || unclaimed + self_q.front().len <= window;
    }

    // (mu held) the group: for every fired pair, our listed payloads out and
    // the peer's listed payloads in; then self payloads
    void build_group_locked(const std::vector<int>& fired, bool with_self) {
        moving_send.assign(world, {});
        moving_recv.assign(world, {});
        in_last_group.assign(world, 0);
        for (int p : fired) in_last_group[p] = 1;
        self_send.clear();
        self_recv.clear();
        for (int p : fired) {
            PeerState& ps = peers[p];
            PairSlot* s = slot(p);
            const PairList& theirs = s->list[ps.round % 2][1 - side_with(p)];
            const PairList& ours = s->list[ps.round % 2][side_with(p)];
            // the peer receives what the shm list says: our sends must be
            // exactly that list, or the pair's sends and receives go out of
            // step (a hang until -rccl_timeout_ms at best)
            bool in_step = ours.n == ps.listed.size();
            for (uint32_t i = 0; in_step && i < ours.n; ++i)
                in_step = ours.e[i].seq == ps.listed[i].seq && ours.e[i].len == ps.listed[i].len;
            if (!in_step && dead_reason.empty()) {
                dead_reason = "pair list out of step with rank " + std::to_string(p) + " (" +
                              std::to_string(ps.listed.size()) + " listed, shm says " + std::to_string(ours.n) + ")";
            }
            moving_send[p].swap(ps.listed);
            const uint32_t n = std::min<uint32_t>(theirs.n, kListMax);
            for (uint32_t i = 0; i < n; ++i) {
                Payload in;
                in.seq = theirs.e[i].seq;
                in.len = (size_t)theirs.e[i].len;
                in.ptr = in.len ? ops->alloc(in.len, &in.hold) : nullptr;
                if (in.len && !in.ptr) {
                    // the landing memory the credit promised is not there:
                    // the peer's group would wait forever, so fail loudly
                    dead_reason = "no memory to land a " + std::to_string(in.len) + " B payload from rank " +
                                  std::to_string(p);
                    break;
                }
                moving_recv[p].push_back(std::move(in));
            }
            ps.round += 1;
            ps.ready = false;
            g_pair_rounds.fetch_add(1, std::memory_order_relaxed);
        }
        uint64_t self_bytes = 0;
        const int self_max = std::max(1, std::min(FLAGS_rccl_round_payloads, 256));
        for (int i = 0; with_self && i < self_max && self_ready_locked(); ++i) {
            const uint64_t len = self_q.front().len;
            if (i > 0 && self_bytes + len > (uint64_t)FLAGS_rccl_round_bytes) break;
            self_bytes += len;
            Payload sp = std::move(self_q.front());
            self_q.pop_front();
            Payload r;
            r.seq = sp.seq;
            r.len = sp.len;
            r.ptr = ops->alloc(sp.len, &r.hold);
            if (!r.ptr) {
                // no memory to land it: the payload is lost (its Recv
                // fails at once) rather than retried every group
                const Key k(rank, sp.seq);
                auto w = waiting.find(k);
                if (w != waiting.end()) {
                    Waiter* wt = w->second.w;
                    waiting.erase(w);
                    finish_locked(wt, false);
                } else {
                    lost[k] = monotonic_us();
                }
                g_withdrawn.fetch_add(1, std::memory_order_relaxed);
                self_bytes -= len;
                continue;
            }
            self_moved += len;
            self_send.push_back(std::move(sp));
            self_recv.push_back(std::move(r));
        }
    }
    std::string dead_reason;

    bool remote_is_shutdown() const { return strcmp(bell->reason, "rank shut down") == 0; }

    std::string remote_reason() const {
        const uint32_t who = bell->abort.load();
        return "rank " + std::to_string((int)who - 1) + " aborted the plane: " + std::string(bell->reason);
    }

    // (mu held) expire unclaimed payloads and stale discard marks
    void housekeeping_locked() {
        const int64_t now = monotonic_us();
        if (now - last_expire_us < 100000) return;
        last_expire_us = now;
        const int64_t ttl = (int64_t)FLAGS_rccl_stash_ttl_ms * 1000;
        for (auto it = stash.begin(); it != stash.end();) {
            if (now - it->second.since_us > ttl) {
                consume_locked(it->first.first, it->second.len);
                g_expired.fetch_add(1, std::memory_order_relaxed);
                it = stash.erase(it);
            } else {
                ++it;
            }
        }
        for (auto it = discards.begin(); it != discards.end();) {
            if (now - it->second > ttl) it = discards.erase(it);
            else ++it;
        }
        for (auto it = lost.begin(); it != lost.end();) {
            if (now - it->second > ttl) it = lost.erase(it);
            else ++it;
        }
    }

    // true when a peer process is gone (the plane is then aborted)
    bool check_liveness() {
        if (world <= 1) return false;
        const int64_t now = monotonic_us();
        if (now - last_liveness_us < 100000) return false;
        last_liveness_us = now;
        for (int q = 0; q < world && q < kMaxRanks; ++q) {
            const int32_t pid = bell->pid[q].load(std::memory_order_acquire);
            if (q != rank && pid > 0 && kill(pid, 0) != 0 && errno == ESRCH) {
                set_remote_abort("rank " + std::to_string(q) + " (pid " + std::to_string(pid) + ") exited");
                return true;
            }
        }
        return false;
    }

    void set_remote_abort(const std::string& why) {
        // the first rank to claim writes the reason, then raises the flag
        uint32_t zero = 0;
        if (bell->claim.compare_exchange_strong(zero, 1)) {
            snprintf(bell->reason, sizeof(bell->reason), "%s", why.c_str());
            bell->abort.store((uint32_t)rank + 1, std::memory_order_release);
        }
        bell->seq.fetch_add(1);
        for (int r = 0; r < world && r < kMaxRanks; ++r) ring(r);
    }

    // Issue the group built under the lock and wait for it. 0 on success;
    // -1 after an abort.
    // Poster only: a group of only self payloads, queued on the stream
    // (one batched copy) and left in flight; reap_self() delivers it.
    int issue_self() {
        std::vector<Segment> segs;
        segs.reserve(self_send.size());
        for (size_t i = 0; i < self_send.size(); ++i)
            segs.push_back(Segment{self_send[i].ptr, self_recv[i].ptr, (uint64_t)self_send[i].len});
        SelfFlight f;
        if (ops->copy(segs) != 0 || ops->record(&f.marker) != 0) {
            abort("self payload copy failed", true);
            return -1;
        }
        f.send.swap(self_send);
        f.recv.swap(self_recv);
        self_flight.push_back(std::move(f));
        g_rounds.fetch_add(1, std::memory_order_relaxed);
        g_payload_rounds.fetch_add(1, std::memory_order_relaxed);
        return 0;
    }

    // Poster only: deliver finished self groups, oldest first; block: wait
    // for all of them (bounded by -rccl_timeout_ms).
    int reap_self(bool block) {
        const int64_t t0 = monotonic_us();
        while (!self_flight.empty()) {
            SelfFlight& f = self_flight.front();
            const int q = ops->query(f.marker);
            if (q < 0) {
                abort("a self payload copy failed on the stream", true);
                return -1;
            }
            if (q == 0) {
                if (!block) return 0;
                const int64_t waited = monotonic_us() - t0;
                if (waited > (int64_t)FLAGS_rccl_timeout_ms * 1000) {
                    abort("a self payload copy made no progress within -rccl_timeout_ms", true);
                    return -1;
                }
                if (waited < FLAGS_rccl_poll_spin_us) {
                    for (int i = 0; i < 64; ++i) __builtin_ia32_pause();
                } else {
                    std::this_thread::yield();
                }
                continue;
            }
            ops->release(f.marker);
            std::vector<Buf> drop;
            {
                std::lock_guard<std::mutex> g(mu);
                for (Payload& sp : f.send) {
                    g_sent.fetch_add(1, std::memory_order_relaxed);
                    g_sent_bytes.fetch_add((int64_t)sp.len, std::memory_order_relaxed);
                    drop.push_back(std::move(sp.hold));
                }
                for (Payload& r : f.recv) deliver_locked(rank, &r);
                housekeeping_locked();  // rate-limited: stash expiry also runs under self-only traffic
            }
            self_flight.pop_front();
        }
        return 0;
    }

    int run_group() {
        if (!dead_reason.empty()) {
            const std::string why = dead_reason;
            dead_reason.clear();
            abort(why, true);
            return -1;
        }
        bool payloads = !self_send.empty();
        for (int p = 0; p < world; ++p) payloads |= !moving_send[p].empty() || !moving_recv[p].empty();
        if (!payloads) return 0;  // fired rounds with nothing to move (both lists empty)
        void* st = ops->stream();
        const int64_t t0 = monotonic_us();
        int rc = 0;
        // self payloads: one batched copy on the plane stream (a send/recv
        // pair to oneself costs RCCL ~16 us of per-op overhead each for
        // what is a device-local copy: the N=1 leg ran ~25 of them per
        // group, 950 us p99)
        const bool self_copy = FLAGS_rccl_self_copy && !self_send.empty();
        if (self_copy) {
            std::vector<Segment> segs;
            segs.reserve(self_send.size());
            for (size_t i = 0; i < self_send.size(); ++i)
                segs.push_back(Segment{self_send[i].ptr, self_recv[i].ptr, (uint64_t)self_send[i].len});
            if (ops->copy(segs) != 0) {
                abort("self payload copy failed", true);
                return -1;
            }
        }
        bool peers_move = false;
        for (int p = 0; p < world; ++p) peers_move |= !moving_send[p].empty() || !moving_recv[p].empty();
        ncclResult_t r = ncclSuccess;
        if (peers_move || !self_copy) r = api.group_start();
        for (int p = 0; p < world && r == ncclSuccess; ++p) {
            if (p == rank) continue;
            for (size_t i = 0; i < moving_send[p].size() && r == ncclSuccess; ++i)
                r = api.send(moving_send[p][i].ptr, moving_send[p][i].len, ncclUint8, p, comm, (hipStream_t)st);
            for (size_t i = 0; i < moving_recv[p].size() && r == ncclSuccess; ++i)
                r = api.recv(moving_recv[p][i].ptr, moving_recv[p][i].len, ncclUint8, p, comm, (hipStream_t)st);
        }
        for (size_t i = 0; !self_copy && i < self_send.size() && r == ncclSuccess; ++i) {
            r = api.send(self_send[i].ptr, self_send[i].len, ncclUint8, rank, comm, (hipStream_t)st);
            if (r == ncclSuccess)
                r = api.recv(self_recv[i].ptr, self_recv[i].len, ncclUint8, rank, comm, (hipStream_t)st);
        }
        if (peers_move || !self_copy) {
            const ncclResult_t e = api.group_end();
            if (r == ncclSuccess) r = e;
        }
        if (r == ncclSuccess) rc = ops->record(&marker);
        marker_live = r == ncclSuccess && rc == 0;
        g_rounds.fetch_add(1, std::memory_order_relaxed);
        g_payload_rounds.fetch_add(1, std::memory_order_relaxed);
        if (r != ncclSuccess || rc != 0) {
            abort(r != ncclSuccess ? std::string("group issue: ") + api.error_string(r) : "group issue: stream op failed",
                  true);
            return -1;
        }
        // wait: the poster polls (briefly spinning, then napping) and keeps
        // an eye on the abort flag, the peers and the watchdog
        int spins = 0;
        for (;;) {
            const int q = ops->query(marker);
            if (q == 1) break;
            if (q < 0) {
                abort("a plane group failed on the stream", true);
                return -1;
            }
            if (bell->abort.load(std::memory_order_acquire)) {
                abort(remote_reason(), false);
                return -1;
            }
            ncclResult_t ae = ncclSuccess;
            api.async_error(comm, &ae);
            if (ae != ncclSuccess && ae != ncclInProgress) {
                abort(std::string("rccl: ") + api.error_string(ae), true);
                return -1;
            }
            const int64_t now = monotonic_us();
            if (now - t0 > (int64_t)FLAGS_rccl_timeout_ms * 1000) {
                abort("a plane group made no progress within -rccl_timeout_ms", true);
                return -1;
            }
            if (check_liveness()) {
                abort(std::string(bell->reason), false);
                return -1;
            }
            if (now - t0 < FLAGS_rccl_poll_spin_us) {
                for (int i = 0; i < 64; ++i) __builtin_ia32_pause();
            } else if (++spins < 200) {
                std::this_thread::yield();
            } else {
                usleep(20);
            }
        }
        ops->release(marker);
        marker_live = false;
        g_group_us.fetch_add(monotonic_us() - t0, std::memory_order_relaxed);
        complete_group();
        return 0;
    }

    void complete_group() {
        std::vector<Buf> drop;  // released outside the lock
        std::lock_guard<std::mutex> g(mu);
        for (int p = 0; p < world; ++p) {
            for (Payload& s : moving_send[p]) {
                g_sent.fetch_add(1, std::memory_order_relaxed);
                g_sent_bytes.fetch_add((int64_t)s.len, std::memory_order_relaxed);
                drop.push_back(std::move(s.hold));
            }
            for (Payload& r : moving_recv[p]) deliver_locked(p, &r);
        }
        for (Payload& s : self_send) {
            g_sent.fetch_add(1, std::memory_order_relaxed);
            g_sent_bytes.fetch_add((int64_t)s.len, std::memory_order_relaxed);
            drop.push_back(std::move(s.hold));
        }
        for (Payload& r : self_recv) deliver_locked(rank, &r);
        moving_send.assign(world, {});
        moving_recv.assign(world, {});
        self_send.clear();
        self_recv.clear();
        housekeeping_locked();
    }

    // (mu held) a payload from `src` landed
    void deliver_locked(int src, Payload* r) {
        g_recv.fetch_add(1, std::memory_order_relaxed);
        g_recv_bytes.fetch_add((int64_t)r->len, std::memory_order_relaxed);
        const Key k(src, r->seq);
        auto w = waiting.find(k);
        if (w != waiting.end()) {
            *w->second.out = std::move(r->hold);
            consume_locked(src, r->len);
            Waiter* wt = w->second.w;
            waiting.erase(w);
            finish_locked(wt, true);
            return;
        }
        auto d = discards.find(k);
        if (d != discards.end()) {
            discards.erase(d);
            consume_locked(src, r->len);
            g_discarded.fetch_add(1, std::memory_order_relaxed);
            r->hold.clear();
            return;
        }
        Stashed& s = stash[k];
        s.buf = std::move(r->hold);
        s.len = r->len;
        s.since_us = monotonic_us();
    }

    // Poster only. Tell the other ranks (propagate), abort the communicator,
    // wait (bounded) for the stream so no kernel still reads or writes our
    // blocks, then fail everything that waits on the plane.
    void abort(const std::string& why, bool propagate, bool is_error = true) {
        {
            std::lock_guard<std::mutex> g(mu);
            if (dead) return;
            dead = true;
            dead_flag.store(true, std::memory_order_release);
        }
        if (is_error) {
            LOG(ERROR) << "rccl plane aborted on rank " << rank << ": " << why
                       << " (payloads fall back to xGMI lending)";
            g_aborts.fetch_add(1, std::memory_order_relaxed);
        } else {
            LOG(INFO) << "rccl plane closed on rank " << rank << ": " << why;
        }
        if (propagate && world > 1) set_remote_abort(why);
        if (comm) api.comm_abort(comm);
        bool drained = true;
        if (marker_live) {
            drained = false;
            const int64_t t0 = monotonic_us();
            while (monotonic_us() - t0 < 2000000) {
                const int q = ops->query(marker);
                if (q != 0) {
                    drained = true;
                    break;
                }
                usleep(100);
            }
            if (drained) ops->release(marker);
            marker_live = false;
        }
        // self groups still on the stream: wait (bounded) for their copies
        bool self_drained = true;
        for (SelfFlight& f : self_flight) {
            const int64_t t1 = monotonic_us();
            int q = 0;
            while ((q = ops->query(f.marker)) == 0 && monotonic_us() - t1 < 2000000) usleep(100);
            if (q != 0) ops->release(f.marker);
            else self_drained = false;
        }
        std::vector<Buf> bufs;
        std::lock_guard<std::mutex> g(mu);
        auto take = [&](std::vector<Payload>& v) {
            for (Payload& p : v) bufs.push_back(std::move(p.hold));
            v.clear();
        };
        for (SelfFlight& f : self_flight) {
            // their receivers fail below (waiting); the blocks may still be
            // written by a copy that did not drain: keep them out of reuse
            std::vector<Buf> fb;
            for (Payload& p : f.send) fb.push_back(std::move(p.hold));
            for (Payload& p : f.recv) fb.push_back(std::move(p.hold));
            for (Buf& b : fb) (self_drained ? bufs : graveyard).push_back(std::move(b));
        }
        self_flight.clear();
        for (auto& v : moving_send) take(v);
        for (auto& v : moving_recv) take(v);
        take(self_send);
        take(self_recv);
        if (!drained) {
            LOG(ERROR) << "rccl plane: stream did not drain after the abort; " << bufs.size()
                       << " in-flight blocks are leaked, not recycled";
            for (Buf& b : bufs) graveyard.push_back(std::move(b));
            bufs.clear();
        }
        for (PeerState& ps : peers) {
            for (Payload& p : ps.queued) bufs.push_back(std::move(p.hold));
            ps.queued.clear();
            take(ps.listed);
        }
        for (Payload& p : self_q) bufs.push_back(std::move(p.hold));
        self_q.clear();
        stash.clear();
        discards.clear();
        for (auto& kv : waiting) finish_locked(kv.second.w, false);
        waiting.clear();
        if (!bell_name.empty()) shm_unlink(bell_name.c_str());
    }

    // Collective, at Init: one group in which every rank exchanges 8 bytes
    // with every peer, so RCCL connects every pair before traffic (it
    // connects p2p peers lazily inside the first group that uses them).
    int warm_up() {
        Buf scratch;
        char* b = static_cast<char*>(ops->alloc((size_t)16 * world, &scratch));
        if (!b) return -1;
        void* st = ops->stream();
        ncclResult_t r = api.group_start();
        for (int p = 0; p < world && r == ncclSuccess; ++p) {
            if (p == rank) continue;
            r = api.send(b + 16 * p, 8, ncclUint8, p, comm, (hipStream_t)st);
            if (r == ncclSuccess) r = api.recv(b + 16 * p + 8, 8, ncclUint8, p, comm, (hipStream_t)st);
        }
        const ncclResult_t e = api.group_end();
        if (r == ncclSuccess) r = e;
        if (r != ncclSuccess || ops->record(&marker) != 0) return -1;
        const int64_t t0 = monotonic_us();
        for (;;) {
            const int q = ops->query(marker);
            if (q == 1) break;
            if (q < 0 || monotonic_us() - t0 > (int64_t)FLAGS_rccl_timeout_ms * 1000) return -1;
            usleep(50);
        }
        ops->release(marker);
        return 0;
    }
};

std::mutex g_mu;
Plane* g_plane = nullptr;
std::atomic<bool> g_active{false};

Doorbell* open_bell(const std::string& name, bool shared) {
    if (!shared) {
        void* m = calloc(1, sizeof(Doorbell));
        if (!m) return nullptr;
        Doorbell* b = static_cast<Doorbell*>(m);
        b->magic = kBellMagic;
        return b;
    }
    const int fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0) return nullptr;
    if (ftruncate(fd, (off_t)sizeof(Doorbell)) != 0) {
        close(fd);
        return nullptr;
    }
    void* m = mmap(nullptr, sizeof(Doorbell), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return nullptr;
    Doorbell* b = static_cast<Doorbell*>(m);
    b->magic = kBellMagic;  // every rank writes the same value
    return b;
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
        if (g_plane->id == fnv1a(unique_id) && g_plane->rank == rank && !g_plane->dead_flag.load()) return 0;
        if (error) *error = "another RCCL plane was set up in this process";
        return -1;
    }
    if (world <= 0 || world > kMaxRanks || rank < 0 || rank >= world || unique_id.size() != sizeof(ncclUniqueId)) {
        if (error) *error = "bad rank/world/unique id (at most " + std::to_string(kMaxRanks) + " ranks per node)";
        return -1;
    }
    std::unique_ptr<Plane> p(new Plane);
    if (!load_api(&p->api, error)) return -1;
    if (p->api.fake()) {
        p->ops.reset(new StubOps(p->api));
    } else {
        if (device < 0) device = CurrentDevice();
        if (gpu::Init(device, error) != 0 || InitHbmPool(device, error) != 0) return -1;
        p->ops.reset(new HipOps);
    }
    p->device = device;
    p->rank = rank;
    p->world = world;
    p->id = fnv1a(unique_id);
    int prev = 0;
    if (!p->api.fake()) hipGetDevice(&prev);
    if (p->ops->init(device, error) != 0) {
        if (!p->api.fake()) hipSetDevice(prev);
        return -1;
    }
    char nb[64];
    snprintf(nb, sizeof(nb), "/mrpc_rccl_bell_%016llx", (unsigned long long)p->id);
    if (world > 1) p->bell_name = nb;
    p->bell = open_bell(nb, world > 1);
    if (!p->bell) {
        if (error) *error = "doorbell shm unavailable";
        return -1;
    }
    p->bell->pid[rank].store(getpid(), std::memory_order_release);
    if (!p->api.fake()) hipSetDevice(device);
    ncclUniqueId id;
    memcpy(id.internal, unique_id.data(), sizeof(id.internal));
    ncclResult_t r = p->api.comm_init_rank(&p->comm, world, id, rank);
    if (r != ncclSuccess) {
        if (!p->api.fake()) hipSetDevice(prev);
        if (error) *error = std::string("ncclCommInitRank: ") + p->api.error_string(r);
        return -1;
    }
    p->peers.assign(world, PeerState());
    p->moving_send.assign(world, {});
    p->moving_recv.assign(world, {});
    const int rc = world > 1 ? p->warm_up() : 0;
    if (!p->api.fake()) hipSetDevice(prev);
    if (rc != 0) {
        if (error) *error = "rccl plane: the warm-up group failed";
        if (!p->bell_name.empty()) shm_unlink(p->bell_name.c_str());
        p.release();  // its comm may still be referenced by the stream
        return -1;
    }
    Plane* raw = p.release();
    raw->poster = std::thread([raw] { raw->run(); });
    g_plane = raw;
    g_active.store(true, std::memory_order_release);
    static var::PassiveStatus<int64_t> v1("rccl_sent_bytes", [] { return g_sent_bytes.load(); });
    static var::PassiveStatus<int64_t> v2("rccl_recv_bytes", [] { return g_recv_bytes.load(); });
    static var::PassiveStatus<int64_t> v3("rccl_rounds", [] { return g_rounds.load(); });
    static var::PassiveStatus<int64_t> v4("rccl_aborts", [] { return g_aborts.load(); });
    static var::PassiveStatus<int64_t> v5("rccl_credit_stalls", [] { return g_credit_stalls.load(); });
    static var::PassiveStatus<int64_t> v6("rccl_pair_rounds", [] { return g_pair_rounds.load(); });
    LOG(INFO) << "rccl plane up: rank " << rank << "/" << world
              << (raw->api.fake() ? " on the stub library (host memory)" : " on device " + std::to_string(device));
    return 0;
}

bool Active() {
    return g_active.load(std::memory_order_acquire) && !g_plane->dead_flag.load(std::memory_order_acquire);
}
int Rank() { return g_active.load(std::memory_order_acquire) ? g_plane->rank : -1; }
int World() { return g_active.load(std::memory_order_acquire) ? g_plane->world : 0; }
uint64_t PlaneId() { return g_active.load(std::memory_order_acquire) ? g_plane->id : 0; }
bool HostMemory() { return g_active.load(std::memory_order_acquire) && g_plane->ops->host_memory(); }
bool AcceptsBlock(const BufBlock* b) { return Active() && g_plane->ops->accepts(b); }

void Shutdown() {
    std::lock_guard<std::mutex> g(g_mu);
    if (!g_plane) return;
    {
        std::lock_guard<std::mutex> lk(g_plane->mu);
        g_plane->stop = true;
    }
    g_plane->ring(g_plane->rank);
    if (g_plane->poster.joinable()) g_plane->poster.join();
    // the plane object stays (Active() is false from now on): late callers
    // may still hold a pointer to it
}

bool FillHello(policy::PlaneHello* h) {
    if (!Active()) return false;
    h->set_rank(g_plane->rank);
    h->set_plane(g_plane->id);
    h->set_pid(getpid());
    return true;
}

int PeerRank(const policy::PlaneHello& h) {
    if (!Active() || h.plane() != g_plane->id || h.rank() < 0 || h.rank() >= g_plane->world) return -1;
    return h.rank();
}

int64_t Send(int peer, const void* p, size_t len, Buf&& hold) {
    if (!Active() || len == 0) return -1;
    return g_plane->send(peer, p, len, std::move(hold));
}

int Recv(int n, const int* src, const uint64_t* seq, const size_t* len, Buf* outs) {
    if (n <= 0) return 0;
    if (!g_active.load(std::memory_order_acquire)) return -1;
    return g_plane->recv(n, src, seq, len, outs);
}

void Discard(int src, uint64_t seq, size_t len) {
    if (!g_active.load(std::memory_order_acquire)) return;
    g_plane->discard(src, seq, len);
}

void Cancelled(int peer, uint64_t seq) {
    if (!g_active.load(std::memory_order_acquire)) return;
    g_plane->cancelled(peer, seq);
}

void AbortForTest(const std::string& why) {
    std::lock_guard<std::mutex> g(g_mu);
    if (!g_plane) return;
    g_plane->set_remote_abort(why);
}

Stats GetStats() {
    Stats s;
    s.sent_payloads = g_sent.load();
    s.sent_bytes = g_sent_bytes.load();
    s.recv_payloads = g_recv.load();
    s.recv_bytes = g_recv_bytes.load();
    s.discarded = g_discarded.load();
    s.rounds = g_rounds.load();
    s.payload_rounds = g_payload_rounds.load();
    s.pair_rounds = g_pair_rounds.load();
    s.withdrawals = g_withdrawals.load();
    s.group_us = g_group_us.load();
    s.aborts = g_aborts.load();
    s.credit_stalls = g_credit_stalls.load();
    s.stash_expired = g_expired.load();
    s.recv_timeouts = g_recv_timeouts.load();
    s.doorbells = g_doorbells.load();
    s.withdrawn = g_withdrawn.load();
    {
        std::lock_guard<std::mutex> g(g_mu);
        if (g_plane) {
            std::lock_guard<std::mutex> lk(g_plane->mu);
            s.stash_payloads = (int64_t)g_plane->stash.size();
            for (const auto& kv : g_plane->stash) s.stash_bytes += (int64_t)kv.second.len;
        }
    }
    s.world = World();
    s.host_memory = HostMemory();
    return s;
}

}  // namespace rccl
}  // namespace gpu
}  // namespace mrpc
