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
#include "mrpc/proto/device_payload.pb.h"
#include "var/var.h"

DEFINE_int32(rccl_timeout_ms, 10000,
             "abort the plane when a round made no progress for this long (and fail Recv waits older than this)");
DEFINE_string(rccl_library, "",
              "RCCL library the plane dlopens (empty: the librccl.so the process has, else ROCm's); "
              "the stub build/lib/libfake_rccl.so runs the plane on CPU hosts");
DEFINE_int64(rccl_window_bytes, int64_t(256) << 20,
             "receiver credit per source rank: payload bytes a peer may announce beyond what this rank consumed");
DEFINE_int32(rccl_round_payloads, 64, "most payloads announced to one peer per round");
DEFINE_int64(rccl_round_bytes, int64_t(64) << 20, "most payload bytes announced to one peer per round");
DEFINE_int32(rccl_stash_ttl_ms, 30000, "received payloads nobody claims are dropped after this long");
DEFINE_int32(rccl_idle_spin_us, 0, "an idle plane poster watches its doorbell this long before sleeping");

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
    int (*fake_stream_memcpy)(void*, void*, const void*, size_t) = nullptr;
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
        a->fake_stream_memcpy =
            reinterpret_cast<int (*)(void*, void*, const void*, size_t)>(dlsym(lib, "mrpcfake_stream_memcpy"));
        a->fake_stream_record = reinterpret_cast<uint64_t (*)(void*)>(dlsym(lib, "mrpcfake_stream_record"));
        a->fake_stream_query = reinterpret_cast<int (*)(void*, uint64_t)>(dlsym(lib, "mrpcfake_stream_query"));
        if (!a->fake_stream_create || !a->fake_stream_memcpy || !a->fake_stream_record || !a->fake_stream_query) {
            if (err) *err = "stub rccl library lacks its mrpcfake_stream_* functions";
            return false;
        }
    }
    return true;
}

// ------------------------------------------------------------------ streams
// The stream-ordered work of a round: header upload, the group, header
// download, a completion marker. HIP on MI355X; the stub's executor on CPU.
class StreamOps {
public:
    virtual ~StreamOps() {}
    virtual int init(int device, size_t hdr_bytes, std::string* err) = 0;
    virtual void* stream() = 0;
    // header buffers: host_out -> dev_out before the group, dev_in -> host_in after
    char* host_out = nullptr;
    char* host_in = nullptr;
    char* dev_out = nullptr;
    char* dev_in = nullptr;
    virtual int upload(size_t n) = 0;
    virtual int download(size_t n) = 0;
    virtual int record(uint64_t* marker) = 0;
    // 1 complete, 0 pending, -1 failed
    virtual int query(uint64_t marker) = 0;
    virtual void release(uint64_t marker) = 0;
    virtual void* alloc(size_t len, Buf* out) = 0;
    virtual bool accepts(const BufBlock* b) const = 0;
    virtual bool host_memory() const = 0;
};

class HipOps : public StreamOps {
public:
    int init(int device, size_t hdr_bytes, std::string* err) override {
        _device = device;
        hipSetDevice(device);
        if (hipStreamCreateWithFlags(&_stream, hipStreamNonBlocking) != hipSuccess) {
            if (err) *err = "hipStreamCreate failed";
            return -1;
        }
        void* d = nullptr;
        void* h = nullptr;
        if (hipMalloc(&d, 2 * hdr_bytes) != hipSuccess || hipHostMalloc(&h, 2 * hdr_bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
            if (err) *err = "header buffers: allocation failed";
            return -1;
        }
        memset(h, 0, 2 * hdr_bytes);
        dev_out = static_cast<char*>(d);
        dev_in = dev_out + hdr_bytes;
        host_out = static_cast<char*>(h);
        host_in = host_out + hdr_bytes;
        return 0;
    }
    void* stream() override { return _stream; }
    int upload(size_t n) override {
        return hipMemcpyAsync(dev_out, host_out, n, hipMemcpyHostToDevice, _stream) == hipSuccess ? 0 : -1;
    }
    int download(size_t n) override {
        return hipMemcpyAsync(host_in, dev_in, n, hipMemcpyDeviceToHost, _stream) == hipSuccess ? 0 : -1;
    }
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

private:
    int _device = -1;
    hipStream_t _stream = nullptr;
};

void free_host(void* p, void*) { free(p); }

class StubOps : public StreamOps {
public:
    explicit StubOps(const Api& a) : _api(a) {}
    int init(int, size_t hdr_bytes, std::string* err) override {
        _stream = _api.fake_stream_create();
        char* b = static_cast<char*>(calloc(4, hdr_bytes));
        if (!_stream || !b) {
            if (err) *err = "stub stream creation failed";
            return -1;
        }
        host_out = b;
        host_in = b + hdr_bytes;
        dev_out = b + 2 * hdr_bytes;
        dev_in = b + 3 * hdr_bytes;
        return 0;
    }
    void* stream() override { return _stream; }
    int upload(size_t n) override { return _api.fake_stream_memcpy(_stream, dev_out, host_out, n); }
    int download(size_t n) override { return _api.fake_stream_memcpy(_stream, host_in, dev_in, n); }
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

private:
    const Api& _api;
    void* _stream = nullptr;
};

// ------------------------------------------------------------------ wire
const uint64_t kHdrMagic = 0x4d5250435244484full;  // "MRPCRDHO"
const size_t kHdrBytes = 4096;
const uint32_t kBusy = 1;

struct HdrEntry {
    uint64_t seq;
    uint64_t len;
};
struct Hdr {
    uint64_t magic;
    uint64_t round;
    uint64_t credit;   // cumulative bytes the receiver (sender of this header) accepts from us
    uint32_t n;
    uint32_t flags;
    uint64_t from;
    uint64_t reserved[3];
    HdrEntry e[(kHdrBytes - 64) / sizeof(HdrEntry)];
};
static_assert(sizeof(Hdr) == kHdrBytes, "round header must be fixed-size");
const int kMaxEntries = (int)((kHdrBytes - 64) / sizeof(HdrEntry));

// The node's doorbell: POSIX shm shared by the ranks of the plane (a
// private allocation for a one-rank plane).
const uint64_t kBellMagic = 0x4d52504342454c4cull;  // "MRPCBELL"
const int kMaxRanks = 64;
struct Doorbell {
    uint64_t magic;
    std::atomic<uint64_t> want_round;
    std::atomic<uint32_t> seq;     // futex word: bumped on every ring / abort
    std::atomic<uint32_t> claim;   // the first aborting rank claims the reason slot
    std::atomic<uint32_t> abort;   // 0, or 1 + the rank that aborted first
    char reason[200];
    std::atomic<int32_t> pid[kMaxRanks];
};

long futex(std::atomic<uint32_t>* w, int op, uint32_t val, const timespec* ts) {
    return syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), op, val, ts, nullptr, 0);
}

uint64_t fnv1a(const std::string& s) {
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
    return h | 1;  // never 0: 0 means "no plane" in the hello
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
    std::deque<Payload> queued;       // not announced yet
    std::vector<Payload> announced;   // announced in the last header: move next round
    std::vector<Payload> incoming;    // from the peer's last header: receive next round
    uint64_t next_seq = 0;
    uint64_t announced_bytes = 0;     // cumulative, to this peer
    uint64_t credit = 0;              // cumulative, granted by this peer
    uint64_t consumed = 0;            // cumulative, from this peer (claimed/dropped)
    std::vector<uint64_t> cancels;    // announced to this peer, then cancelled: tell it to drop them
};

// A header entry with this length cancels an earlier announcement of its
// sequence (the receiver drops the payload instead of stashing it).
const uint64_t kCancelLen = ~0ull;

std::atomic<int64_t> g_sent{0}, g_sent_bytes{0}, g_recv{0}, g_recv_bytes{0}, g_discarded{0}, g_rounds{0},
    g_payload_rounds{0}, g_aborts{0}, g_credit_stalls{0}, g_expired{0}, g_recv_timeouts{0}, g_doorbells{0},
    g_withdrawn{0};

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
    std::deque<Payload> self_q;
    std::map<Key, Stashed> stash;
    std::map<Key, WaitSlot> waiting;
    std::map<Key, int64_t> discards;
    std::map<Key, int64_t> lost;   // self payloads that found no memory to land in: their Recv fails
    uint64_t self_moved = 0;       // cumulative self bytes landed (credit: vs peers[rank].consumed)
    bool idle = false, dead = false, stop = false;
    bool busy_next = false;        // some rank's round header asked for another round
    uint64_t completed_round = 0;  // poster only (read under mu by Send)
    std::atomic<bool> dead_flag{false};
    std::thread poster;
    int64_t last_expire_us = 0, last_liveness_us = 0;

    // the round in flight (poster only)
    std::vector<std::vector<Payload>> moving_send, moving_recv;
    std::vector<Payload> self_send, self_recv;
    uint64_t marker = 0;
    bool marker_live = false;
    std::vector<Buf> graveyard;  // blocks RCCL may still touch after an abort

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
        if (idle) ring_locked();
        return seq;
    }

    void ring_locked() {
        uint64_t want = completed_round + 1, cur = bell->want_round.load();
        while (cur < want && !bell->want_round.compare_exchange_weak(cur, want)) {
        }
        bell->seq.fetch_add(1);
        futex(&bell->seq, FUTEX_WAKE, INT_MAX, nullptr);
        idle = false;
        g_doorbells.fetch_add(1, std::memory_order_relaxed);
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

    void consume_locked(int src, size_t len) { peers[src].consumed += len; }

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
        // already announced. To ourselves: drop it here (now or when it
        // lands). To a peer: the next round header tells it to.
        if (peer == rank) {
            Buf dropped;
            discard_locked(rank, seq, &dropped);
            drop.append(std::move(dropped));
        } else {
            peers[peer].cancels.push_back(seq);
        }
        g_withdrawn.fetch_add(1, std::memory_order_relaxed);
    }

    // ---------------------------------------------------------------- poster
    void run() {
        if (!ops->host_memory()) hipSetDevice(device);
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                for (;;) {
                    if (stop || dead) break;
                    if (bell->abort.load(std::memory_order_acquire)) break;
                    const bool local = !self_q.empty() || any_queued_locked();
                    const uint64_t want = bell->want_round.load(std::memory_order_acquire);
                    if (busy_next || want > completed_round) break;
                    if (local) {
                        ring_locked();  // the other ranks learn about round k+1 from the doorbell
                        break;
                    }
                    idle = true;
                    const uint32_t s = bell->seq.load(std::memory_order_acquire);
                    housekeeping_locked();
                    lk.unlock();
                    // watch the doorbell a little while before sleeping: the
                    // next payload of a busy stream is usually close behind
                    const int64_t until = monotonic_us() + std::max(0, FLAGS_rccl_idle_spin_us);
                    while (bell->seq.load(std::memory_order_acquire) == s && monotonic_us() < until) {
                        for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
                    }
                    timespec ts{0, 50 * 1000 * 1000};
                    futex(&bell->seq, FUTEX_WAIT, s, &ts);
                    lk.lock();
                    if (check_liveness()) break;
                }
                idle = false;
                if (stop) break;
            }
            if (bell->abort.load(std::memory_order_acquire)) {
                abort(remote_reason(), false, !remote_is_shutdown());
                break;
            }
            if (dead) break;
            if (run_round(completed_round + 1) != 0) break;
        }
        if (!dead) abort("rank shut down", true, /*is_error=*/false);
    }

    bool any_queued_locked() const {
        for (const PeerState& p : peers)
            if (!p.queued.empty()) return true;
        return false;
    }

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
        futex(&bell->seq, FUTEX_WAKE, INT_MAX, nullptr);
    }

    // Build, issue and complete round k. 0 on success; -1 after an abort.
    int run_round(uint64_t k) {
        bool my_busy = false, stalled = false;
        {
            std::lock_guard<std::mutex> g(mu);
            moving_send.assign(world, {});
            moving_recv.assign(world, {});
            for (int p = 0; p < world; ++p) {
                if (p == rank) continue;
                PeerState& ps = peers[p];
                Hdr* h = reinterpret_cast<Hdr*>(ops->host_out + (size_t)p * kHdrBytes);
                h->magic = kHdrMagic;
                h->round = k;
                h->credit = ps.consumed + (uint64_t)std::max<int64_t>(FLAGS_rccl_window_bytes, 1);
                h->from = (uint64_t)rank;
                h->n = 0;
                moving_send[p].swap(ps.announced);
                moving_recv[p].swap(ps.incoming);
                uint64_t round_bytes = 0;
                const int max_n = std::max(1, std::min(FLAGS_rccl_round_payloads, kMaxEntries));
                while (!ps.queued.empty() && (int)h->n < max_n) {
                    const Payload& q = ps.queued.front();
                    if (h->n > 0 && round_bytes + q.len > (uint64_t)FLAGS_rccl_round_bytes) break;
                    // within credit, or the peer consumed everything we announced
                    const uint64_t granted = ps.credit;
                    const uint64_t window = (uint64_t)std::max<int64_t>(FLAGS_rccl_window_bytes, 1);
                    const bool drained = granted >= window && ps.announced_bytes <= granted - window;
                    if (ps.announced_bytes + q.len > granted && !drained) {
                        stalled = true;
                        break;
                    }
                    h->e[h->n].seq = q.seq;
                    h->e[h->n].len = q.len;
                    ++h->n;
                    round_bytes += q.len;
                    ps.announced_bytes += q.len;
                    ps.announced.push_back(std::move(ps.queued.front()));
                    ps.queued.pop_front();
                }
                // cancellations of earlier announcements ride in the same entries
                size_t nc = 0;
                while (nc < ps.cancels.size() && (int)h->n < kMaxEntries) {
                    h->e[h->n].seq = ps.cancels[nc++];
                    h->e[h->n].len = kCancelLen;
                    ++h->n;
                }
                ps.cancels.erase(ps.cancels.begin(), ps.cancels.begin() + (long)nc);
                my_busy |= !ps.announced.empty() || !ps.queued.empty() || !ps.cancels.empty();
            }
            self_send.clear();
            self_recv.clear();
            // self pairs: no credit (the stash is ours) but the same per-round
            // byte bound as a peer's announcements, so a burst of large
            // payloads does not land all at once
            uint64_t self_bytes = 0;
            const int self_max = std::max(1, std::min(FLAGS_rccl_round_payloads, 256));
            const uint64_t window = (uint64_t)std::max<int64_t>(FLAGS_rccl_window_bytes, 1);
            for (int i = 0; i < self_max && !self_q.empty(); ++i) {
                const uint64_t len = self_q.front().len;
                if (i > 0 && self_bytes + len > (uint64_t)FLAGS_rccl_round_bytes) break;
                // the same window a peer grants: landed-but-unclaimed self
                // bytes stay under -rccl_window_bytes
                const uint64_t unclaimed = self_moved - peers[rank].consumed;
                if (unclaimed > 0 && unclaimed + len > window) {
                    stalled = true;
                    break;
                }
                self_bytes += len;
                Payload s = std::move(self_q.front());
                self_q.pop_front();
                Payload r;
                r.seq = s.seq;
                r.len = s.len;
                r.ptr = ops->alloc(s.len, &r.hold);
                if (!r.ptr) {
                    // no memory to land it: the payload is lost (its Recv
                    // fails at once) rather than retried every round
                    const Key k(rank, s.seq);
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
                self_send.push_back(std::move(s));
                self_recv.push_back(std::move(r));
            }
            my_busy |= !self_q.empty();
            for (int p = 0; p < world; ++p) {
                if (p == rank) continue;
                reinterpret_cast<Hdr*>(ops->host_out + (size_t)p * kHdrBytes)->flags = my_busy ? kBusy : 0;
            }
        }
        if (stalled) g_credit_stalls.fetch_add(1, std::memory_order_relaxed);
        bool payloads = !self_send.empty();
        for (int p = 0; p < world; ++p) payloads |= !moving_send[p].empty() || !moving_recv[p].empty();

        // issue: headers up, one group, headers down, one marker
        void* st = ops->stream();
        const size_t hdr_total = (size_t)world * kHdrBytes;
        int rc = world > 1 ? ops->upload(hdr_total) : 0;
        ncclResult_t r = ncclSuccess;
        if (rc == 0) {
            r = api.group_start();
            for (int p = 0; p < world && r == ncclSuccess; ++p) {
                if (p == rank) continue;
                r = api.send(ops->dev_out + (size_t)p * kHdrBytes, kHdrBytes, ncclUint8, p, comm, (hipStream_t)st);
                if (r == ncclSuccess)
                    r = api.recv(ops->dev_in + (size_t)p * kHdrBytes, kHdrBytes, ncclUint8, p, comm, (hipStream_t)st);
                for (size_t i = 0; i < moving_send[p].size() && r == ncclSuccess; ++i)
                    r = api.send(moving_send[p][i].ptr, moving_send[p][i].len, ncclUint8, p, comm, (hipStream_t)st);
                for (size_t i = 0; i < moving_recv[p].size() && r == ncclSuccess; ++i)
                    r = api.recv(moving_recv[p][i].ptr, moving_recv[p][i].len, ncclUint8, p, comm, (hipStream_t)st);
            }
            for (size_t i = 0; i < self_send.size() && r == ncclSuccess; ++i) {
                r = api.send(self_send[i].ptr, self_send[i].len, ncclUint8, rank, comm, (hipStream_t)st);
                if (r == ncclSuccess)
                    r = api.recv(self_recv[i].ptr, self_recv[i].len, ncclUint8, rank, comm, (hipStream_t)st);
            }
            const ncclResult_t e = api.group_end();
            if (r == ncclSuccess) r = e;
            if (r == ncclSuccess && world > 1) rc = ops->download(hdr_total);
            if (r == ncclSuccess && rc == 0) rc = ops->record(&marker);
            marker_live = r == ncclSuccess && rc == 0;
        }
        g_rounds.fetch_add(1, std::memory_order_relaxed);
        if (payloads) g_payload_rounds.fetch_add(1, std::memory_order_relaxed);
        if (r != ncclSuccess || rc != 0) {
            abort(r != ncclSuccess ? std::string("round issue: ") + api.error_string(r) : "round issue: stream op failed",
                  true);
            return -1;
        }
        // wait: the poster polls (briefly spinning, then napping) and keeps
        // an eye on the doorbell, the peers and the watchdog
        const int64_t t0 = monotonic_us();
        int spins = 0;
        for (;;) {
            const int q = ops->query(marker);
            if (q == 1) break;
            if (q < 0) {
                abort("round " + std::to_string(k) + " failed on the stream", true);
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
                abort("round " + std::to_string(k) + " made no progress within -rccl_timeout_ms", true);
                return -1;
            }
            if (check_liveness()) {
                abort(std::string(bell->reason), false);
                return -1;
            }
            if (++spins < 200) std::this_thread::yield();
            else usleep(20);
        }
        ops->release(marker);
        marker_live = false;
        const int rc2 = complete_round(k, my_busy);
        // nothing could move for want of credit: give the receivers a moment
        // to consume instead of spinning empty rounds
        if (rc2 == 0 && stalled && !payloads) usleep(50);
        return rc2;
    }

    int complete_round(uint64_t k, bool my_busy) {
        std::vector<Buf> drop;  // released outside the lock
        Buf drop_cancelled;
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
        bool busy = my_busy;
        for (int p = 0; p < world; ++p) {
            if (p == rank) continue;
            const Hdr* h = reinterpret_cast<const Hdr*>(ops->host_in + (size_t)p * kHdrBytes);
            if (h->magic != kHdrMagic || h->round != k || h->from != (uint64_t)p || h->n > (uint32_t)kMaxEntries) {
                mu.unlock();
                abort("round " + std::to_string(k) + ": bad header from rank " + std::to_string(p), true);
                mu.lock();
                return -1;
            }
            PeerState& ps = peers[p];
            ps.credit = std::max(ps.credit, h->credit);
            busy |= (h->flags & kBusy) != 0;
            for (uint32_t i = 0; i < h->n; ++i) {
                if (h->e[i].len == kCancelLen) {  // the sender gave this payload up
                    discard_locked(p, h->e[i].seq, &drop_cancelled);
                    continue;
                }
                Payload in;
                in.seq = h->e[i].seq;
                in.len = (size_t)h->e[i].len;
                in.ptr = in.len ? ops->alloc(in.len, &in.hold) : nullptr;
                if (!in.ptr) {
                    mu.unlock();
                    abort("no memory to land a " + std::to_string(in.len) + " B payload from rank " +
                              std::to_string(p),
                          true);
                    mu.lock();
                    return -1;
                }
                ps.incoming.push_back(std::move(in));
            }
        }
        busy_next = busy;
        completed_round = k;
        housekeeping_locked();
        return 0;
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
        std::vector<Buf> bufs;
        std::lock_guard<std::mutex> g(mu);
        auto take = [&](std::vector<Payload>& v) {
            for (Payload& p : v) bufs.push_back(std::move(p.hold));
            v.clear();
        };
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
            take(ps.announced);
            take(ps.incoming);
        }
        for (Payload& p : self_q) bufs.push_back(std::move(p.hold));
        self_q.clear();
        stash.clear();
        discards.clear();
        for (auto& kv : waiting) finish_locked(kv.second.w, false);
        waiting.clear();
        if (!bell_name.empty()) shm_unlink(bell_name.c_str());
    }
};

std::mutex g_mu;
Plane* g_plane = nullptr;
std::atomic<bool> g_active{false};

Doorbell* open_bell(const std::string& name, bool shared) {
    if (!shared) return new Doorbell();
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
        if (error) *error = "bad rank/world/unique id";
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
    if (p->ops->init(device, (size_t)world * kHdrBytes, error) != 0) {
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
    for (PeerState& ps : p->peers) ps.credit = (uint64_t)std::max<int64_t>(FLAGS_rccl_window_bytes, 1);
    // round 1, collectively and synchronously: connects every pair (RCCL
    // connects p2p peers lazily inside the first group that uses them)
    const int rc = world > 1 ? p->run_round(1) : 0;
    if (!p->api.fake()) hipSetDevice(prev);
    if (rc != 0) {
        if (error) *error = "rccl plane: the first round failed";
        if (!p->bell_name.empty()) shm_unlink(p->bell_name.c_str());
        p.release();  // its comm is aborted; the stream may still reference it
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
    g_plane->bell->seq.fetch_add(1);
    futex(&g_plane->bell->seq, FUTEX_WAKE, INT_MAX, nullptr);
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
