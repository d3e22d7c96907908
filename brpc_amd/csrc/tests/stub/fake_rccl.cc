// Stub RCCL library (libfake_rccl.so) for running the RCCL payload plane
// (gpu/rccl_plane.h) on hosts without GPUs: the plane dlopen()s it through
// -rccl_library exactly as it would librccl.so, so 2/3/8-rank CPU jobs
// (gloo for the control plane) drive the same round/credit/abort logic the
// MI355X jobs run.
//
// The stub models RCCL's point-to-point semantics at their most hostile:
//  * every rank pair (src, dst) is a bounded byte FIFO in POSIX shared
//    memory (kChanCap bytes, much smaller than a 1 MiB payload), so a send
//    completes only as fast as the receiver's matching recv drains it —
//    there is no eager buffer to hide an ordering bug;
//  * the k-th send src->dst matches the k-th recv at dst from src (each
//    message carries its length, a mismatch is an error);
//  * every stream of the process feeds ONE executor thread, i.e. all
//    streams share a single in-order hardware queue (the worst case of
//    GPU_MAX_HW_QUEUES false dependencies). A group blocks that queue
//    until all of its ops are matched and done;
//  * ncclCommAbort is local: peers waiting on an aborted rank block until
//    their own plane gives up (or notice the process is gone), as with
//    the real library.
// Besides the nccl* subset the plane resolves, the stub exports mrpcfake_*
// stream functions (create, in-order memcpy, record/query a marker) that
// the plane uses instead of HIP streams and events when it runs on it.
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#define EXPORT extern "C" __attribute__((visibility("default")))

namespace {

// ---- the ABI subset (matches rccl/rccl.h)
enum ncclResult_t {
    ncclSuccess = 0,
    ncclUnhandledCudaError = 1,
    ncclSystemError = 2,
    ncclInternalError = 3,
    ncclInvalidArgument = 4,
    ncclInvalidUsage = 5,
    ncclRemoteError = 6,
    ncclInProgress = 7,
};
struct ncclUniqueId {
    char internal[128];
};
enum ncclDataType_t { ncclInt8 = 0, ncclUint8 = 1 };

const uint64_t kSegMagic = 0x4d52504346414b45ull;  // "MRPCFAKE"
const int kMaxRanks = 16;
const size_t kChanCap = 64 << 10;

struct alignas(64) Chan {
    std::atomic<uint64_t> written;
    char pad0[56];
    std::atomic<uint64_t> read;
    char pad1[56];
    char ring[kChanCap];
};

struct Seg {
    uint64_t magic;
    uint32_t nranks;
    std::atomic<uint32_t> joined;
    std::atomic<int32_t> pid[kMaxRanks];
    char pad[64];
    Chan chan[kMaxRanks * kMaxRanks];  // [src * kMaxRanks + dst]
};

int64_t now_us() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (int64_t)ts.tv_sec * 1000000 + ts.tv_nsec / 1000;
}

int64_t timeout_us() {
    const char* e = getenv("MRPC_FAKE_RCCL_TIMEOUT_MS");
    return (e ? atoll(e) : 60000) * 1000;
}

struct Comm {
    Seg* seg = nullptr;
    std::string name;
    int rank = 0, nranks = 0;
    std::atomic<bool> aborted{false};
    std::atomic<int> async_error{ncclSuccess};
};

struct Op {
    bool send = false;
    Comm* comm = nullptr;
    int peer = 0;
    char* buf = nullptr;
    size_t len = 0;
    size_t done = 0;
    int hdr = 0;  // header bytes moved (8 = header done)
    uint64_t hdr_val = 0;
};

struct Stream;

struct Item {
    enum Kind { GROUP, MEMCPY, MARKER } kind = GROUP;
    Stream* stream = nullptr;
    std::vector<Op> ops;
    void* dst = nullptr;
    const void* src = nullptr;
    size_t n = 0;
    uint64_t ticket = 0;
};

struct Stream {
    std::atomic<uint64_t> done_ticket{0};
    std::atomic<bool> failed{false};
    uint64_t next_ticket = 0;  // under the executor mutex
};

// ---- ring I/O on one channel (single producer, single consumer)
size_t ring_write(Chan* c, const char* src, size_t n) {
    const uint64_t w = c->written.load(std::memory_order_relaxed);
    const uint64_t r = c->read.load(std::memory_order_acquire);
    const size_t space = kChanCap - (size_t)(w - r);
    n = std::min(n, space);
    size_t off = (size_t)(w % kChanCap), first = std::min(n, kChanCap - off);
    memcpy(c->ring + off, src, first);
    if (n > first) memcpy(c->ring, src + first, n - first);
    c->written.store(w + n, std::memory_order_release);
    return n;
}

size_t ring_read(Chan* c, char* dst, size_t n) {
    const uint64_t r = c->read.load(std::memory_order_relaxed);
    const uint64_t w = c->written.load(std::memory_order_acquire);
    n = std::min(n, (size_t)(w - r));
    size_t off = (size_t)(r % kChanCap), first = std::min(n, kChanCap - off);
    memcpy(dst, c->ring + off, first);
    if (n > first) memcpy(dst + first, c->ring, n - first);
    c->read.store(r + n, std::memory_order_release);
    return n;
}

size_t ring_avail(Chan* c) {
    return (size_t)(c->written.load(std::memory_order_acquire) - c->read.load(std::memory_order_relaxed));
}
size_t ring_space(Chan* c) {
    return kChanCap - (size_t)(c->written.load(std::memory_order_relaxed) - c->read.load(std::memory_order_acquire));
}

// One non-blocking step; returns bytes moved, -1 on a protocol error.
long step(Op& op) {
    Seg* s = op.comm->seg;
    const int me = op.comm->rank;
    if (op.send) {
        Chan* c = &s->chan[me * kMaxRanks + op.peer];
        if (op.hdr < 8) {
            if (ring_space(c) < 8) return 0;
            uint64_t len = op.len;
            ring_write(c, reinterpret_cast<const char*>(&len), 8);
            op.hdr = 8;
            return 8;
        }
        const size_t n = ring_write(c, op.buf + op.done, op.len - op.done);
        op.done += n;
        return (long)n;
    }
    Chan* c = &s->chan[op.peer * kMaxRanks + me];
    if (op.hdr < 8) {
        if (ring_avail(c) < 8) return 0;
        ring_read(c, reinterpret_cast<char*>(&op.hdr_val), 8);
        op.hdr = 8;
        if (op.hdr_val != op.len) {
            fprintf(stderr, "fake_rccl: rank %d recv of %zu bytes from %d matched a send of %llu bytes\n", me, op.len,
                    op.peer, (unsigned long long)op.hdr_val);
            return -1;
        }
        return 8;
    }
    const size_t n = ring_read(c, op.buf + op.done, op.len - op.done);
    op.done += n;
    return (long)n;
}

bool op_done(const Op& op) { return op.hdr == 8 && op.done == op.len; }

bool peer_gone(Seg* s, int peer) {
    const int32_t pid = s->pid[peer].load(std::memory_order_acquire);
    return pid > 0 && kill(pid, 0) != 0 && errno == ESRCH;
}

// Run a group to completion (or failure) on the executor thread.
ncclResult_t run_group(std::vector<Op>& ops) {
    int64_t last = now_us();
    int idle = 0;
    // ops on one channel (same comm, direction and peer) move in issue
    // order: the k-th send matches the k-th recv
    std::vector<int> chan_of(ops.size());
    for (size_t i = 0; i < ops.size(); ++i) chan_of[i] = (ops[i].send ? 1 : 0) + 2 * ops[i].peer;
    for (;;) {
        bool all = true, moved = false;
        std::vector<char> busy_chan(2 * kMaxRanks, 0);
        for (size_t i = 0; i < ops.size(); ++i) {
            Op& op = ops[i];
            if (op_done(op)) continue;
            if (busy_chan[chan_of[i]]) {  // an earlier op of this channel is unfinished
                all = false;
                continue;
            }
            busy_chan[chan_of[i]] = 1;
            if (op.comm->aborted.load(std::memory_order_acquire)) return ncclSystemError;
            const long n = step(op);
            if (n < 0) return ncclInvalidUsage;
            if (n > 0) moved = true;
            if (!op_done(op)) all = false;
        }
        if (all) return ncclSuccess;
        if (moved) {
            last = now_us();
            idle = 0;
            continue;
        }
        if (++idle < 64) {
            std::this_thread::yield();
            continue;
        }
        usleep(20);
        const int64_t t = now_us();
        if ((idle & 255) == 0) {
            for (const Op& op : ops)
                if (!op_done(op) && peer_gone(op.comm->seg, op.peer)) return ncclRemoteError;
        }
        if (t - last > timeout_us()) {
            fprintf(stderr, "fake_rccl: group made no progress for %lld ms\n", (long long)(timeout_us() / 1000));
            return ncclSystemError;
        }
    }
}

// ---- the process's single in-order "hardware queue"
class Executor {
public:
    void push(Item&& it) {
        std::lock_guard<std::mutex> g(mu_);
        if (!started_) {
            started_ = true;
            std::thread([this] { loop(); }).detach();
        }
        q_.push_back(std::move(it));
        cv_.notify_one();
    }
    uint64_t record(Stream* s) {
        std::lock_guard<std::mutex> g(mu_);
        Item it;
        it.kind = Item::MARKER;
        it.stream = s;
        it.ticket = ++s->next_ticket;
        const uint64_t t = it.ticket;
        if (!started_) {
            started_ = true;
            std::thread([this] { loop(); }).detach();
        }
        q_.push_back(std::move(it));
        cv_.notify_one();
        return t;
    }

private:
    void loop() {
        for (;;) {
            Item it;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return !q_.empty(); });
                it = std::move(q_.front());
                q_.pop_front();
            }
            Stream* s = it.stream;
            switch (it.kind) {
            case Item::GROUP: {
                if (s->failed.load()) break;  // an aborted stream drops its queue
                const ncclResult_t r = run_group(it.ops);
                if (r != ncclSuccess) {
                    s->failed.store(true);
                    for (Op& op : it.ops) {
                        int expect = ncclSuccess;
                        op.comm->async_error.compare_exchange_strong(expect, r);
                    }
                }
                break;
            }
            case Item::MEMCPY:
                if (!s->failed.load()) memcpy(it.dst, it.src, it.n);
                break;
            case Item::MARKER:
                s->done_ticket.store(it.ticket, std::memory_order_release);
                break;
            }
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Item> q_;
    bool started_ = false;
};

Executor& executor() {
    static Executor* e = new Executor;
    return *e;
}

// ---- groups (per calling thread)
thread_local int g_depth = 0;
thread_local std::vector<std::pair<Stream*, Op>> g_pending;

ncclResult_t enqueue(Stream* s, Op&& op) {
    if (!s) return ncclInvalidArgument;
    g_pending.emplace_back(s, std::move(op));
    if (g_depth > 0) return ncclSuccess;
    // flush: one group item per stream, in first-use order
    std::vector<std::pair<Stream*, Op>> ops;
    ops.swap(g_pending);
    while (!ops.empty()) {
        Stream* st = ops.front().first;
        Item it;
        it.kind = Item::GROUP;
        it.stream = st;
        std::vector<std::pair<Stream*, Op>> rest;
        for (auto& p : ops) {
            if (p.first == st) it.ops.push_back(std::move(p.second));
            else rest.push_back(std::move(p));
        }
        executor().push(std::move(it));
        ops.swap(rest);
    }
    return ncclSuccess;
}

std::string seg_name(const ncclUniqueId& id) {
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < 32; ++i) h = (h ^ (unsigned char)id.internal[i]) * 1099511628211ull;
    char b[64];
    snprintf(b, sizeof(b), "/mrpc_fake_rccl_%016llx", (unsigned long long)h);
    return b;
}

const char* err_str(int r) {
    switch (r) {
    case ncclSuccess: return "no error (fake_rccl)";
    case ncclSystemError: return "unhandled system error (fake_rccl: timeout or abort)";
    case ncclInternalError: return "internal error (fake_rccl)";
    case ncclInvalidArgument: return "invalid argument (fake_rccl)";
    case ncclInvalidUsage: return "invalid usage (fake_rccl: mismatched send/recv)";
    case ncclRemoteError: return "remote process exited (fake_rccl)";
    case ncclInProgress: return "in progress (fake_rccl)";
    default: return "unknown (fake_rccl)";
    }
}

}  // namespace

EXPORT int mrpcfake_abi_version() { return 1; }

EXPORT ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    memset(id->internal, 0, sizeof(id->internal));
    FILE* f = fopen("/dev/urandom", "rb");
    size_t got = f ? fread(id->internal, 1, 32, f) : 0;
    if (f) fclose(f);
    if (got != 32) {
        const int64_t t = now_us();
        const int pid = getpid();
        memcpy(id->internal, &t, sizeof(t));
        memcpy(id->internal + 8, &pid, sizeof(pid));
    }
    strcpy(id->internal + 40, "fake_rccl");
    return ncclSuccess;
}

EXPORT ncclResult_t ncclCommInitRank(Comm** out, int nranks, ncclUniqueId id, int rank) {
    if (nranks <= 0 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    const std::string name = seg_name(id);
    const int fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0) return ncclSystemError;
    if (ftruncate(fd, (off_t)sizeof(Seg)) != 0) {
        close(fd);
        return ncclSystemError;
    }
    void* m = mmap(nullptr, sizeof(Seg), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return ncclSystemError;
    Seg* s = static_cast<Seg*>(m);
    s->pid[rank].store(getpid(), std::memory_order_release);
    s->joined.fetch_add(1);
    // like ncclCommInitRank: blocks until every rank joined
    const int64_t t0 = now_us();
    while ((int)s->joined.load() < nranks) {
        if (now_us() - t0 > timeout_us()) {
            munmap(m, sizeof(Seg));
            return ncclSystemError;
        }
        usleep(200);
    }
    s->magic = kSegMagic;
    s->nranks = (uint32_t)nranks;
    Comm* c = new Comm;
    c->seg = s;
    c->name = name;
    c->rank = rank;
    c->nranks = nranks;
    *out = c;
    return ncclSuccess;
}

EXPORT ncclResult_t ncclCommAbort(Comm* c) {
    if (!c) return ncclSuccess;
    c->aborted.store(true, std::memory_order_release);
    int expect = ncclSuccess;
    c->async_error.compare_exchange_strong(expect, ncclSystemError);
    // the segment stays mapped: the executor may still be looking at it,
    // and the last rank out unlinks the name
    shm_unlink(c->name.c_str());
    return ncclSuccess;
}

EXPORT ncclResult_t ncclCommGetAsyncError(Comm* c, ncclResult_t* r) {
    *r = c ? (ncclResult_t)c->async_error.load() : ncclInvalidArgument;
    return ncclSuccess;
}

EXPORT ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t dt, int peer, Comm* c, Stream* s) {
    if (!c || (dt != ncclInt8 && dt != ncclUint8) || peer < 0 || peer >= c->nranks) return ncclInvalidArgument;
    if (c->aborted.load()) return ncclInvalidUsage;
    Op op;
    op.send = true;
    op.comm = c;
    op.peer = peer;
    op.buf = const_cast<char*>(static_cast<const char*>(buf));
    op.len = count;
    return enqueue(s, std::move(op));
}

EXPORT ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t dt, int peer, Comm* c, Stream* s) {
    if (!c || (dt != ncclInt8 && dt != ncclUint8) || peer < 0 || peer >= c->nranks) return ncclInvalidArgument;
    if (c->aborted.load()) return ncclInvalidUsage;
    Op op;
    op.comm = c;
    op.peer = peer;
    op.buf = static_cast<char*>(buf);
    op.len = count;
    return enqueue(s, std::move(op));
}

EXPORT ncclResult_t ncclGroupStart() {
    ++g_depth;
    return ncclSuccess;
}

EXPORT ncclResult_t ncclGroupEnd() {
    if (g_depth <= 0) return ncclInvalidUsage;
    if (--g_depth > 0 || g_pending.empty()) return ncclSuccess;
    Stream* s = g_pending.back().first;
    Op last = std::move(g_pending.back().second);
    g_pending.pop_back();
    return enqueue(s, std::move(last));
}

EXPORT const char* ncclGetErrorString(ncclResult_t r) { return err_str(r); }

// ---- stream stand-ins for the plane
EXPORT void* mrpcfake_stream_create() { return new Stream; }
EXPORT void mrpcfake_stream_destroy(void* s) { (void)s; /* the executor may still hold it: leaked */ }
EXPORT int mrpcfake_stream_memcpy(void* s, void* dst, const void* src, size_t n) {
    Item it;
    it.kind = Item::MEMCPY;
    it.stream = static_cast<Stream*>(s);
    it.dst = dst;
    it.src = src;
    it.n = n;
    executor().push(std::move(it));
    return 0;
}
EXPORT uint64_t mrpcfake_stream_record(void* s) { return executor().record(static_cast<Stream*>(s)); }
// 1 done, 0 pending, -1 the stream failed (a group errored or was aborted)
EXPORT int mrpcfake_stream_query(void* s, uint64_t ticket) {
    Stream* st = static_cast<Stream*>(s);
    if (st->done_ticket.load(std::memory_order_acquire) >= ticket) return st->failed.load() ? -1 : 1;
    return 0;
}
