// RDMA global state, registered block pool, handshake and the endpoint
// (see rdma/rdma.h). Reference parity: rdma_helper.cpp:373
// GlobalRdmaInitializeOrDieImpl + :157 RegisterMemoryForRdma; block_pool.cpp
// :189 InitBlockPool / :362 AllocBlock / :389 DeallocBlock;
// rdma_endpoint.cpp :409/:552 hello exchange, :771-895 CutFromIOBufList,
// :926 HandleCompletion, :1008 PostRecv, :1317-1342 PollCq.
//
// Flow control: each side posts rq_size receive blocks. The sender's window
// is the peer's rq_size minus a small reserve for pure ACKs; every SEND
// carries, as immediate data, the number of receive blocks this side has
// reposted since its last SEND (so credits ride on normal traffic, as in a
// request/response ping-pong), and a zero-length SEND_WITH_IMM returns
// credits only when half the local ring has been consumed silently. Send
// completions are signalled every sq_size/4 work requests; one completion
// retires every earlier request (RC completes in order), releasing the Buf
// references that kept the zero-copy payload alive.
#include <sys/epoll.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <shared_mutex>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"
#include "fiber/butex.h"
#include "net/socket.h"
#include "rdma/rdma.h"
#include "rpc/errno.h"

DEFINE_string(rdma_provider, "auto", "verbs provider: auto (ibverbs if an HCA is present, else soft), ibverbs, soft");
DEFINE_int32(rdma_sq_size, 128, "send queue depth of RDMA endpoints");
DEFINE_int32(rdma_rq_size, 128, "receive queue depth (receive blocks posted) of RDMA endpoints");
DEFINE_string(rdma_recv_block_type, "default", "receive block size: default (8KiB), large (64KiB), huge (2MiB)");
DEFINE_int32(rdma_memory_pool_initial_size_mb, 64, "first registered region of the RDMA block pool");
DEFINE_int32(rdma_memory_pool_increase_size_mb, 64, "size of every further registered region");
DEFINE_int32(rdma_memory_pool_max_regions, 16, "max registered regions of the RDMA block pool");
DEFINE_int32(rdma_handshake_timeout_ms, 2000, "timeout of the RDMA hello exchange");

namespace mrpc {
namespace rdma {

const char kMagic[4] = {'R', 'D', 'M', 'A'};

namespace {

const size_t kBlockHeader = (sizeof(BufBlock) + 15) & ~(size_t)15;
const size_t kClassTotal[3] = {Buf::DEFAULT_BLOCK_SIZE, 64 * 1024, 2 * 1024 * 1024};
const int kMaxRegions = 64;
const int kReservedAckWrs = 4;

struct Region {
    char* base;
    size_t len;
    uint32_t lkey;
};

struct UserRegion {
    size_t len;
    uint32_t lkey;
    MemKind kind;
};

struct Pool {
    std::mutex region_mu;
    Region regions[kMaxRegions];
    std::atomic<int> nregions{0};
    char* bump = nullptr;
    size_t bump_left = 0;
    std::mutex class_mu[3];
    std::vector<void*> free_list[3];
    std::atomic<int64_t> handed[3];
    std::atomic<int64_t> fallback{0};
    std::atomic<int64_t> region_bytes{0};
    std::shared_mutex user_mu;
    std::map<uintptr_t, UserRegion> user;
    Pool() {
        for (auto& h : handed) h.store(0);
    }
};

Pool& pool() {
    static Pool* p = new Pool;
    return *p;
}

std::mutex g_init_mu;
std::unique_ptr<Provider> g_provider;
std::atomic<bool> g_available{false};
DmabufExportFn g_dmabuf_export = nullptr;

int class_of(size_t bytes) {
    for (int i = 0; i < 3; ++i) {
        if (bytes == kClassTotal[i]) return i;
    }
    return -1;
}

// Grow the pool by one registered region (region_mu held).
bool AddRegionLocked(Pool& p, size_t bytes) {
    const int n = p.nregions.load(std::memory_order_relaxed);
    if (n >= std::min(kMaxRegions, FLAGS_rdma_memory_pool_max_regions) || !g_provider) return false;
    void* mem = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (mem == MAP_FAILED) return false;
    uint32_t lkey = 0;
    if (g_provider->RegisterMemory(mem, bytes, false, -1, &lkey) != 0) {
        munmap(mem, bytes);
        return false;
    }
    p.regions[n] = Region{static_cast<char*>(mem), bytes, lkey};
    p.nregions.store(n + 1, std::memory_order_release);
    p.bump = static_cast<char*>(mem);
    p.bump_left = bytes;
    p.region_bytes.fetch_add((int64_t)bytes, std::memory_order_relaxed);
    return true;
}

void* CarveLocked(Pool& p, size_t bytes) {
    if (p.bump_left < bytes) {
        const size_t inc = (size_t)std::max(1, p.nregions.load() == 0 ? FLAGS_rdma_memory_pool_initial_size_mb
                                                                          : FLAGS_rdma_memory_pool_increase_size_mb)
                           << 20;
        if (!AddRegionLocked(p, std::max(inc, bytes))) return nullptr;
    }
    void* r = p.bump;
    p.bump += bytes;
    p.bump_left -= bytes;
    return r;
}

bool in_pool(const void* ptr) {
    Pool& p = pool();
    const int n = p.nregions.load(std::memory_order_acquire);
    const char* c = static_cast<const char*>(ptr);
    for (int i = 0; i < n; ++i) {
        if (c >= p.regions[i].base && c < p.regions[i].base + p.regions[i].len) return true;
    }
    return false;
}

void* PoolAlloc(size_t bytes) {
    Pool& p = pool();
    const int c = class_of(bytes);
    if (c >= 0) {
        {
            std::lock_guard<std::mutex> g(p.class_mu[c]);
            if (!p.free_list[c].empty()) {
                void* r = p.free_list[c].back();
                p.free_list[c].pop_back();
                p.handed[c].fetch_add(1, std::memory_order_relaxed);
                return r;
            }
        }
        void* r;
        {
            std::lock_guard<std::mutex> g(p.region_mu);
            r = CarveLocked(p, bytes);
        }
        if (r) {
            p.handed[c].fetch_add(1, std::memory_order_relaxed);
            return r;
        }
    }
    p.fallback.fetch_add(1, std::memory_order_relaxed);
    return aligned_alloc(64, (bytes + 63) & ~(size_t)63);
}

void PoolFree(void* ptr, size_t bytes) {
    Pool& p = pool();
    const int c = class_of(bytes);
    if (c >= 0 && in_pool(ptr)) {
        p.handed[c].fetch_sub(1, std::memory_order_relaxed);
        std::lock_guard<std::mutex> g(p.class_mu[c]);
        p.free_list[c].push_back(ptr);
        return;
    }
    free(ptr);
}

size_t recv_block_total() {
    if (FLAGS_rdma_recv_block_type == "large") return kClassTotal[1];
    if (FLAGS_rdma_recv_block_type == "huge") return kClassTotal[2];
    return kClassTotal[0];
}

void put_be16(char* p, uint16_t v) {
    p[0] = (char)(v >> 8);
    p[1] = (char)v;
}
void put_be32(char* p, uint32_t v) {
    for (int i = 0; i < 4; ++i) p[i] = (char)(v >> (24 - 8 * i));
}
void put_be64(char* p, uint64_t v) {
    for (int i = 0; i < 8; ++i) p[i] = (char)(v >> (56 - 8 * i));
}
uint16_t get_be16(const char* p) { return (uint16_t)(((uint8_t)p[0] << 8) | (uint8_t)p[1]); }
uint32_t get_be32(const char* p) {
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) v = (v << 8) | (uint8_t)p[i];
    return v;
}
uint64_t get_be64(const char* p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v = (v << 8) | (uint8_t)p[i];
    return v;
}

// Blocking (fiber-aware) full write / read on a non-blocking fd.
int write_full(int fd, const char* p, size_t n, const timespec* abstime) {
    while (n > 0) {
        const ssize_t w = ::write(fd, p, n);
        if (w > 0) {
            p += w;
            n -= (size_t)w;
            continue;
        }
        if (w < 0 && errno == EINTR) continue;
        if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
            if (fiber::fd_timedwait(fd, EPOLLOUT, abstime) != 0) return -1;
            continue;
        }
        return -1;
    }
    return 0;
}

int read_full(int fd, char* p, size_t n, const timespec* abstime) {
    while (n > 0) {
        const ssize_t r = ::read(fd, p, n);
        if (r > 0) {
            p += r;
            n -= (size_t)r;
            continue;
        }
        if (r == 0) {
            errno = ECONNRESET;
            return -1;
        }
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) {
            if (fiber::fd_timedwait(fd, EPOLLIN, abstime) != 0) return -1;
            continue;
        }
        return -1;
    }
    return 0;
}

}  // namespace

// ---------------------------------------------------------------- global

int GlobalRdmaInitialize(std::string* err) {
    std::lock_guard<std::mutex> g(g_init_mu);
    if (g_available.load()) return 0;
    std::string why;
    const std::string want = FLAGS_rdma_provider;
    if (want == "auto" || want == "ibverbs") g_provider = CreateIbverbsProvider(&why);
    if (!g_provider) {
        if (want == "ibverbs") {
            if (err) *err = "ibverbs provider unavailable: " + why;
            return -1;
        }
        if (want != "auto" && want != "soft") {
            if (err) *err = "unknown -rdma_provider=" + want;
            return -1;
        }
        if (want == "auto") LOG(INFO) << "RDMA: no HCA (" << why << "), using the in-process soft provider";
        g_provider = CreateSoftProvider();
    }
    {
        Pool& p = pool();
        std::lock_guard<std::mutex> rg(p.region_mu);
        if (!AddRegionLocked(p, (size_t)std::max(1, FLAGS_rdma_memory_pool_initial_size_mb) << 20)) {
            if (err) *err = "fail to register the initial RDMA memory region";
            g_provider.reset();
            return -1;
        }
    }
    // Every default Buf block now comes from registered memory (the
    // reference swaps butil::iobuf::blockmem_allocate the same way).
    SetBlockMemAllocator(BlockMemAllocator{PoolAlloc, PoolFree, MemKind::HOST});
    g_available.store(true, std::memory_order_release);
    LOG(INFO) << "RDMA initialised: provider=" << g_provider->name() << " device=" << g_provider->device_name();
    return 0;
}

bool RdmaAvailable() { return g_available.load(std::memory_order_acquire); }
Provider* GetProvider() { return g_available.load(std::memory_order_acquire) ? g_provider.get() : nullptr; }

void SetDmabufExportHook(DmabufExportFn fn) { g_dmabuf_export = fn; }
DmabufExportFn GetDmabufExportHook() { return g_dmabuf_export; }

int RegisterMemoryForRdma(void* ptr, size_t n, MemKind kind, int gpu) {
    Provider* pr = GetProvider();
    if (!pr || !ptr || n == 0) {
        errno = EINVAL;
        return -1;
    }
    uint32_t lkey = 0;
    if (pr->RegisterMemory(ptr, n, kind == MemKind::DEVICE || kind == MemKind::PEER, gpu, &lkey) != 0) return -1;
    Pool& p = pool();
    std::unique_lock<std::shared_mutex> g(p.user_mu);
    p.user[reinterpret_cast<uintptr_t>(ptr)] = UserRegion{n, lkey, kind};
    return 0;
}

void DeregisterMemoryForRdma(void* ptr) {
    Provider* pr = GetProvider();
    if (!pr) return;
    Pool& p = pool();
    {
        std::unique_lock<std::shared_mutex> g(p.user_mu);
        if (p.user.erase(reinterpret_cast<uintptr_t>(ptr)) == 0) return;
    }
    pr->DeregisterMemory(ptr);
}

bool LookupLkey(const void* ptr, size_t n, uint32_t* lkey) {
    Pool& p = pool();
    const char* c = static_cast<const char*>(ptr);
    const int nr = p.nregions.load(std::memory_order_acquire);
    for (int i = 0; i < nr; ++i) {
        const Region& r = p.regions[i];
        if (c >= r.base && c + n <= r.base + r.len) {
            *lkey = r.lkey;
            return true;
        }
    }
    std::shared_lock<std::shared_mutex> g(p.user_mu);
    if (p.user.empty()) return false;
    auto it = p.user.upper_bound(reinterpret_cast<uintptr_t>(ptr));
    if (it == p.user.begin()) return false;
    --it;
    if (reinterpret_cast<uintptr_t>(ptr) + n <= it->first + it->second.len) {
        *lkey = it->second.lkey;
        return true;
    }
    return false;
}

PoolStats GetPoolStats() {
    Pool& p = pool();
    PoolStats s;
    s.regions = p.nregions.load();
    s.region_bytes = p.region_bytes.load();
    s.blocks_8k = p.handed[0].load();
    s.blocks_64k = p.handed[1].load();
    s.blocks_2m = p.handed[2].load();
    s.fallback_allocs = p.fallback.load();
    std::shared_lock<std::shared_mutex> g(p.user_mu);
    s.user_regions = (int64_t)p.user.size();
    return s;
}

BufBlock* NewRegisteredBlock(size_t total) {
    // NewBlock() rounds (header + cap) up to 4 KiB, which lands exactly on
    // the pool classes; the default class comes from the TLS block cache.
    BufBlock* b = NewBlock(total - kBlockHeader);
    if (!b) return nullptr;
    uint32_t lkey;
    if (!LookupLkey(b->data, b->cap, &lkey)) {
        b->dec_ref();  // a block cached before the allocator swap
        return nullptr;
    }
    return b;
}

// ---------------------------------------------------------------- hello

void Hello::Serialize(char* out) const {
    memcpy(out, kMagic, 4);
    put_be16(out + 4, version);
    put_be16(out + 6, sq_size);
    put_be16(out + 8, rq_size);
    put_be16(out + 10, flags);
    put_be32(out + 12, block_size);
    put_be64(out + 16, addr.gid_hi);
    put_be64(out + 24, addr.gid_lo);
    put_be32(out + 32, addr.qpn);
    put_be16(out + 36, addr.lid);
    memset(out + 38, 0, kSize - 38);
}

bool Hello::Parse(const char* in) {
    if (memcmp(in, kMagic, 4) != 0) return false;
    version = get_be16(in + 4);
    sq_size = get_be16(in + 6);
    rq_size = get_be16(in + 8);
    flags = get_be16(in + 10);
    block_size = get_be32(in + 12);
    addr.gid_hi = get_be64(in + 16);
    addr.gid_lo = get_be64(in + 24);
    addr.qpn = get_be32(in + 32);
    addr.lid = get_be16(in + 36);
    return version == kVersion && rq_size > kReservedAckWrs && sq_size > 0 && block_size >= 64;
}

// ---------------------------------------------------------------- endpoint

Endpoint::Endpoint(SocketId host) : _host(host), _write_butex(fiber::butex_create()) {}

Endpoint::~Endpoint() {
    _qp.reset();
    _cq.reset();
    for (BufBlock* b : _rbuf) {
        if (b) b->dec_ref();
    }
    _sbuf.clear();
    fiber::butex_destroy(_write_butex);
}

int Endpoint::Init(std::string* err) {
    Provider* pr = GetProvider();
    if (!pr) {
        if (err) *err = "RDMA is not initialised";
        return -1;
    }
    _sq_size = std::max(8, std::min(FLAGS_rdma_sq_size, 4096));
    _rq_size = std::max(kReservedAckWrs + 4, std::min(FLAGS_rdma_rq_size, 4096));
    _recv_block_total = recv_block_total();
    _local_block_cap = (uint32_t)(_recv_block_total - kBlockHeader);
    _cq = pr->CreateCq(_sq_size + _rq_size);
    if (!_cq) {
        if (err) *err = "fail to create CQ";
        return -1;
    }
    _qp = pr->CreateQp(_cq.get(), _sq_size, _rq_size);
    if (!_qp) {
        if (err) *err = "fail to create QP";
        return -1;
    }
    _sbuf.resize((size_t)_sq_size);
    _rbuf.assign((size_t)_rq_size, nullptr);
    if (_qp->Prepare() != 0) {
        if (err) *err = std::string("fail to move the QP to INIT: ") + strerror(errno);
        return -1;
    }
    // receives are posted in INIT, before the peer can send (no RNR gap)
    for (size_t i = 0; i < _rbuf.size(); ++i) {
        if (PostRecvSlot(i) != 0) {
            if (err) *err = "fail to post receive blocks";
            return -1;
        }
    }
    return 0;
}

int Endpoint::PostRecvSlot(size_t slot) {
    BufBlock* b = _rbuf[slot];
    if (!b) {
        b = NewRegisteredBlock(_recv_block_total);
        if (!b) b = NewRegisteredBlock(_recv_block_total);  // retry once past a stale TLS block
        if (!b) return -1;
        _rbuf[slot] = b;
    }
    Sge s;
    s.addr = reinterpret_cast<uint64_t>(b->data);
    s.length = b->cap;
    if (!LookupLkey(b->data, b->cap, &s.lkey)) return -1;
    return _qp->PostRecv(slot, s);
}

void Endpoint::FillHello(Hello* h) const {
    h->sq_size = (uint16_t)_sq_size;
    h->rq_size = (uint16_t)_rq_size;
    h->flags = GetDmabufExportHook() ? 1 : 0;
    h->block_size = _local_block_cap;
    h->addr = _qp->local();
}

int Endpoint::Start(const Hello& h, std::string* err) {
    if (_qp->Connect(h.addr) != 0) {
        if (err) *err = std::string("fail to connect QP: ") + strerror(errno);
        return -1;
    }
    _remote_block_cap = h.block_size;
    _remote_gpudirect = (h.flags & 1) != 0;
    _window.store((int)h.rq_size - kReservedAckWrs, std::memory_order_release);
    auto* self = new std::shared_ptr<Endpoint>(shared_from_this());
    _started.store(true, std::memory_order_release);
    if (fiber::start_background(&_poller, &fiber::ATTR_NORMAL, PollLoop, self) != 0) {
        delete self;
        _started.store(false);
        if (err) *err = "fail to start the completion poller";
        return -1;
    }
    _poller_running = true;
    return 0;
}

void* Endpoint::PollLoop(void* arg) {
    std::shared_ptr<Endpoint>* holder = static_cast<std::shared_ptr<Endpoint>*>(arg);
    Endpoint* ep = holder->get();
    while (!ep->_stop.load(std::memory_order_acquire)) {
        if (ep->HandleCompletions() < 0) break;
        ep->_cq->Arm();
        if (ep->HandleCompletions() < 0) break;
        timespec ts = realtime_after_us(100000);
        fiber::fd_timedwait(ep->_cq->notify_fd(), EPOLLIN, &ts);
        ep->_cq->AckEvent();
    }
    delete holder;
    return nullptr;
}

void Endpoint::FailHost(int err, const char* what) {
    _stop.store(true, std::memory_order_release);
    SocketUniquePtr s;
    if (Socket::Address(_host, &s) == 0) s->SetFailed(err, "rdma: %s", what);
    _write_butex->fetch_add(1, std::memory_order_release);
    fiber::butex_wake_all(_write_butex);
}

int Endpoint::HandleCompletions() {
    WorkCompletion wc[32];
    bool got_data = false, wake = false;
    for (;;) {
        const int n = _cq->Poll(wc, 32);
        if (n < 0) {
            FailHost(ERDMA, "poll CQ failed");
            return -1;
        }
        if (n == 0) break;
        for (int i = 0; i < n; ++i) {
            const WorkCompletion& c = wc[i];
            if (c.status != 0) {
                FailHost(ERDMA, c.opcode == WC_RECV ? "receive completion error" : "send completion error");
                return -1;
            }
            if (c.opcode == WC_RECV) {
                const size_t slot = (size_t)c.wr_id;
                if (c.has_imm && c.imm > 0) {
                    _window.fetch_add((int)c.imm, std::memory_order_release);
                    wake = true;
                }
                if (c.byte_len > 0) {
                    BufBlock* b = _rbuf[slot];
                    b->size = b->cap;  // never appended into again
                    {
                        std::lock_guard<std::mutex> g(_in_mu);
                        _in.append_block(b, 0, c.byte_len);
                    }
                    b->dec_ref();
                    _rbuf[slot] = nullptr;
                    got_data = true;
                    std::lock_guard<std::mutex> g(_stat_mu);
                    ++_stats.recv_msgs;
                    _stats.recv_bytes += c.byte_len;
                }
                if (PostRecvSlot(slot) != 0) {
                    FailHost(ERDMA, "fail to repost a receive block");
                    return -1;
                }
                if (c.byte_len > 0) _new_acks.fetch_add(1, std::memory_order_acq_rel);
            } else {
                std::lock_guard<std::mutex> g(_send_mu);
                for (uint64_t k = _sq_completed; k <= c.wr_id && k < _sq_posted; ++k) _sbuf[k % _sbuf.size()].clear();
                if (c.wr_id + 1 > _sq_completed) _sq_completed = c.wr_id + 1;
                wake = true;
            }
        }
    }
    if (got_data) Socket::StartInputEvent(_host, EPOLLIN);
    if (_new_acks.load(std::memory_order_acquire) >= std::max(1, _rq_size / 2)) {
        std::lock_guard<std::mutex> g(_send_mu);
        if (_new_acks.load() >= std::max(1, _rq_size / 2)) SendPureAckLocked();
    }
    if (wake) {
        _write_butex->fetch_add(1, std::memory_order_release);
        fiber::butex_wake_all(_write_butex);
    }
    return 0;
}

int Endpoint::SendPureAckLocked() {
    if (_sq_posted - _sq_completed >= (uint64_t)_sq_size) return -1;  // retried on the next completion
    const uint32_t imm = (uint32_t)_new_acks.exchange(0, std::memory_order_acq_rel);
    const uint64_t wr = _sq_posted;
    const bool signaled = ++_unsignaled >= std::max(1, _sq_size / 4);
    if (signaled) _unsignaled = 0;
    if (_qp->PostSend(wr, nullptr, 0, true, imm, signaled) != 0) {
        _new_acks.fetch_add((int)imm);
        return -1;
    }
    _sbuf[wr % _sbuf.size()].clear();
    ++_sq_posted;
    std::lock_guard<std::mutex> g(_stat_mu);
    ++_stats.pure_acks_sent;
    return 0;
}

ssize_t Endpoint::CutFromBufList(Buf* const* pieces, size_t count) {
    std::lock_guard<std::mutex> g(_send_mu);
    if (_stop.load(std::memory_order_acquire)) {
        errno = EPIPE;
        return -1;
    }
    Provider* pr = GetProvider();
    const int max_sge = std::min(16, pr ? pr->max_sge() : 1);
    ssize_t total = 0;
    bool blocked = false;
    int64_t msgs = 0, bounces = 0;
    for (size_t i = 0; i < count && !blocked; ++i) {
        Buf* b = pieces[i];
        while (!b->empty()) {
            if (_window.load(std::memory_order_acquire) <= 0 ||
                _sq_posted - _sq_completed >= (uint64_t)(_sq_size - 1)) {  // one slot stays for a pure ACK
                blocked = true;
                break;
            }
            Buf chunk;
            b->cutn(&chunk, std::min(b->size(), (size_t)_remote_block_cap));
            const size_t n = chunk.size();
            Sge sge[16];
            int nsge = 0;
            bool zero_copy = (int)chunk.backing_block_num() <= max_sge;
            for (size_t k = 0; zero_copy && k < chunk.backing_block_num(); ++k) {
                // DEVICE blocks go zero-copy only from registered HBM (the
                // HCA reads it directly: GPUDirect); the peer always lands
                // the bytes in its host receive blocks.
                sge[nsge].addr = reinterpret_cast<uint64_t>(chunk.block_data(k));
                sge[nsge].length = (uint32_t)chunk.block_len(k);
                if (!LookupLkey(chunk.block_data(k), chunk.block_len(k), &sge[nsge].lkey)) zero_copy = false;
                ++nsge;
            }
            if (!zero_copy) {
                // Unregistered (or too fragmented) payload: one copy into a
                // registered block of the smallest class that fits.
                size_t total_sz = kClassTotal[0];
                for (size_t cls : kClassTotal) {
                    if (cls - kBlockHeader >= n) {
                        total_sz = cls;
                        break;
                    }
                }
                BufBlock* nb = NewRegisteredBlock(total_sz);
                if (!nb || nb->cap < n) {
                    if (nb) nb->dec_ref();
                    errno = ENOMEM;
                    return total > 0 ? total : -1;
                }
                chunk.copy_to(nb->data, n);
                nb->size = nb->cap;
                chunk.clear();
                chunk.append_block(nb, 0, (uint32_t)n);
                nb->dec_ref();
                nsge = 1;
                sge[0].addr = reinterpret_cast<uint64_t>(nb->data);
                sge[0].length = (uint32_t)n;
                LookupLkey(nb->data, n, &sge[0].lkey);
                ++bounces;
            }
            const uint64_t wr = _sq_posted;
            const bool signaled = ++_unsignaled >= std::max(1, _sq_size / 4);
            if (signaled) _unsignaled = 0;
            const uint32_t imm = (uint32_t)_new_acks.exchange(0, std::memory_order_acq_rel);
            if (_qp->PostSend(wr, sge, nsge, true, imm, signaled) != 0) {
                _new_acks.fetch_add((int)imm);
                const int saved = errno ? errno : EIO;
                errno = saved;
                return -1;
            }
            _sbuf[wr % _sbuf.size()] = std::move(chunk);
            ++_sq_posted;
            _window.fetch_sub(1, std::memory_order_acq_rel);
            total += (ssize_t)n;
            ++msgs;
        }
    }
    {
        std::lock_guard<std::mutex> sg(_stat_mu);
        _stats.sent_msgs += msgs;
        _stats.sent_bytes += total;
        _stats.bounce_copies += bounces;
        if (blocked) ++_stats.window_full;
    }
    if (total == 0 && blocked) {
        errno = EAGAIN;
        return -1;
    }
    return total;
}

ssize_t Endpoint::ReadInto(Buf* out) {
    std::lock_guard<std::mutex> g(_in_mu);
    if (_in.empty()) {
        errno = EAGAIN;
        return -1;
    }
    const ssize_t n = (ssize_t)_in.size();
    out->append(std::move(_in));
    _in.clear();
    return n;
}

int Endpoint::WaitWritable(const timespec* abstime) {
    const int expected = _write_butex->load(std::memory_order_acquire);
    if (_stop.load(std::memory_order_acquire)) {
        errno = EPIPE;
        return -1;
    }
    {
        std::lock_guard<std::mutex> g(_send_mu);
        if (_window.load() > 0 && _sq_posted - _sq_completed < (uint64_t)(_sq_size - 1)) return 0;
    }
    if (fiber::butex_wait(_write_butex, expected, abstime) < 0 && errno != EWOULDBLOCK && errno != EINTR) return -1;
    return 0;
}

void Endpoint::Shutdown() {
    _stop.store(true, std::memory_order_release);
    _write_butex->fetch_add(1, std::memory_order_release);
    fiber::butex_wake_all(_write_butex);
}

EndpointStats Endpoint::stats() const {
    std::lock_guard<std::mutex> g(_stat_mu);
    return _stats;
}

std::string Endpoint::Describe() const {
    EndpointStats s = stats();
    return string_printf("rdma{window=%d sq=%d rq=%d block=%u/%u sent=%lld/%lldB recv=%lld/%lldB acks=%lld bounce=%lld}",
                         _window.load(), _sq_size, _rq_size, _local_block_cap, _remote_block_cap,
                         (long long)s.sent_msgs, (long long)s.sent_bytes, (long long)s.recv_msgs,
                         (long long)s.recv_bytes, (long long)s.pure_acks_sent, (long long)s.bounce_copies);
}

// ---------------------------------------------------------------- handshake

std::shared_ptr<Endpoint> ClientHandshake(SocketId host, int fd, const timespec* abstime, std::string* err) {
    timespec ts;
    if (!abstime) {
        ts = realtime_after_us((int64_t)FLAGS_rdma_handshake_timeout_ms * 1000);
        abstime = &ts;
    }
    std::shared_ptr<Endpoint> ep = std::make_shared<Endpoint>(host);
    if (ep->Init(err) != 0) return nullptr;
    Hello mine;
    ep->FillHello(&mine);
    char buf[Hello::kSize];
    mine.Serialize(buf);
    if (write_full(fd, buf, sizeof(buf), abstime) != 0 || read_full(fd, buf, sizeof(buf), abstime) != 0) {
        if (err) *err = std::string("hello exchange failed: ") + strerror(errno);
        return nullptr;
    }
    Hello peer;
    if (!peer.Parse(buf)) {
        if (err) *err = "bad RDMA hello from server";
        return nullptr;
    }
    if (ep->Start(peer, err) != 0) return nullptr;
    return ep;
}

int ServerTryHandshake(SocketId host, int fd, Buf* in, std::shared_ptr<Endpoint>* out, std::string* err) {
    char head[Hello::kSize];
    const size_t have = std::min(in->size(), sizeof(head));
    in->copy_to(head, have);
    if (memcmp(head, kMagic, std::min(have, sizeof(kMagic))) != 0) return -1;
    if (have < Hello::kSize) return 0;
    Hello peer;
    if (!peer.Parse(head)) {
        if (err) *err = "malformed RDMA hello";
        return -1;
    }
    in->pop_front(Hello::kSize);
    if (!RdmaAvailable()) {
        if (err) *err = "RDMA hello on a server without RDMA";
        return -1;
    }
    std::shared_ptr<Endpoint> ep = std::make_shared<Endpoint>(host);
    if (ep->Init(err) != 0 || ep->Start(peer, err) != 0) return -1;
    Hello mine;
    ep->FillHello(&mine);
    char buf[Hello::kSize];
    mine.Serialize(buf);
    timespec ts = realtime_after_us((int64_t)FLAGS_rdma_handshake_timeout_ms * 1000);
    if (write_full(fd, buf, sizeof(buf), &ts) != 0) {
        if (err) *err = std::string("fail to reply hello: ") + strerror(errno);
        ep->Shutdown();
        return -1;
    }
    *out = std::move(ep);
    return 1;
}

std::string DescribeRdma() {
    PoolStats s = GetPoolStats();
    Provider* pr = GetProvider();
    return string_printf(
        "rdma_available: %d\nprovider: %s\ndevice: %s\nibverbs_compiled_in: %d\nregions: %lld (%lld MiB)\n"
        "blocks_in_use: 8k=%lld 64k=%lld 2m=%lld\nunregistered_fallback_allocs: %lld\nuser_regions: %lld\n",
        RdmaAvailable() ? 1 : 0, pr ? pr->name() : "-", pr ? pr->device_name().c_str() : "-",
        IbverbsCompiledIn() ? 1 : 0, (long long)s.regions, (long long)(s.region_bytes >> 20), (long long)s.blocks_8k,
        (long long)s.blocks_64k, (long long)s.blocks_2m, (long long)s.fallback_allocs, (long long)s.user_regions);
}

}  // namespace rdma
}  // namespace mrpc
