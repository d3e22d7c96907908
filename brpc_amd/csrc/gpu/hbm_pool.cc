#include "gpu/hbm_pool.h"

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "base/flags.h"
#include "base/logging.h"
#include "gpu/gpu.h"

DEFINE_int32(hbm_arena_mb, 16384,
             "IPC-exportable HBM arena per device for RPC payload blocks (MiB; 288 GB HBM3E per MI355X)");
DEFINE_int32(hbm_fallback_max_mb, 8192,
             "dedicated hipMalloc blocks (arena exhausted) may hold at most this much HBM; beyond it allocations fail");
DEFINE_int32(pinned_region_mb, 64, "pinned host memory is carved from hipHostMalloc regions of this size (MiB)");

namespace mrpc {
namespace gpu {

namespace {

const int kMaxDev = 16;
const int kMinClass = 8;    // 256 B
const int kMaxClass = 28;   // 256 MiB
const int kNumClass = kMaxClass + 1;
const int kTlsMax = 16;

inline int class_of(size_t n) {
    int c = kMinClass;
    while (c <= kMaxClass && ((size_t)1 << c) < n) ++c;
    return c;
}

// How many free blocks of class c a thread keeps for itself: about 1 MiB
// worth, at least one, at most kTlsMax.
inline int tls_limit(int c) {
    if (c > 21) return 0;
    const int n = (int)((1u << 20) >> c);
    return n < 1 ? 1 : (n > kTlsMax ? kTlsMax : n);
}

struct FreeList {
    std::mutex mu;
    std::vector<char*> items;
};

struct TlsCache {
    char* items[kNumClass][kTlsMax];
    int n[kNumClass];
};

// ------------------------------------------------------------------ HBM
struct Arena {
    std::once_flag once;
    bool ok = false;
    char* base = nullptr;
    size_t size = 0;
    hipIpcMemHandle_t handle;
    std::atomic<size_t> bump{0};
    FreeList lists[kNumClass];
    std::atomic<int64_t> live_blocks{0}, live_bytes{0}, fallbacks{0}, splits{0}, fallback_bytes{0};
};

Arena g_arena[kMaxDev];
std::atomic<void (*)()> g_reclaim{nullptr};

struct HbmTls {
    TlsCache c[kMaxDev];
    bool alive = true;
    HbmTls() { memset(c, 0, sizeof(c)); }
    ~HbmTls() {
        alive = false;
        for (int d = 0; d < kMaxDev; ++d) {
            for (int k = 0; k < kNumClass; ++k) {
                if (c[d].n[k] == 0) continue;
                std::lock_guard<std::mutex> g(g_arena[d].lists[k].mu);
                for (int i = 0; i < c[d].n[k]; ++i) g_arena[d].lists[k].items.push_back(c[d].items[k][i]);
                c[d].n[k] = 0;
            }
        }
    }
};
// The per-thread caches live on the heap behind a 16-byte TLS holder: the
// caches are 60+ KiB, and a TLS segment that small lets libmrpc use the
// initial-exec TLS model (no __tls_get_addr call per thread-local access).
template <typename T>
struct TlsHolder {
    T* p = nullptr;
    bool dead = false;
    ~TlsHolder() {
        dead = true;
        delete p;
        p = nullptr;
    }
    T* get() {
        if (!p && !dead) p = new T;
        return p;
    }
};
thread_local TlsHolder<HbmTls> tls_hbm;

bool arena_init(int device, std::string* error) {
    Arena& a = g_arena[device];
    std::call_once(a.once, [&] {
        if (Init(device, error) != 0) return;
        const size_t bytes = (size_t)std::max(64, FLAGS_hbm_arena_mb) << 20;
        void* p = Malloc(bytes, device, error);
        if (!p) return;
        int prev = 0;
        hipGetDevice(&prev);
        if (prev != device) hipSetDevice(device);
        const hipError_t r = hipIpcGetMemHandle(&a.handle, p);
        if (prev != device) hipSetDevice(prev);
        if (r != hipSuccess) {
            if (error) *error = std::string("hipIpcGetMemHandle: ") + hipGetErrorString(r);
            Free(p);
            return;
        }
        a.base = static_cast<char*>(p);
        a.size = bytes;
        a.ok = true;
    });
    if (!a.ok && error && error->empty()) *error = "HBM arena of device " + std::to_string(device) + " unavailable";
    return a.ok;
}

void hbm_block_deleter(void* p, void* arg) {
    const uint64_t v = reinterpret_cast<uint64_t>(arg);
    HbmFree(p, (size_t)(v >> 8), (int)(v & 0xff));
}

// ------------------------------------------------------------------ pinned
struct PinnedState {
    std::mutex region_mu;
    std::vector<std::pair<char*, size_t>> regions;
    char* cur = nullptr;
    size_t cur_left = 0;
    FreeList lists[kNumClass];
    std::atomic<int64_t> bytes{0};
};
PinnedState& pinned() {
    static PinnedState* s = new PinnedState;
    return *s;
}
struct PinnedTls {
    TlsCache c;
    bool alive = true;
    PinnedTls() { memset(&c, 0, sizeof(c)); }
    ~PinnedTls() {
        alive = false;
        PinnedState& ps = pinned();
        for (int k = 0; k < kNumClass; ++k) {
            if (c.n[k] == 0) continue;
            std::lock_guard<std::mutex> g(ps.lists[k].mu);
            for (int i = 0; i < c.n[k]; ++i) ps.lists[k].items.push_back(c.items[k][i]);
            c.n[k] = 0;
        }
    }
};
thread_local TlsHolder<PinnedTls> tls_pinned;
const int kPinnedMaxClass = 22;  // 4 MiB; larger pinned buffers are dedicated allocations

// Arena fully carved: cut the smallest free block of a larger class into
// blocks of class c (one returned, the rest onto c's free list) rather than
// falling back to a dedicated hipMalloc (milliseconds, not IPC-lendable,
// and its hipFree synchronises the device). Blocks are never merged back;
// a workload that moves from small to large payloads is what the arena's
// size (-hbm_arena_mb) is for.
char* split_larger(Arena& a, int c) {
    for (int k = c + 1; k <= kMaxClass; ++k) {
        char* big = nullptr;
        {
            std::lock_guard<std::mutex> g(a.lists[k].mu);
            if (a.lists[k].items.empty()) continue;
            big = a.lists[k].items.back();
            a.lists[k].items.pop_back();
        }
        const size_t sz = (size_t)1 << c;
        const size_t pieces = (size_t)1 << (k - c);
        std::lock_guard<std::mutex> g(a.lists[c].mu);
        for (size_t i = 1; i < pieces; ++i) a.lists[c].items.push_back(big + i * sz);
        a.splits.fetch_add(1, std::memory_order_relaxed);
        return big;
    }
    return nullptr;
}

}  // namespace

void SetHbmReclaimHook(void (*fn)()) { g_reclaim.store(fn, std::memory_order_release); }

int InitHbmPool(int device, std::string* error) {
    if (device < 0) device = CurrentDevice();
    if (device < 0 || device >= kMaxDev) {
        if (error) *error = "no HIP device for the HBM pool";
        return -1;
    }
    return arena_init(device, error) ? 0 : -1;
}

bool HbmPoolReady(int device) { return device >= 0 && device < kMaxDev && g_arena[device].ok; }

ArenaDesc GetArena(int device) {
    ArenaDesc d;
    if (!HbmPoolReady(device)) return d;
    const Arena& a = g_arena[device];
    d.base = a.base;
    d.size = a.size;
    d.device = device;
    d.ipc_handle.assign(reinterpret_cast<const char*>(&a.handle), sizeof(a.handle));
    return d;
}

int64_t ArenaOffset(const void* p, int device) {
    if (!HbmPoolReady(device)) return -1;
    const Arena& a = g_arena[device];
    const char* c = static_cast<const char*>(p);
    if (c < a.base || c >= a.base + a.size) return -1;
    return c - a.base;
}

void* HbmAlloc(size_t n, int device) {
    if (device < 0) device = CurrentDevice();
    if (device < 0 || device >= kMaxDev) return nullptr;
    if (n == 0) n = 1;
    const int c = class_of(n);
    Arena& a = g_arena[device];
    if (c <= kMaxClass && arena_init(device, nullptr)) {
        char* p = nullptr;
        HbmTls* t = tls_hbm.get();
        if (t && t->alive && t->c[device].n[c] > 0) {
            p = t->c[device].items[c][--t->c[device].n[c]];
        } else {
            {
                std::lock_guard<std::mutex> g(a.lists[c].mu);
                if (!a.lists[c].items.empty()) {
                    p = a.lists[c].items.back();
                    a.lists[c].items.pop_back();
                }
            }
            if (!p) {
                const size_t sz = (size_t)1 << c;
                size_t off = a.bump.load(std::memory_order_relaxed);
                while (off + sz <= a.size && !a.bump.compare_exchange_weak(off, off + sz, std::memory_order_relaxed)) {
                }
                if (off + sz <= a.size) p = a.base + off;
            }
            if (!p) p = split_larger(a, c);
            if (!p) {
                // before a dedicated allocation: let the transports give
                // back what their peers already released, then look again
                void (*reclaim)() = g_reclaim.load(std::memory_order_acquire);
                if (reclaim) {
                    reclaim();
                    {
                        std::lock_guard<std::mutex> g(a.lists[c].mu);
                        if (!a.lists[c].items.empty()) {
                            p = a.lists[c].items.back();
                            a.lists[c].items.pop_back();
                        }
                    }
                    if (!p) p = split_larger(a, c);
                }
            }
        }
        if (p) {
            a.live_blocks.fetch_add(1, std::memory_order_relaxed);
            a.live_bytes.fetch_add((int64_t)1 << c, std::memory_order_relaxed);
            return p;
        }
    }
    // arena exhausted (or a block above 256 MiB): a dedicated allocation,
    // bounded so a leak or a burst cannot take the whole GPU
    const int64_t cap = (int64_t)FLAGS_hbm_fallback_max_mb << 20;
    if (a.fallback_bytes.fetch_add((int64_t)n, std::memory_order_relaxed) + (int64_t)n > cap) {
        a.fallback_bytes.fetch_sub((int64_t)n, std::memory_order_relaxed);
        LOG_EVERY_SECOND(ERROR) << "HBM arena of device " << device << " exhausted and " << FLAGS_hbm_fallback_max_mb
                                << " MiB of dedicated allocations in use: refusing " << n << " bytes";
        return nullptr;
    }
    a.fallbacks.fetch_add(1, std::memory_order_relaxed);
    LOG_EVERY_SECOND(WARNING) << "HBM arena of device " << device << " exhausted (" << a.live_bytes.load()
                              << " bytes live): dedicated allocation of " << n << " bytes";
    void* p = Malloc(n, device);
    if (!p) a.fallback_bytes.fetch_sub((int64_t)n, std::memory_order_relaxed);
    return p;
}

void HbmFree(void* p, size_t n, int device) {
    if (!p) return;
    if (ArenaOffset(p, device) < 0) {
        Free(p);
        if (device >= 0 && device < kMaxDev) g_arena[device].fallback_bytes.fetch_sub((int64_t)n, std::memory_order_relaxed);
        return;
    }
    if (n == 0) n = 1;
    const int c = class_of(n);
    Arena& a = g_arena[device];
    a.live_blocks.fetch_sub(1, std::memory_order_relaxed);
    a.live_bytes.fetch_sub((int64_t)1 << c, std::memory_order_relaxed);
    HbmTls* t = tls_hbm.get();
    if (t && t->alive && t->c[device].n[c] < tls_limit(c)) {
        t->c[device].items[c][t->c[device].n[c]++] = static_cast<char*>(p);
        return;
    }
    std::lock_guard<std::mutex> g(a.lists[c].mu);
    a.lists[c].items.push_back(static_cast<char*>(p));
}

void* AppendNewDeviceBlock(Buf* b, size_t n, int device) {
    if (device < 0) device = CurrentDevice();
    void* p = HbmAlloc(n, device);
    if (!p) return nullptr;
    const uint64_t arg = ((uint64_t)n << 8) | (uint64_t)(device & 0xff);
    if (b->append_user_data(p, n, hbm_block_deleter, reinterpret_cast<void*>(arg), MemKind::DEVICE, device) != 0) {
        HbmFree(p, n, device);
        return nullptr;
    }
    return p;
}

HbmPoolStats GetHbmPoolStats(int device) {
    HbmPoolStats s;
    if (device < 0 || device >= kMaxDev) return s;
    const Arena& a = g_arena[device];
    s.arena_bytes = (int64_t)a.size;
    s.carved_bytes = (int64_t)a.bump.load(std::memory_order_relaxed);
    s.live_blocks = a.live_blocks.load(std::memory_order_relaxed);
    s.live_bytes = a.live_bytes.load(std::memory_order_relaxed);
    s.fallback_allocs = a.fallbacks.load(std::memory_order_relaxed);
    s.splits = a.splits.load(std::memory_order_relaxed);
    return s;
}

// ------------------------------------------------------------------ pinned
void* PinnedAlloc(size_t n) {
    if (n == 0) n = 1;
    const int c = class_of(n);
    PinnedState& ps = pinned();
    if (c > kPinnedMaxClass) {
        void* p = HostMallocPinned(n);
        if (p) ps.bytes.fetch_add((int64_t)n, std::memory_order_relaxed);
        return p;
    }
    PinnedTls* t = tls_pinned.get();
    if (t && t->alive && t->c.n[c] > 0) return t->c.items[c][--t->c.n[c]];
    {
        std::lock_guard<std::mutex> g(ps.lists[c].mu);
        if (!ps.lists[c].items.empty()) {
            char* p = ps.lists[c].items.back();
            ps.lists[c].items.pop_back();
            return p;
        }
    }
    const size_t sz = (size_t)1 << c;
    std::lock_guard<std::mutex> g(ps.region_mu);
    if (ps.cur_left < sz) {
        const size_t rbytes = std::max(sz, (size_t)std::max(1, FLAGS_pinned_region_mb) << 20);
        char* r = static_cast<char*>(HostMallocPinned(rbytes));
        if (!r) return nullptr;
        ps.regions.emplace_back(r, rbytes);
        ps.bytes.fetch_add((int64_t)rbytes, std::memory_order_relaxed);
        ps.cur = r;
        ps.cur_left = rbytes;
    }
    char* p = ps.cur;
    ps.cur += sz;
    ps.cur_left -= sz;
    return p;
}

void PinnedFree(void* p, size_t n) {
    if (!p) return;
    if (n == 0) n = 1;
    const int c = class_of(n);
    PinnedState& ps = pinned();
    if (c > kPinnedMaxClass) {
        HostFreePinned(p);
        ps.bytes.fetch_sub((int64_t)n, std::memory_order_relaxed);
        return;
    }
    PinnedTls* t = tls_pinned.get();
    if (t && t->alive && t->c.n[c] < tls_limit(c)) {
        t->c.items[c][t->c.n[c]++] = static_cast<char*>(p);
        return;
    }
    std::lock_guard<std::mutex> g(ps.lists[c].mu);
    ps.lists[c].items.push_back(static_cast<char*>(p));
}

int64_t PinnedBytes() { return pinned().bytes.load(std::memory_order_relaxed); }

}  // namespace gpu
}  // namespace mrpc
