// Sampling heap profiler (the role tcmalloc's sampler plays for the
// reference's /hotspots/heap, /hotspots/growth and /pprof/heap,
// builtin/hotspots_service.cpp + details/tcmalloc_extension.cpp).
//
// Link this object into an executable (or LD_PRELOAD libmrpc_heapprof.so):
// it interposes malloc/free/calloc/realloc/memalign & co on glibc's
// __libc_* entry points. Every thread draws the distance to its next sample
// from an exponential distribution with mean -heap_sample_bytes (env
// MRPC_HEAP_SAMPLE_BYTES, default 512 KiB), so the cost of an unsampled
// allocation is one thread-local subtraction. A sampled allocation records
// its call stack (backtrace) and is remembered in a lock-free open-addressing
// set, so free() of an unsampled pointer is one probe. The builtin pages
// find mrpc_heap_profile_text() with dlsym and print the legacy pprof heap
// format (in-use and cumulative "growth" views) plus symbolized stacks.
#include <dlfcn.h>
#include <execinfo.h>
#include <malloc.h>
#include <pthread.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

extern "C" {
void* __libc_malloc(size_t);
void __libc_free(void*);
void* __libc_calloc(size_t, size_t);
void* __libc_realloc(void*, size_t);
void* __libc_memalign(size_t, size_t);
}

namespace {

constexpr int kMaxFrames = 32;
constexpr size_t kStackSlots = 1 << 14;  // distinct sampled stacks
constexpr size_t kLiveSlots = 1 << 18;   // live sampled pointers

struct StackRec {
    std::atomic<uint64_t> hash{0};
    int depth = 0;
    void* frames[kMaxFrames];
    std::atomic<int64_t> live_count{0}, live_bytes{0}, total_count{0}, total_bytes{0};
};

struct LiveRec {
    std::atomic<uintptr_t> ptr{0};
    uint32_t stack = 0;
    int64_t bytes = 0;  // sample weight
};

StackRec* g_stacks = nullptr;
LiveRec* g_live = nullptr;
std::atomic<bool> g_ready{false};
int64_t g_mean = 512 * 1024;
pthread_mutex_t g_stack_mu = PTHREAD_MUTEX_INITIALIZER;

thread_local bool t_in_hook = false;
thread_local int64_t t_until = -1;
thread_local uint64_t t_rng = 0;

inline uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

int64_t next_gap() {
    if (t_rng == 0) t_rng = mix((uint64_t)(uintptr_t)&t_rng ^ (uint64_t)getpid() ^ 0x9e3779b97f4a7c15ull);
    t_rng = mix(t_rng + 0x9e3779b97f4a7c15ull);
    const double u = ((t_rng >> 11) + 0.5) * (1.0 / 9007199254740992.0);
    return (int64_t)(-std::log(u) * (double)g_mean) + 1;
}

void init_once() {
    static std::atomic<int> state{0};
    int expect = 0;
    if (!state.compare_exchange_strong(expect, 1)) return;
    t_in_hook = true;
    if (const char* e = getenv("MRPC_HEAP_SAMPLE_BYTES")) {
        const long long v = atoll(e);
        if (v > 0) g_mean = v;
    }
    g_stacks = static_cast<StackRec*>(__libc_calloc(kStackSlots, sizeof(StackRec)));
    g_live = static_cast<LiveRec*>(__libc_calloc(kLiveSlots, sizeof(LiveRec)));
    void* warm[2];
    backtrace(warm, 2);  // the unwinder allocates on first use
    t_in_hook = false;
    g_ready.store(g_stacks && g_live, std::memory_order_release);
}

uint32_t intern_stack(void* const* frames, int depth) {
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < depth; ++i) h = mix(h ^ (uint64_t)(uintptr_t)frames[i]);
    if (h == 0) h = 1;
    for (size_t probe = 0; probe < kStackSlots; ++probe) {
        const uint32_t slot = (uint32_t)((h + probe) & (kStackSlots - 1));
        StackRec& r = g_stacks[slot];
        const uint64_t cur = r.hash.load(std::memory_order_acquire);
        if (cur == h) return slot;
        if (cur == 0) {
            pthread_mutex_lock(&g_stack_mu);
            if (r.hash.load(std::memory_order_relaxed) == 0) {
                r.depth = depth;
                memcpy(r.frames, frames, sizeof(void*) * depth);
                r.hash.store(h, std::memory_order_release);
            }
            const bool mine = r.hash.load(std::memory_order_relaxed) == h;
            pthread_mutex_unlock(&g_stack_mu);
            if (mine) return slot;
        }
    }
    return 0;  // table full: charge to slot 0
}

void record(void* p, size_t n) {
    if (!p || t_in_hook) return;
    if (t_until < 0) t_until = next_gap();
    t_until -= (int64_t)n;
    if (t_until > 0) return;
    t_until = next_gap();
    if (!g_ready.load(std::memory_order_acquire)) {
        init_once();
        if (!g_ready.load(std::memory_order_acquire)) return;
    }
    t_in_hook = true;
    void* frames[kMaxFrames + 2];
    int depth = backtrace(frames, kMaxFrames + 2);
    const int skip = depth > 2 ? 2 : 0;  // record() and the malloc wrapper
    const uint32_t sid = intern_stack(frames + skip, depth - skip);
    // unbiased weight for exponential-gap sampling: an allocation of n bytes
    // is sampled with probability 1 - exp(-n/mean), so it stands for
    // n / (1 - exp(-n/mean)) bytes (tends to max(n, mean) at both ends)
    const double q = 1.0 - std::exp(-(double)n / (double)g_mean);
    const int64_t weight = q > 0 ? (int64_t)((double)n / q + 0.5) : g_mean;
    StackRec& sr = g_stacks[sid];
    sr.live_count.fetch_add(1, std::memory_order_relaxed);
    sr.live_bytes.fetch_add(weight, std::memory_order_relaxed);
    sr.total_count.fetch_add(1, std::memory_order_relaxed);
    sr.total_bytes.fetch_add(weight, std::memory_order_relaxed);
    const uint64_t h = mix((uint64_t)(uintptr_t)p);
    for (size_t probe = 0; probe < 64; ++probe) {
        LiveRec& lr = g_live[(h + probe) & (kLiveSlots - 1)];
        uintptr_t zero = 0;
        if (lr.ptr.load(std::memory_order_relaxed) == 0 &&
            lr.ptr.compare_exchange_strong(zero, (uintptr_t)1, std::memory_order_acq_rel)) {
            lr.stack = sid;
            lr.bytes = weight;
            lr.ptr.store((uintptr_t)p, std::memory_order_release);
            break;
        }
    }
    t_in_hook = false;
}

void forget(void* p) {
    if (!p || !g_ready.load(std::memory_order_acquire)) return;
    const uint64_t h = mix((uint64_t)(uintptr_t)p);
    for (size_t probe = 0; probe < 64; ++probe) {
        LiveRec& lr = g_live[(h + probe) & (kLiveSlots - 1)];
        uintptr_t cur = lr.ptr.load(std::memory_order_acquire);
        if (cur == (uintptr_t)p && lr.ptr.compare_exchange_strong(cur, (uintptr_t)1, std::memory_order_acq_rel)) {
            StackRec& sr = g_stacks[lr.stack];
            sr.live_count.fetch_sub(1, std::memory_order_relaxed);
            sr.live_bytes.fetch_sub(lr.bytes, std::memory_order_relaxed);
            lr.ptr.store(0, std::memory_order_release);
            return;
        }
    }
}

}  // namespace

extern "C" {

void* malloc(size_t n) {
    void* p = __libc_malloc(n);
    record(p, n);
    return p;
}
void free(void* p) {
    forget(p);
    __libc_free(p);
}
void* calloc(size_t a, size_t b) {
    void* p = __libc_calloc(a, b);
    record(p, a * b);
    return p;
}
void* realloc(void* old, size_t n) {
    void* p = __libc_realloc(old, n);
    // a failed realloc leaves `old` live (and tracked); realloc(p, 0) frees
    if (p || n == 0) forget(old);
    record(p, n);
    return p;
}
void* memalign(size_t al, size_t n) {
    void* p = __libc_memalign(al, n);
    record(p, n);
    return p;
}
void* aligned_alloc(size_t al, size_t n) { return memalign(al, n); }
int posix_memalign(void** out, size_t al, size_t n) {
    void* p = __libc_memalign(al, n);
    if (!p) return ENOMEM;
    record(p, n);
    *out = p;
    return 0;
}

// Legacy pprof heap profile ("heap profile: ..." + MAPPED_LIBRARIES), the
// in-use view, or cumulative allocations when growth != 0. The caller frees
// the returned string with free().
char* mrpc_heap_profile_text(int growth) {
    init_once();
    if (!g_ready.load(std::memory_order_acquire)) return nullptr;
    const bool saved = t_in_hook;
    t_in_hook = true;
    size_t cap = 1 << 16, len = 0;
    char* out = static_cast<char*>(__libc_malloc(cap));
    auto append = [&](const char* s, size_t n) {
        if (len + n + 1 > cap) {
            while (len + n + 1 > cap) cap *= 2;
            out = static_cast<char*>(__libc_realloc(out, cap));
        }
        memcpy(out + len, s, n);
        len += n;
        out[len] = 0;
    };
    int64_t c = 0, b = 0, tc = 0, tb = 0;
    for (size_t i = 0; i < kStackSlots; ++i) {
        StackRec& r = g_stacks[i];
        if (!r.hash.load(std::memory_order_acquire)) continue;
        c += r.live_count.load();
        b += r.live_bytes.load();
        tc += r.total_count.load();
        tb += r.total_bytes.load();
    }
    char line[512];
    int k = snprintf(line, sizeof(line), "heap profile: %lld: %lld [%lld: %lld] @ %s/%lld\n", (long long)(growth ? tc : c),
                     (long long)(growth ? tb : b), (long long)tc, (long long)tb, growth ? "growthz" : "heap_v2",
                     (long long)g_mean);
    append(line, (size_t)k);
    for (size_t i = 0; i < kStackSlots; ++i) {
        StackRec& r = g_stacks[i];
        if (!r.hash.load(std::memory_order_acquire)) continue;
        const long long lc = growth ? r.total_count.load() : r.live_count.load();
        const long long lb = growth ? r.total_bytes.load() : r.live_bytes.load();
        if (lc <= 0) continue;
        k = snprintf(line, sizeof(line), "%lld: %lld [%lld: %lld] @", lc, lb, (long long)r.total_count.load(),
                     (long long)r.total_bytes.load());
        append(line, (size_t)k);
        for (int f = 0; f < r.depth; ++f) {
            k = snprintf(line, sizeof(line), " %p", r.frames[f]);
            append(line, (size_t)k);
        }
        append("\n", 1);
    }
    append("\nMAPPED_LIBRARIES:\n", 19);
    if (FILE* f = fopen("/proc/self/maps", "r")) {
        size_t n;
        while ((n = fread(line, 1, sizeof(line), f)) > 0) append(line, n);
        fclose(f);
    }
    t_in_hook = saved;
    return out;
}

int64_t mrpc_heap_sample_bytes() { return g_mean; }

}  // extern "C"
