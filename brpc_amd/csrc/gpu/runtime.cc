#include "gpu/gpu.h"

#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <sys/prctl.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <vector>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "fiber/butex.h"
#include "fiber/fiber.h"
#include "gpu/hbm_pool.h"
#include "gpu/kernels.h"
#include "rdma/rdma.h"

DEFINE_bool(pinned_coherent, true,
            "allocate pinned host memory coherent (fine-grained, not cached in the GPU L2); false: non-coherent "
            "(cached), which is only safe when kernels never re-read recycled pinned blocks");
DEFINE_int32(gpu_streams_per_device, 4, "HIP streams per device in the pool (<= GPU_MAX_HW_QUEUES)");
DEFINE_int32(gpu_poller_spin_us, 50, "event poller busy-polls this long after the last completion before backing off");
DEFINE_int32(gpu_poller_wait_pct, 50,
             "the event poller sleeps until the oldest in-flight event reached this share of the recent "
             "hand-over-to-completion time before polling (0: poll continuously)");
DEFINE_int32(gpu_poller_sleep_us, 2, "event poller sleep between polls once the spin budget is spent");
DEFINE_int32(gpu_poller_codec_wait_pct, 0,
             "-gpu_poller_wait_pct for codec-batch events (0: poll them continuously: a device-body RPC waits "
             "on four codec batches in a row, and the nap before each completion was measured on its latency)");
DEFINE_int32(gpu_poller_codec_idle_spin_us, 100,
             "after a codec batch completed, an idle event poller watches for the next one this long before "
             "sleeping on its condvar (codec streams hand over a batch every few tens of microseconds)");
DEFINE_int32(gpu_done_word_fallback_ms, 50,
             "a launch whose completion word is this overdue is completed by its event instead (a failed launch "
             "never stores the word)");
DEFINE_int32(gpu_done_word_slots, 4096, "completion-word slots per device (launches in flight with a word)");
DEFINE_int32(gpu_poller_idle_spin_us, 0,
             "with nothing in flight the event poller watches for new events this long before sleeping "
             "(saves a condvar wake-up per batch on busy RPC streams; costs that much CPU per idle period)");

namespace mrpc {
namespace gpu {

namespace {

const int kMaxDevices = 64;

struct DeviceState {
    std::once_flag once;
    int ok = 0;
    std::vector<hipStream_t> streams;
    std::atomic<uint32_t> rr{0};
};

DeviceState g_dev[kMaxDevices];
std::atomic<int> g_count{-1};

// ---- event pool
std::mutex g_ev_mu;
std::vector<hipEvent_t> g_ev_free;

hipEvent_t get_event() {
    {
        std::lock_guard<std::mutex> g(g_ev_mu);
        if (!g_ev_free.empty()) {
            hipEvent_t e = g_ev_free.back();
            g_ev_free.pop_back();
            return e;
        }
    }
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    return e;
}

void put_event(hipEvent_t e) {
    std::lock_guard<std::mutex> g(g_ev_mu);
    g_ev_free.push_back(e);
}

// ---- completion poller: fibers park on a butex, one pthread polls events.
// The poller stores 1 (completed) or -1 (failed) into *butex and wakes
// every fiber/pthread parked on it, so one event can release a whole batch.
struct Waiter {
    hipEvent_t ev;
    std::atomic<int>* butex;
    int64_t* done_us;  // optional: when the poller saw the event complete
    // resident-worker batches [first, last] instead of an event
    ResidentRing* ring = nullptr;
    uint64_t first = 0, last = 0;
    // completion-word launches: done when *word == first
    const uint64_t* word = nullptr;
    bool* fell_back = nullptr;
    int64_t since_us = 0;
    int64_t added_us = 0;  // when the poller was handed the event
    int cls = kEventOther;  // EventClass: whose completion-time average applies
};

class EventPoller {
public:
    void add(const Waiter& w) {
        bool wake;
        {
            std::unique_lock<std::mutex> g(_mu);
            if (!_started) {
                _started = true;
                pthread_create(&_th, nullptr, &EventPoller::run, this);
            }
            _incoming.push_back(w);
            _incoming.back().added_us = now_us();
            _nincoming.store(1, std::memory_order_release);
            wake = _sleeping;
        }
        // only a sleeping poller needs the futex wake; a polling or
        // idle-spinning one sees _nincoming
        if (wake) _cv.notify_one();
    }
    int64_t polled() const { return _polled.load(std::memory_order_relaxed); }

private:
    static void* run(void* arg) {
        pthread_setname_np(pthread_self(), "gpu_poller");
        // the back-off sleeps are a few microseconds: without this the
        // kernel rounds each one up to the default 50 us timer slack
        prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);
        static_cast<EventPoller*>(arg)->loop();
        return nullptr;
    }
    static int64_t now_us() {
        timespec now;
        clock_gettime(CLOCK_MONOTONIC, &now);
        return now.tv_sec * 1000000LL + now.tv_nsec / 1000;
    }
    void loop() {
        std::vector<Waiter> active;
        int64_t last_progress_us = 0;
        int64_t last_codec_done_us = INT64_MIN / 2;
        for (;;) {
            bool progressed = false;
            if (active.empty()) {
                // idle: keep watching for new work a little while before
                // sleeping — the next batch of a busy RPC stream is usually
                // microseconds away, and a condvar wake-up costs a kernel
                // round trip (and a CPU idle exit) per batch
                const int64_t t0 = now_us();
                int spin = std::max(0, FLAGS_gpu_poller_idle_spin_us);
                if (t0 - last_codec_done_us < 1000) spin = std::max(spin, FLAGS_gpu_poller_codec_idle_spin_us);
                const int64_t until = t0 + spin;
                while (!_nincoming.load(std::memory_order_acquire) && now_us() < until) {
                    for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
                }
            }
            {
                std::unique_lock<std::mutex> g(_mu);
                if (active.empty() && _incoming.empty()) {
                    _sleeping = true;
                    _cv.wait(g, [&] { return !_incoming.empty(); });
                    _sleeping = false;
                }
                progressed = !_incoming.empty();
                active.insert(active.end(), _incoming.begin(), _incoming.end());
                _incoming.clear();
                _nincoming.store(0, std::memory_order_relaxed);
            }
            const size_t before = active.size();
            size_t keep = 0;
            int64_t now_pass = 0;
            for (size_t i = 0; i < active.size(); ++i) {
                hipError_t r;
                if (active[i].word) {
                    if (__atomic_load_n(active[i].word, __ATOMIC_ACQUIRE) == active[i].first) {
                        r = hipSuccess;
                    } else {
                        if (!now_pass) now_pass = monotonic_us();
                        r = hipErrorNotReady;
                        if (active[i].ev &&
                            now_pass - active[i].added_us > (int64_t)FLAGS_gpu_done_word_fallback_ms * 1000) {
                            // overdue: the event decides (a failed launch)
                            r = hipEventQuery(active[i].ev);
                            if (r != hipErrorNotReady && active[i].fell_back) *active[i].fell_back = true;
                        }
                    }
                    if (r == hipErrorNotReady) {
                        active[keep++] = active[i];
                        continue;
                    }
                } else if (active[i].ring) {
                    // plain reads of the ring's pinned done words
                    if (!ResidentDone(active[i].ring, active[i].first, active[i].last)) {
                        if (!now_pass) now_pass = monotonic_us();
                        if (now_pass - active[i].since_us > 2000) {  // watchdog: no instance consuming?
                            ResidentKick(active[i].ring);
                            active[i].since_us = now_pass;
                        }
                        active[keep++] = active[i];
                        continue;
                    }
                    r = hipSuccess;
                } else {
                    r = hipEventQuery(active[i].ev);
                }
                if (r == hipErrorNotReady) {
                    active[keep++] = active[i];
                    continue;
                }
                {
                    const int64_t t = now_us();
                    if (active[i].done_us) *active[i].done_us = t;
                    if (active[i].cls == kEventCodec) last_codec_done_us = t;
                    // how long events take from hand-over to completion
                    const int64_t took = t - active[i].added_us;
                    int64_t& ema = _ema_us[active[i].cls];
                    if (took > 0 && took < 100000) ema += (took - ema) / 8;
                }
                active[i].butex->store(r == hipSuccess ? 1 : -1, std::memory_order_release);
                // queue the woken fibers without signalling; one signal for
                // the whole pass below (fewer futex wake-ups of idle workers)
                fiber::butex_wake_all(active[i].butex, /*nosignal=*/true);
                _polled.fetch_add(1, std::memory_order_relaxed);
            }
            if (keep != before) fiber::flush();
            active.resize(keep);
            if (keep != before) progressed = true;
            if (!active.empty()) {
                const int64_t t = now_us();
                if (progressed) last_progress_us = t;
                // nothing can be due before the oldest event reached a share
                // of the typical completion time: sleep until then instead of
                // calling hipEventQuery in a loop (each call walks the HIP
                // runtime's thread-locals and locks; a spinning poller was a
                // full host core under codec load)
                // Each event is due at its hand-over plus a share of ITS
                // class's typical completion time; the earliest due event
                // sets the nap (one global average let a short
                // copy behind long codec batches wait up to 200 us).
                int64_t due = INT64_MAX, shortest = INT64_MAX;
                bool eager = false;  // an event whose class polls continuously (wait share 0)
                for (const Waiter& w : active) {
                    const int64_t ema = _ema_us[w.cls];
                    const int pct = w.cls == kEventCodec ? FLAGS_gpu_poller_codec_wait_pct : FLAGS_gpu_poller_wait_pct;
                    eager |= pct <= 0;
                    due = std::min(due, w.added_us + ema * std::max(0, pct) / 100);
                    shortest = std::min(shortest, ema);
                }
                int64_t sleep_us = 0;
                if (!eager && due - t >= 8) {
                    sleep_us = std::min<int64_t>(due - t, 200);
                } else if (!eager && !progressed && shortest >= 20) {
                    // only long events pending (codec batches, large pulls):
                    // one pass per ~tenth of the shortest class's duration
                    sleep_us = std::max<int64_t>(2, std::min<int64_t>(shortest / 10, 10));
                } else if (t - last_progress_us > FLAGS_gpu_poller_spin_us) {
                    sleep_us = std::max(1, FLAGS_gpu_poller_sleep_us);
                }
                if (sleep_us) {
                    timespec ts{0, 1000L * sleep_us};
                    nanosleep(&ts, nullptr);
                }
            }
        }
    }

    std::mutex _mu;
    std::condition_variable _cv;
    std::vector<Waiter> _incoming;
    std::atomic<int> _nincoming{0};
    bool _sleeping = false;
    bool _started = false;
    pthread_t _th;
    std::atomic<int64_t> _polled{0};
    int64_t _ema_us[kEventClasses] = {};  // hand-over to completion per EventClass (poller thread only)
};

EventPoller* poller() {
    static EventPoller* p = new EventPoller;
    return p;
}

int copy_hook(void* dst, const void* src, size_t n, MemKind kind, int device) {
    (void)kind;
    return CopyDeviceToHost(dst, src, n, device);
}

int check_device(int device) {
    if (device < 0) device = CurrentDevice();
    if (device < 0 || device >= kMaxDevices || device >= DeviceCount()) return -1;
    return device;
}

}  // namespace

int DeviceCount() {
    int c = g_count.load(std::memory_order_acquire);
    if (c >= 0) return c;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    g_count.store(n, std::memory_order_release);
    return n;
}

bool Available() { return DeviceCount() > 0; }

int CurrentDevice() {
    if (!Available()) return -1;
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) return -1;
    return d;
}

// GPUDirect RDMA: export an HBM range as a dmabuf fd for ibv_reg_dmabuf_mr.
int dmabuf_export_hook(void* p, size_t n, int gpu, int* fd, uint64_t* offset) {
    (void)gpu;
    const uintptr_t page = 4096;
    const uintptr_t base = reinterpret_cast<uintptr_t>(p) & ~(page - 1);
    const size_t len = ((reinterpret_cast<uintptr_t>(p) + n + page - 1) & ~(page - 1)) - base;
    int h = -1;
    if (hipMemGetHandleForAddressRange(&h, reinterpret_cast<hipDeviceptr_t>(base), len,
                                       hipMemRangeHandleTypeDmaBufFd, 0) != hipSuccess) {
        return -1;
    }
    *fd = h;
    *offset = reinterpret_cast<uintptr_t>(p) - base;
    return 0;
}

int Init(int device, std::string* error) {
    device = check_device(device);
    if (device < 0) {
        if (error) *error = "no HIP device available";
        return -1;
    }
    DeviceState& st = g_dev[device];
    std::call_once(st.once, [&] {
        int prev = 0;
        hipGetDevice(&prev);
        if (hipSetDevice(device) != hipSuccess) return;
        const int ns = std::max(1, std::min(FLAGS_gpu_streams_per_device, 4));
        for (int i = 0; i < ns; ++i) {
            hipStream_t s = nullptr;
            if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) break;
            st.streams.push_back(s);
        }
        hipSetDevice(prev);
        st.ok = st.streams.empty() ? 0 : 1;
        SetDeviceCopyHook(copy_hook);
        rdma::SetDmabufExportHook(dmabuf_export_hook);
    });
    if (!st.ok) {
        if (error) *error = "fail to initialise HIP device " + std::to_string(device);
        return -1;
    }
    return 0;
}

std::string DeviceName(int device) {
    hipDeviceProp_t p;
    if (check_device(device) < 0 || hipGetDeviceProperties(&p, device) != hipSuccess) return "";
    return p.name;
}

std::string DeviceArch(int device) {
    hipDeviceProp_t p;
    if (check_device(device) < 0 || hipGetDeviceProperties(&p, device) != hipSuccess) return "";
    std::string a = p.gcnArchName;
    const size_t colon = a.find(':');
    return colon == std::string::npos ? a : a.substr(0, colon);
}

std::string PciBusId(int device) {
    char id[64] = {0};
    if (check_device(device) < 0 || hipDeviceGetPCIBusId(id, sizeof(id) - 1, device) != hipSuccess) return "";
    std::string s = id;
    for (char& c : s) c = (char)tolower((unsigned char)c);
    return s;
}

hipStream_t PoolStream(int device) {
    device = check_device(device);
    if (device < 0 || Init(device) != 0) return nullptr;
    DeviceState& st = g_dev[device];
    return st.streams[st.rr.fetch_add(1, std::memory_order_relaxed) % st.streams.size()];
}

int WaitEvent(hipEvent_t ev) {
    hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return 0;
    if (q != hipErrorNotReady) return -1;
    if (fiber::worker_index() < 0) {
        return hipEventSynchronize(ev) == hipSuccess ? 0 : -1;
    }
    std::atomic<int>* b = fiber::butex_create();
    b->store(0, std::memory_order_relaxed);
    poller()->add(Waiter{ev, b});
    while (b->load(std::memory_order_acquire) == 0) fiber::butex_wait(b, 0);
    const int v = b->load(std::memory_order_acquire);
    fiber::butex_destroy(b);
    return v == 1 ? 0 : -1;
}

void WatchEvent(hipEvent_t ev, std::atomic<int>* butex, int64_t* done_us, int cls) {
    Waiter w{ev, butex, done_us};
    w.cls = cls >= 0 && cls < kEventClasses ? cls : kEventOther;
    poller()->add(w);
}

void WatchResident(ResidentRing* ring, uint64_t first_seq, uint64_t last_seq, std::atomic<int>* butex,
                   int64_t* done_us) {
    Waiter w{nullptr, butex, done_us};
    w.ring = ring;
    w.first = first_seq;
    w.last = last_seq;
    w.since_us = monotonic_us();
    w.cls = kEventCopy;
    poller()->add(w);
}

void WatchWord(const uint64_t* word, uint64_t seq, hipEvent_t ev, std::atomic<int>* butex, int64_t* done_us,
               int cls, bool* fell_back) {
    Waiter w{ev, butex, done_us};
    w.word = word;
    w.first = seq;
    w.fell_back = fell_back;
    w.cls = cls >= 0 && cls < kEventClasses ? cls : kEventOther;
    poller()->add(w);
}

namespace {
// Completion-word slots per device: counters in HBM (zero between
// launches: every launch's last workgroup resets its own), words in pinned
// coherent host memory. Sequence numbers only grow, so a word never
// matches a later launch's seq by accident.
struct DoneSlots {
    std::mutex mu;
    bool init = false, ok = false;
    uint32_t* counters = nullptr;
    uint64_t* words = nullptr;
    std::vector<uint32_t> free;
    uint64_t next_seq = 0;
};
DoneSlots g_done[kMaxDevices];
}  // namespace

bool AcquireDoneWord(int device, DoneWord* out, uint32_t* slot) {
    if (device < 0 || device >= kMaxDevices) return false;
    DoneSlots& d = g_done[device];
    std::lock_guard<std::mutex> g(d.mu);
    if (!d.init) {
        d.init = true;
        const uint32_t n = (uint32_t)std::max(64, FLAGS_gpu_done_word_slots);
        int prev = 0;
        hipGetDevice(&prev);
        if (prev != device) hipSetDevice(device);
        void* c = nullptr;
        if (hipMalloc(&c, n * sizeof(uint32_t)) == hipSuccess && hipMemset(c, 0, n * sizeof(uint32_t)) == hipSuccess &&
            hipDeviceSynchronize() == hipSuccess) {
            d.counters = static_cast<uint32_t*>(c);
            d.words = static_cast<uint64_t*>(HostMallocPinned(n * 4 * sizeof(uint64_t)));
        }
        if (prev != device) hipSetDevice(prev);
        if (d.counters && d.words) {
            memset(d.words, 0, n * 4 * sizeof(uint64_t));
            for (uint32_t i = n; i > 0; --i) d.free.push_back(i - 1);
            d.ok = true;
        }
    }
    if (!d.ok || d.free.empty()) return false;
    const uint32_t s = d.free.back();
    d.free.pop_back();
    *slot = s;
    out->counter = d.counters + s;
    out->word = d.words + 4 * (size_t)s;  // [word, kernel start, kernel end, -] (GPU wall clock)
    out->seq = ++d.next_seq;
    return true;
}

void ReleaseDoneWord(int device, uint32_t slot) {
    DoneSlots& d = g_done[device];
    std::lock_guard<std::mutex> g(d.mu);
    d.free.push_back(slot);
}

hipEvent_t AcquireEvent() { return get_event(); }
void ReleaseEvent(hipEvent_t e) {
    if (e) put_event(e);
}

int SyncStream(hipStream_t s) {
    hipEvent_t e = get_event();
    if (!e) return -1;
    int rc = -1;
    if (hipEventRecord(e, s) == hipSuccess) rc = WaitEvent(e);
    put_event(e);
    return rc;
}

int64_t PolledEvents() { return poller()->polled(); }

void* Malloc(size_t n, int device, std::string* error) {
    device = check_device(device);
    if (device < 0) {
        if (error) *error = "no HIP device available";
        return nullptr;
    }
    int prev = 0;
    hipGetDevice(&prev);
    if (prev != device) hipSetDevice(device);
    void* p = nullptr;
    hipError_t r = hipMalloc(&p, n ? n : 1);
    if (prev != device) hipSetDevice(prev);
    if (r != hipSuccess) {
        if (error) *error = std::string("hipMalloc failed: ") + hipGetErrorString(r);
        return nullptr;
    }
    return p;
}

void Free(void* p) {
    if (p) hipFree(p);
}

// Pinned host memory is COHERENT (fine-grained), whatever HIP_HOST_COHERENT
// says. The pool recycles blocks: a socket block whose earlier bytes a
// kernel read is refilled by recv() and read by the next kernel. With
// non-coherent memory the GPU's L2 may still hold the old lines, and
// kernels on one queue are dispatched with agent-scope acquires that do
// not invalidate them, so the next kernel reads stale bytes. Measured: the
// GPU-handler leg returned device CRC32Cs of stale data (226 of ~4.7k
// checked replies, profiles/r4_bench_handler_crc_mismatch_repro.json) and
// none with coherent memory, at the same throughput.
void* HostMallocPinned(size_t n) {
    void* p = nullptr;
    const unsigned flags = FLAGS_pinned_coherent ? (hipHostMallocCoherent | hipHostMallocMapped)
                                                 : (hipHostMallocNonCoherent | hipHostMallocMapped);
    if (hipHostMalloc(&p, n, flags) != hipSuccess) return nullptr;
    return p;
}

void HostFreePinned(void* p) {
    if (p) hipHostFree(p);
}

// Socket blocks come from the pinned slab pool (gpu/hbm_pool.cc); the
// pool never falls back to pageable memory, so the kind tag stays true.
static void* pinned_alloc(size_t n) { return PinnedAlloc(n); }
static void pinned_dealloc(void* p, size_t n) { PinnedFree(p, n); }

int UsePinnedBlocks() {
    if (!Available()) return -1;
    static std::once_flag once;
    std::call_once(once, [] { SetBlockMemAllocator(BlockMemAllocator{pinned_alloc, pinned_dealloc, MemKind::PINNED}); });
    return 0;
}

bool PinnedBlocksInUse() { return GetBlockMemAllocator().kind == MemKind::PINNED; }

static int copy_impl(void* dst, const void* src, size_t n, hipMemcpyKind kind, int device) {
    if (n == 0) return 0;
    hipStream_t s = PoolStream(device);
    if (!s) return -1;
    if (hipMemcpyAsync(dst, src, n, kind, s) != hipSuccess) return -1;
    return SyncStream(s);
}

int CopyHostToDevice(void* dst, const void* src, size_t n, int device) {
    return copy_impl(dst, src, n, hipMemcpyHostToDevice, device);
}
int CopyDeviceToHost(void* dst, const void* src, size_t n, int device) {
    return copy_impl(dst, src, n, hipMemcpyDeviceToHost, device);
}
int CopyDeviceToDevice(void* dst, const void* src, size_t n, int device) {
    return copy_impl(dst, src, n, hipMemcpyDeviceToDevice, device);
}

int Memset(void* dst, int value, size_t n, int device) {
    hipStream_t s = PoolStream(device);
    if (!s) return -1;
    if (hipMemsetAsync(dst, value, n, s) != hipSuccess) return -1;
    return SyncStream(s);
}

int AppendDevice(Buf* b, void* dev, size_t n, int device, void (*deleter)(void*, void*), void* arg) {
    if (device < 0) device = CurrentDevice();
    return b->append_user_data(dev, n, deleter, arg, MemKind::DEVICE, device);
}

int AppendHostAsDevice(Buf* b, const void* data, size_t n, int device, std::string* error) {
    if (device < 0) device = CurrentDevice();
    Buf tmp;
    void* d = AppendNewDeviceBlock(&tmp, n, device);
    if (!d) {
        if (error) *error = "HBM allocation failed";
        return -1;
    }
    if (CopyHostToDevice(d, data, n, device) != 0) {
        if (error) *error = "host->device copy failed";
        return -1;
    }
    b->append(std::move(tmp));
    return 0;
}

int GatherToDevice(const Buf& in, Buf* out, int device, std::string* error) {
    if (device < 0) device = CurrentDevice();
    const size_t n = in.size();
    if (n == 0) return 0;
    if (in.backing_block_num() == 1 && in.ref_at(0).block->kind == MemKind::DEVICE &&
        in.ref_at(0).block->device == device) {
        out->append(in);
        return 0;
    }
    Buf tmp;
    char* d = static_cast<char*>(AppendNewDeviceBlock(&tmp, n, device));
    if (!d) {
        if (error) *error = "HBM allocation failed";
        return -1;
    }
    hipStream_t s = PoolStream(device);
    size_t off = 0;
    for (size_t i = 0; i < in.backing_block_num(); ++i) {
        const BlockRef& r = in.ref_at(i);
        const hipMemcpyKind k = IsHostAccessible(r.block->kind) ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
        if (hipMemcpyAsync(d + off, r.block->data + r.offset, r.length, k, s) != hipSuccess) {
            if (error) *error = "gather copy failed";
            SyncStream(s);  // earlier copies may still target d
            return -1;
        }
        off += r.length;
    }
    if (SyncStream(s) != 0) {
        if (error) *error = "gather sync failed";
        return -1;
    }
    out->append(std::move(tmp));
    return 0;
}

bool HasDeviceBlocks(const Buf& b) { return !b.all_host_accessible(); }

int CopyBufToHost(const Buf& in, std::string* out) {
    out->clear();
    out->resize(in.size());
    size_t off = 0;
    for (size_t i = 0; i < in.backing_block_num(); ++i) {
        const BlockRef& r = in.ref_at(i);
        if (IsHostAccessible(r.block->kind)) {
            memcpy(&(*out)[off], r.block->data + r.offset, r.length);
        } else if (CopyDeviceToHost(&(*out)[off], r.block->data + r.offset, r.length, r.block->device) != 0) {
            return -1;
        }
        off += r.length;
    }
    return 0;
}

}  // namespace gpu
}  // namespace mrpc
