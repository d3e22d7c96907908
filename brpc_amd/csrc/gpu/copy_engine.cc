#include "gpu/copy_engine.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <vector>

#include "base/crc32c.h"
#include "base/flags.h"
#include "base/logging.h"
#include "fiber/butex.h"
#include "gpu/gpu.h"
#include "gpu/hbm_pool.h"
#include "base/time.h"
#include "base/util.h"
#include "rpc/span.h"

DEFINE_bool(copy_engine_resident, false,
            "run batches on the resident copy worker (a persistent kernel fed from a pinned ring: no launch or "
            "event per batch) instead of one kernel launch each");
DEFINE_int32(copy_engine_resident_idle_us, 200, "a resident instance exits after this long without a batch");
DEFINE_int32(copy_engine_resident_groups, 16, "workgroups of a resident instance (each polls the ring)");
DEFINE_int32(copy_engine_resident_max_us, 4000,
             "a resident instance exits after this long in any case (bounds how long work sharing its hardware "
             "queue can wait); the next batch relaunches it");

DEFINE_bool(copy_engine_done_words, false,
            "batches complete through a word the kernel's last workgroup stores into pinned memory (the poller "
            "reads it, the event stays as the fallback), with the kernel's start/end GPU clock: the diagnostic "
            "split of launch -> kernel start -> end -> seen (bench.py diag). Off by default: every workgroup's "
            "agent-scope release (an L2 write-back) halved 1 MiB pull bandwidth, and with the in-flight limit "
            "event completion is as fast (profiles/r6_xproc_diagnosis.txt)");

DEFINE_bool(copy_engine_crc_mfma, true,
            "verified pulls of at least -copy_engine_crc_mfma_min_bytes per launch fold their CRC32C on the matrix "
            "cores (copy_crc32c_mfma_kernel); false: always the byte-table kernel");
DEFINE_int64(copy_engine_crc_mfma_min_bytes, 2 << 20,
             "launch size from which verified pulls take the MFMA CRC kernel: it won on 1 MiB payload batches "
             "(135k vs 122k QPS, 57 vs 64 us per launch) and lost on 64 KiB ones (392k vs 421k, 9.9 vs 8.0 us), "
             "where the A-fragment staging and MFMA chain add latency to one-chunk workgroups "
             "(profiles/r6_crc_kernels.txt)");
DEFINE_int32(copy_engine_max_inflight, 4,
             "launches of one device's copy engine in flight at once (0: no limit). Submissions that find the "
             "limit reached join the open batch, which the first waiter of the next completed batch launches: "
             "with 50 RPCs in flight and a few workers per process, unlimited launches of ~1 segment each queued "
             "up in the HIP streams (~600 us from launch to kernel start at 2 ranks per GPU, "
             "profiles/r6_xproc_diagnosis.txt)");
DEFINE_bool(copy_engine_word_event, true,
            "launches with a completion word still record an event (the fallback verdict of a launch that "
            "never stores its word)");

namespace mrpc {
namespace gpu {

namespace {

const int kMaxDev = 16;

// One launch worth of segments. Every submitter of the batch parks on
// `butex`; the poller sets it to 1 (or -1) when the batch's event fires.
struct Batch {
    std::vector<Segment> segs;
    std::vector<int> msg_of;        // CRC message of each segment (want_crc)
    int nmsg = 0;
    bool want_crc = false;          // some submitter asked for checksums
    uint32_t* crc_host = nullptr;   // per-segment CRC32C, stored by the kernel (pinned)
    size_t crc_cap = 0;
    std::atomic<int>* butex = nullptr;
    hipEvent_t ev = nullptr;
    std::atomic<int> refs{0};
    // completion word (FLAGS_copy_engine_done_words); fell_back: the event
    // completed the batch, so the slot's counter is not known to be zero
    std::atomic<bool> retired{false};  // its in-flight slot was given back (first waiter to wake)
    bool has_word = false, fell_back = false;
    uint32_t word_slot = 0;
    const uint64_t* word = nullptr;  // the slot's pinned words (stamps at [1], [2])
    // latency breakdown (monotonic us): first submission, launch issued,
    // completion seen by the poller
    int64_t t_open = 0, t_issue_begin = 0, t_issued = 0, t_done = 0;
};

struct Engine {
    std::mutex mu;
    Batch* open = nullptr;     // batch accepting submissions
    bool launching = false;    // a leader is draining `open`
    int inflight = 0;          // launched, not yet retired (FLAGS_copy_engine_max_inflight)
    std::vector<Batch*> spare; // recycled batches
};

Engine g_engine[kMaxDev];
std::atomic<int64_t> g_submits{0}, g_launches{0}, g_segments{0}, g_bytes{0};
// sums over submissions (us): waiting for the batch to be issued, the
// launch API calls, launch-to-completion-seen, completion-to-resumed
std::atomic<int64_t> g_t_queue{0}, g_t_api{0}, g_t_gpu{0}, g_t_wake{0};
// completion-word launches: GPU wall-clock ticks from workgroup 0's start
// to the last workgroup's end, and how many launches that covers
std::atomic<int64_t> g_kernel_ticks{0}, g_kernel_timed{0};
// ... and, with the GPU clock correlated to the host's (calibrate_clock),
// launch API return -> kernel start and kernel end -> the poller saw it
std::atomic<int64_t> g_start_delay_us{0}, g_notice_us{0};
std::atomic<int64_t> g_clock_offset_us{INT64_MIN};  // host monotonic us - GPU ticks / 100

// Correlate the GPU wall clock with the host's monotonic clock: a one-lane
// kernel stores its clock into pinned memory while the host spins on it;
// of 20 probes the one seen soonest after its launch bounds the offset
// within a few microseconds.
void calibrate_clock(int device) {
    static std::once_flag once;
    std::call_once(once, [device] {
        uint64_t* w = static_cast<uint64_t*>(HostMallocPinned(64));
        hipStream_t s = PoolStream(device);
        if (!w || !s) return;
        int64_t best_win = INT64_MAX, best_off = INT64_MIN;
        for (int i = 0; i < 20; ++i) {
            __atomic_store_n(w, 0ull, __ATOMIC_RELEASE);
            const int64_t t0 = monotonic_us();
            if (LaunchClockProbe(w, s) != 0) break;
            uint64_t v = 0;
            int64_t t1 = t0;
            while ((v = __atomic_load_n(w, __ATOMIC_ACQUIRE)) == 0) {
                t1 = monotonic_us();
                if (t1 - t0 > 100000) break;
            }
            t1 = monotonic_us();
            if (v && t1 - t0 < best_win) {
                best_win = t1 - t0;
                best_off = t1 - (int64_t)(v / 100);
            }
        }
        hipStreamSynchronize(s);
        g_clock_offset_us.store(best_off, std::memory_order_relaxed);
        HostFreePinned(w);
    });
}

// One submitter per batch accounts the batch-wide stamps: the one whose
// segments come first.
inline bool leader_of_batch(const Batch*, size_t first) { return first == 0; }

Batch* new_batch(Engine& e) {
    if (!e.spare.empty()) {
        Batch* b = e.spare.back();
        e.spare.pop_back();
        return b;
    }
    Batch* b = new Batch;
    b->butex = fiber::butex_create();
    return b;
}

// Resident path: publish the batch to the device's ring; the poller reads
// its done words. false: not available (the caller launches instead).
bool submit_resident(Batch* b, int device) {
    if (!FLAGS_copy_engine_resident) return false;
    ResidentRing* ring = ResidentRingFor(device, (uint32_t)std::max(1, FLAGS_copy_engine_resident_idle_us),
                                         (uint32_t)std::max(10, FLAGS_copy_engine_resident_max_us),
                                         (uint32_t)FLAGS_copy_engine_resident_groups);
    if (!ring) return false;
    if (b->want_crc && b->crc_cap < (size_t)b->nmsg) {
        PinnedFree(b->crc_host, b->crc_cap * sizeof(uint32_t));
        b->crc_cap = std::max<size_t>((size_t)b->nmsg, 64);
        b->crc_host = static_cast<uint32_t*>(PinnedAlloc(b->crc_cap * sizeof(uint32_t)));
        if (!b->crc_host) return false;
    }
    int prev = 0;
    hipGetDevice(&prev);
    if (prev != device) hipSetDevice(device);
    uint64_t first = 0, last = 0;
    const int rc = ResidentSubmit(ring, b->segs.data(), b->want_crc ? b->msg_of.data() : nullptr, (int)b->segs.size(),
                                  b->want_crc ? b->crc_host : nullptr, &first, &last);
    b->t_issued = monotonic_us();
    if (prev != device) hipSetDevice(prev);
    g_launches.fetch_add(1, std::memory_order_relaxed);
    if (rc != 0) {
        LOG_EVERY_SECOND(ERROR) << "resident copy worker refused a batch of " << b->segs.size() << " segments";
        b->butex->store(-1, std::memory_order_release);
        fiber::butex_wake_all(b->butex);
        return true;
    }
    WatchResident(ring, first, last, b->butex, &b->t_done);
    return true;
}

// Issue one batch: kernel + event + poller registration. On failure the
// batch's waiters are released with an error.
void launch(Batch* b, int device) {
    if (submit_resident(b, device)) return;
    int prev = 0;
    hipGetDevice(&prev);
    if (prev != device) hipSetDevice(device);
    hipStream_t s = PoolStream(device);
    b->ev = AcquireEvent();
    int rc = (s && b->ev) ? 0 : -1;
    const size_t n = b->segs.size();
    DoneWord dw;
    b->fell_back = false;
    if (FLAGS_copy_engine_done_words) calibrate_clock(device);
    b->has_word = rc == 0 && FLAGS_copy_engine_done_words && AcquireDoneWord(device, &dw, &b->word_slot);
    const DoneWord* done = b->has_word ? &dw : nullptr;
    b->word = b->has_word ? dw.word : nullptr;
    if (rc == 0 && b->want_crc) {
        // fused pull + checksum: the kernel stores the CRCs straight into
        // pinned host memory (one launch, no memset, no D2H copy)
        if (b->crc_cap < (size_t)b->nmsg) {
            PinnedFree(b->crc_host, b->crc_cap * sizeof(uint32_t));
            b->crc_cap = std::max<size_t>((size_t)b->nmsg, 64);
            b->crc_host = static_cast<uint32_t*>(PinnedAlloc(b->crc_cap * sizeof(uint32_t)));
        }
        uint64_t launch_bytes = 0;
        for (const Segment& g : b->segs) launch_bytes += g.len;
        const bool mfma = FLAGS_copy_engine_crc_mfma && launch_bytes >= (uint64_t)FLAGS_copy_engine_crc_mfma_min_bytes;
        if (!b->crc_host ||
            LaunchBatchedCopyCrc32cMessages(b->segs.data(), b->msg_of.data(), (int)n, b->crc_host, s, done, mfma) != 0) {
            rc = -1;
        }
    } else if (rc == 0) {
        rc = LaunchBatchedCopy(b->segs.data(), (int)n, s, done);
    }
    // with a completion word the event is only the fallback of a launch
    // that never stores its word; -copy_engine_word_event=false drops it
    const bool record = !b->has_word || FLAGS_copy_engine_word_event;
    if (rc == 0 && record && hipEventRecord(b->ev, s) != hipSuccess) rc = -1;
    b->t_issued = monotonic_us();
    if (prev != device) hipSetDevice(prev);
    g_launches.fetch_add(1, std::memory_order_relaxed);
    if (rc != 0) {
        LOG_EVERY_SECOND(ERROR) << "batched copy launch of " << b->segs.size() << " segments failed on device " << device;
        b->fell_back = true;  // part of it may have run: its word slot is not reused
        b->butex->store(-1, std::memory_order_release);
        fiber::butex_wake_all(b->butex);
        return;
    }
    if (b->has_word) {
        WatchWord(dw.word, dw.seq, record ? b->ev : nullptr, b->butex, &b->t_done, kEventCopy, &b->fell_back);
    } else {
        WatchEvent(b->ev, b->butex, &b->t_done, kEventCopy);
    }
}

bool at_limit(const Engine& e) {
    return FLAGS_copy_engine_max_inflight > 0 && e.inflight >= FLAGS_copy_engine_max_inflight;
}

// Launch the open batch, and whatever collects while launching, until
// nothing is open or the in-flight limit is reached (the next retiring
// waiter picks up from there). The caller set e.launching.
void drain(Engine& e, int device) {
    for (;;) {
        Batch* cur;
        {
            std::lock_guard<std::mutex> g(e.mu);
            cur = e.open;
            if (!cur || at_limit(e)) {
                e.launching = false;
                return;
            }
            e.open = nullptr;
            ++e.inflight;
        }
        uint64_t bytes = 0;
        for (const Segment& s : cur->segs) bytes += s.len;
        g_segments.fetch_add((int64_t)cur->segs.size(), std::memory_order_relaxed);
        g_bytes.fetch_add((int64_t)bytes, std::memory_order_relaxed);
        cur->t_issue_begin = monotonic_us();
        launch(cur, device);
    }
}

}  // namespace

int BatchedCopy(const Segment* segs, int n, int device, uint32_t* crcs, bool fold_crc) {
    if (n <= 0) return 0;
    if (device < 0) device = CurrentDevice();
    if (device < 0 || device >= kMaxDev || Init(device) != 0) return -1;
    Engine& e = g_engine[device];
    g_submits.fetch_add(1, std::memory_order_relaxed);
    // rpcz: the call this copy is done for gets the device wait annotated
    Span* span = IsRpczEnabled() ? Span::tls_parent() : nullptr;
    const int64_t t0 = span ? monotonic_us() : 0;
    Batch* mine;
    size_t first = 0;  // index of our first segment in the batch
    int first_msg = 0; // ... and of our first CRC message
    bool fold = false;
    bool leader = false;
    {
        std::lock_guard<std::mutex> g(e.mu);
        if (!e.open) {
            e.open = new_batch(e);
            e.open->butex->store(0, std::memory_order_relaxed);
            e.open->retired.store(false, std::memory_order_relaxed);
            e.open->t_open = monotonic_us();
        }
        mine = e.open;
        first = mine->segs.size();
        mine->segs.insert(mine->segs.end(), segs, segs + n);
        // CRC messages: the whole submission as one (folded on the device)
        // or one per segment. Segments of copy-only submissions get their
        // own messages too (their CRC is computed but unused).
        first_msg = mine->nmsg;
        fold = fold_crc && n <= kInlineSegments;
        for (int i = 0; i < n; ++i) mine->msg_of.push_back(fold ? mine->nmsg : mine->nmsg + i);
        mine->nmsg += fold ? 1 : n;
        if (crcs) mine->want_crc = true;
        mine->refs.fetch_add(1, std::memory_order_relaxed);
        if (!e.launching && !at_limit(e)) {
            e.launching = true;
            leader = true;
        }
    }
    if (leader) drain(e, device);
    const int64_t t_submit = monotonic_us();
    while (mine->butex->load(std::memory_order_acquire) == 0) fiber::butex_wait(mine->butex, 0);
    const int rc = mine->butex->load(std::memory_order_acquire) == 1 ? 0 : -1;
    // the first waiter of a finished batch gives its in-flight slot back and
    // launches what collected meanwhile
    if (!mine->retired.exchange(true, std::memory_order_acq_rel)) {
        bool lead = false;
        {
            std::lock_guard<std::mutex> g(e.mu);
            --e.inflight;
            if (e.open && !e.launching) e.launching = lead = true;
        }
        if (lead) drain(e, device);
    }
    if (rc == 0 && mine->t_done) {
        const int64_t now = monotonic_us();
        g_t_queue.fetch_add(std::max<int64_t>(0, mine->t_issue_begin - t_submit), std::memory_order_relaxed);
        g_t_api.fetch_add(std::max<int64_t>(0, mine->t_issued - mine->t_issue_begin), std::memory_order_relaxed);
        g_t_gpu.fetch_add(std::max<int64_t>(0, mine->t_done - mine->t_issued), std::memory_order_relaxed);
        g_t_wake.fetch_add(std::max<int64_t>(0, now - mine->t_done), std::memory_order_relaxed);
    }
    if (rc == 0 && leader_of_batch(mine, first) && mine->word && !mine->fell_back) {
        const uint64_t t0 = mine->word[1], t1 = mine->word[2];
        if (t1 >= t0 && t1 - t0 < 100000000ull) {
            g_kernel_ticks.fetch_add((int64_t)(t1 - t0), std::memory_order_relaxed);
            g_kernel_timed.fetch_add(1, std::memory_order_relaxed);
            const int64_t off = g_clock_offset_us.load(std::memory_order_relaxed);
            if (off != INT64_MIN && mine->t_done) {
                g_start_delay_us.fetch_add(off + (int64_t)(t0 / 100) - mine->t_issued, std::memory_order_relaxed);
                g_notice_us.fetch_add(mine->t_done - (off + (int64_t)(t1 / 100)), std::memory_order_relaxed);
            }
        }
    }
    if (rc == 0 && crcs) {
        if (fold) {
            crcs[0] = mine->crc_host[first_msg];
        } else {
            memcpy(crcs, mine->crc_host + first_msg, sizeof(uint32_t) * (size_t)n);
            if (fold_crc) {  // too many segments to fold on the device
                uint32_t c = crcs[0];
                for (int i = 1; i < n; ++i) c = crc32c::Combine(c, crcs[i], segs[i].len);
                crcs[0] = c;
            }
        }
    }
    if (span) {
        uint64_t bytes = 0;
        for (int i = 0; i < n; ++i) bytes += segs[i].len;
        span->AnnotateDevice(string_printf("%s %d segs %llu B dev%d%s", crcs ? "copy+crc32c" : "batched copy", n,
                                           (unsigned long long)bytes, device, rc ? " FAILED" : ""),
                             (float)(monotonic_us() - t0) / 1000.0f);
    }
    if (mine->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        // a slot whose launch completed through the event (failed) keeps
        // an unknown counter: it is never reused
        if (mine->has_word && !mine->fell_back) ReleaseDoneWord(device, mine->word_slot);
        mine->has_word = false;
        ReleaseEvent(mine->ev);
        mine->ev = nullptr;
        mine->t_done = 0;
        mine->segs.clear();
        mine->msg_of.clear();
        mine->nmsg = 0;
        mine->want_crc = false;
        std::lock_guard<std::mutex> g(e.mu);
        e.spare.push_back(mine);
    }
    return rc;
}

CopyEngineStats GetCopyEngineStats() {
    CopyEngineStats s;
    s.submits = g_submits.load(std::memory_order_relaxed);
    s.launches = g_launches.load(std::memory_order_relaxed);
    s.segments = g_segments.load(std::memory_order_relaxed);
    s.bytes = g_bytes.load(std::memory_order_relaxed);
    s.queue_us = g_t_queue.load(std::memory_order_relaxed);
    s.api_us = g_t_api.load(std::memory_order_relaxed);
    s.gpu_us = g_t_gpu.load(std::memory_order_relaxed);
    s.wake_us = g_t_wake.load(std::memory_order_relaxed);
    s.kernel_ticks = g_kernel_ticks.load(std::memory_order_relaxed);
    s.kernel_timed = g_kernel_timed.load(std::memory_order_relaxed);
    s.start_delay_us = g_start_delay_us.load(std::memory_order_relaxed);
    s.notice_us = g_notice_us.load(std::memory_order_relaxed);
    return s;
}

}  // namespace gpu
}  // namespace mrpc
