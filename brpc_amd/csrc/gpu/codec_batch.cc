#include "gpu/codec_batch.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <deque>
#include <mutex>

#include "base/flags.h"
#include "base/time.h"
#include "base/logging.h"
#include "fiber/butex.h"
#include "gpu/gpu.h"
#include "gpu/hbm_pool.h"

DEFINE_bool(codec_fused, true,
            "run codec batches of compress blocks and decode pieces (<= 8 KiB) as one launch (then the pb scans, "
            "if any, as a second one) instead of one launch per stage: 158-161 k vs 115 k QPS on the device-body "
            "text leg (profiles/r5_device_codec_ab.txt)");
DEFINE_bool(codec_fused_scan_in_kernel, false,
            "fused batches: the wave that finishes a message's last piece scans its fields in the same launch "
            "(else the pb scan is a second launch). Off: the hand-off needs a device-scope fence per piece, "
            "which on gfx950 compiles to buffer_wbl2 + buffer_inv (an L2 write-back of the XCD) in every wave; "
            "in the RPC leg, with batches overlapping, that made the one-launch kernels 1.5-4x slower per launch");
DEFINE_int32(codec_batch_max_inflight, 4,
             "codec batches in flight per device before the next one waits for a completion (0: no limit); "
             "while it waits, the requests that arrive join it, so a busy GPU gets fewer, larger batches "
             "(device text leg, 50 RPCs in flight: 4 -> 171-174k QPS with the codec events polled "
             "continuously, 6 -> 161-163k, 3 -> 161k, 8 -> 142k; profiles/r5_device_codec_ab.txt)");

namespace mrpc {
namespace gpu {

namespace {

const int kMaxDev = 16;

// A pinned host array the kernels read (job tables) or write (results);
// grows, never shrinks, owned by one batch.
template <typename T>
struct PinnedArray {
    T* p = nullptr;
    size_t cap = 0;
    bool reserve(size_t n) {
        if (n <= cap) return true;
        if (p) PinnedFree(p, cap * sizeof(T));
        cap = std::max<size_t>(n, 64);
        p = static_cast<T*>(PinnedAlloc(cap * sizeof(T)));
        if (!p) cap = 0;
        return p != nullptr;
    }
};

struct CBatch {
    std::vector<CodecRequest*> reqs;
    std::vector<size_t> comp_first, decomp_first, stream_first, piece_first, scan_row, run_first;
    PinnedArray<PbRunChunk> run_jobs;
    PinnedArray<int32_t> run_err;
    std::vector<size_t> dec_first;
    PinnedArray<PbRunDecodeChunk> dec_jobs;
    PinnedArray<uint32_t> dec_counts;
    PinnedArray<int32_t> dec_err;
    PinnedArray<SnappyPiece> piece_jobs;
    PinnedArray<int> piece_job_err;
    PinnedArray<SnappyJob> comp_jobs, decomp_jobs;
    PinnedArray<SnappyStream> stream_jobs;
    PinnedArray<int> stream_err, piece_err;
    SnappyPiece* pieces = nullptr;  // HBM: written by the split kernel, read by the piece decoder
    size_t pieces_cap = 0;
    uint32_t* dec_prefix = nullptr;  // HBM: per-chunk counts, scanned, of the packed-run decoder
    size_t dec_prefix_cap = 0;
    PinnedArray<uint32_t> comp_len, decomp_len;
    PinnedArray<int> comp_err, decomp_err;
    PinnedArray<PbScanJob> scan_jobs;
    PinnedArray<uint32_t> piece_group, group_pieces;  // fused launches: piece -> scan group, pieces per group
    uint32_t* group_done = nullptr;                   // HBM counters, zero between launches
    size_t group_done_cap = 0;
    PinnedArray<uint64_t> scan_fields;
    PinnedArray<int32_t> scan_n;
    void* scratch = nullptr;  // compress slots of blocks above 16 KiB
    size_t scratch_bytes = 0;
    std::atomic<int>* butex = nullptr;
    hipEvent_t ev = nullptr;
    std::atomic<int> refs{0};
    // latency breakdown (monotonic us): launch began, event recorded, the
    // poller saw the completion
    int64_t launch_us = 0, launched_us = 0, done_us = 0;
};

struct Engine {
    std::mutex mu;
    CBatch* open = nullptr;
    bool launching = false;
    std::vector<CBatch*> spare;
    std::deque<CBatch*> flying;  // launched, each holding one ref until the leader retires it
};

void release(Engine& e, CBatch* b) {
    if (b->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        if (b->ev) ReleaseEvent(b->ev);
        b->ev = nullptr;
        b->reqs.clear();
        std::lock_guard<std::mutex> g(e.mu);
        e.spare.push_back(b);
    }
}

// Retire completed batches from the front of the in-flight list (any
// thread; non-blocking).
void retire_done(Engine& e) {
    for (;;) {
        CBatch* oldest = nullptr;
        {
            std::lock_guard<std::mutex> g(e.mu);
            if (e.flying.empty()) return;
            oldest = e.flying.front();
            if (oldest->butex->load(std::memory_order_acquire) == 0) return;
            e.flying.pop_front();
        }
        release(e, oldest);
    }
}

Engine g_engine[kMaxDev];
std::atomic<int64_t> g_requests{0}, g_launches{0}, g_run_chunks{0}, g_dec_chunks{0}, g_fused_launches{0};
// per request, summed: waiting for a launch, the batch's launch API time,
// launch -> completion seen by the poller (device time + queueing + poll),
// completion seen -> requester running again
std::atomic<int64_t> g_queue_us{0}, g_api_us{0}, g_gpu_us{0}, g_wake_us{0}, g_timed{0};

CBatch* new_batch(Engine& e) {
    if (!e.spare.empty()) {
        CBatch* b = e.spare.back();
        e.spare.pop_back();
        return b;
    }
    CBatch* b = new CBatch;
    b->butex = fiber::butex_create();
    return b;
}

// Lay the batch's requests out in its pinned tables and issue one stream
// sequence; false when nothing could be launched.
bool launch(CBatch* b, int device) {
    size_t ncomp = 0, ndecomp = 0, nscan = 0, nstreams = 0, npieces = 0, nhpieces = 0, nruns = 0, ndec = 0;
    uint32_t comp_max = 1, decomp_max = 1, piece_limit = 0, hpiece_max = 1;
    std::vector<Segment> h2d, d2h;
    b->comp_first.clear();
    b->decomp_first.clear();
    b->stream_first.clear();
    b->piece_first.clear();
    b->scan_row.clear();
    b->run_first.clear();
    b->dec_first.clear();
    for (CodecRequest* r : b->reqs) {
        b->run_first.push_back(nruns);
        nruns += r->runs.size();
        b->dec_first.push_back(ndec);
        ndec += r->dec_runs.size();
        b->comp_first.push_back(ncomp);
        b->decomp_first.push_back(ndecomp);
        b->stream_first.push_back(nstreams);
        b->piece_first.push_back(nhpieces);
        nhpieces += r->pieces.size();
        hpiece_max = std::max(hpiece_max, r->pieces_max_ulen);
        nstreams += r->streams.size();
        for (const SnappyStream& st : r->streams) npieces += st.max_pieces;
        if (!r->streams.empty()) piece_limit = std::max(piece_limit, r->stream_piece_limit);
        b->scan_row.push_back(nscan);
        ncomp += r->comp.size();
        ndecomp += r->decomp.size();
        nscan += r->scans.size();
        comp_max = std::max(comp_max, r->comp_max_ulen);
        decomp_max = std::max(decomp_max, r->decomp_max_ulen);
        h2d.insert(h2d.end(), r->h2d.begin(), r->h2d.end());
        d2h.insert(d2h.end(), r->d2h.begin(), r->d2h.end());
    }
    if (!b->comp_jobs.reserve(ncomp) || !b->comp_len.reserve(ncomp) || !b->comp_err.reserve(ncomp) ||
        !b->decomp_jobs.reserve(ndecomp) || !b->decomp_len.reserve(ndecomp) || !b->decomp_err.reserve(ndecomp) ||
        !b->scan_jobs.reserve(nscan) || !b->scan_fields.reserve(nscan * 2 * kCodecScanFields) ||
        !b->scan_n.reserve(nscan) || !b->stream_jobs.reserve(nstreams) || !b->stream_err.reserve(nstreams) ||
        !b->piece_err.reserve(npieces) || !b->piece_jobs.reserve(nhpieces) || !b->piece_job_err.reserve(nhpieces) ||
        !b->run_jobs.reserve(nruns) || !b->run_err.reserve(nruns) || !b->dec_jobs.reserve(ndec) ||
        !b->dec_counts.reserve(ndec) || !b->dec_err.reserve(ndec)) {
        return false;
    }
    if (npieces > b->pieces_cap) {
        if (b->pieces) HbmFree(b->pieces, b->pieces_cap * sizeof(SnappyPiece), device);
        const size_t cap = std::max<size_t>(npieces, 256);
        b->pieces = static_cast<SnappyPiece*>(HbmAlloc(cap * sizeof(SnappyPiece), device));
        b->pieces_cap = b->pieces ? cap : 0;
        if (!b->pieces) return false;
    }
    for (size_t i = 0; i < b->reqs.size(); ++i) {
        const CodecRequest* r = b->reqs[i];
        std::copy(r->comp.begin(), r->comp.end(), b->comp_jobs.p + b->comp_first[i]);
        std::copy(r->decomp.begin(), r->decomp.end(), b->decomp_jobs.p + b->decomp_first[i]);
        std::copy(r->scans.begin(), r->scans.end(), b->scan_jobs.p + b->scan_row[i]);
        std::copy(r->pieces.begin(), r->pieces.end(), b->piece_jobs.p + b->piece_first[i]);
        std::copy(r->runs.begin(), r->runs.end(), b->run_jobs.p + b->run_first[i]);
        for (size_t k = 0; k < r->dec_runs.size(); ++k) {
            PbRunDecodeChunk c = r->dec_runs[k];
            c.first += (uint32_t)b->dec_first[i];
            b->dec_jobs.p[b->dec_first[i] + k] = c;
        }
    }
    for (size_t i = 0, g = 0, first = 0; i < b->reqs.size(); ++i) {
        for (const SnappyStream& st : b->reqs[i]->streams) {
            SnappyStream& d = b->stream_jobs.p[g++];
            d = st;
            d.first = (uint32_t)first;
            first += st.max_pieces;
        }
    }
    if (ndec > b->dec_prefix_cap) {
        if (b->dec_prefix) HbmFree(b->dec_prefix, b->dec_prefix_cap * sizeof(uint32_t), device);
        const size_t cap = std::max<size_t>(ndec, 1024);
        b->dec_prefix = static_cast<uint32_t*>(HbmAlloc(cap * sizeof(uint32_t), device));
        b->dec_prefix_cap = b->dec_prefix ? cap : 0;
        if (!b->dec_prefix) return false;
    }
    if (ncomp && SnappyCompressUsesScratch(comp_max)) {
        const size_t need = ncomp * SnappyCompressScratchPerBlock();
        if (need > b->scratch_bytes) {
            if (b->scratch) HbmFree(b->scratch, b->scratch_bytes, device);
            b->scratch = HbmAlloc(need, device);
            b->scratch_bytes = b->scratch ? need : 0;
        }
        if (!b->scratch) return false;
    }
    // one fused launch when the batch is codec work only: compress blocks
    // and headerless pieces that fit the one-launch kernels (the pb scans
    // follow as a second launch unless -codec_fused_scan_in_kernel, which
    // needs every scan to name the pieces forming its message)
    const bool fused = FLAGS_codec_fused && nruns == 0 && ndec == 0 && h2d.empty() && d2h.empty() && ndecomp == 0 &&
                       nstreams == 0 && (ncomp || nhpieces) && comp_max <= kFusedMaxBlock && hpiece_max <= kFusedMaxBlock;
    bool scan_in_kernel = fused && FLAGS_codec_fused_scan_in_kernel && nscan > 0;
    for (size_t i = 0; scan_in_kernel && i < b->reqs.size(); ++i) {
        const CodecRequest* r = b->reqs[i];
        if (r->scans.empty()) continue;
        if (r->scan_piece_first.size() != r->scans.size() || r->scan_piece_count.size() != r->scans.size()) {
            scan_in_kernel = false;
            break;
        }
        for (size_t k = 0; k < r->scans.size(); ++k) {
            if (r->scan_piece_count[k] == 0 || r->scan_piece_first[k] + r->scan_piece_count[k] > r->pieces.size()) {
                scan_in_kernel = false;
            }
        }
    }
    if (scan_in_kernel && (!b->piece_group.reserve(nhpieces) || !b->group_pieces.reserve(nscan))) return false;
    int prev = 0;
    hipGetDevice(&prev);
    if (prev != device) hipSetDevice(device);
    hipStream_t s = PoolStream(device);
    b->ev = AcquireEvent();
    int rc = (s && b->ev) ? 0 : -1;
    if (rc == 0 && fused) {
        if (scan_in_kernel) {
            if (nscan > b->group_done_cap) {
                if (b->group_done) HbmFree(b->group_done, b->group_done_cap * sizeof(uint32_t), device);
                const size_t cap = std::max<size_t>(nscan, 256);
                b->group_done = static_cast<uint32_t*>(HbmAlloc(cap * sizeof(uint32_t), device));
                b->group_done_cap = b->group_done ? cap : 0;
            }
            // zeroed before EVERY launch, ordered before it on the same
            // stream: a launch that stopped partway (a fault) must not leave
            // counters that start the next launch's scans early
            if (!b->group_done || hipMemsetAsync(b->group_done, 0, nscan * sizeof(uint32_t), s) != hipSuccess) {
                rc = -1;
            }
            for (size_t p = 0; p < nhpieces; ++p) b->piece_group.p[p] = kFusedNoGroup;
            for (size_t i = 0; i < b->reqs.size(); ++i) {
                const CodecRequest* r = b->reqs[i];
                for (size_t k = 0; k < r->scans.size(); ++k) {
                    const size_t g = b->scan_row[i] + k;
                    b->group_pieces.p[g] = r->scan_piece_count[k];
                    for (uint32_t q = 0; q < r->scan_piece_count[k]; ++q)
                        b->piece_group.p[b->piece_first[i] + r->scan_piece_first[k] + q] = (uint32_t)g;
                }
            }
        }
        FusedCodecArgs fa;
        fa.comp = b->comp_jobs.p;
        fa.ncomp = (int)ncomp;
        fa.comp_len = b->comp_len.p;
        fa.comp_err = b->comp_err.p;
        fa.pieces = b->piece_jobs.p;
        fa.npieces = (int)nhpieces;
        fa.piece_err = b->piece_job_err.p;
        fa.piece_group = scan_in_kernel ? b->piece_group.p : nullptr;
        fa.scans = b->scan_jobs.p;
        fa.group_pieces = b->group_pieces.p;
        fa.group_done = b->group_done;
        fa.scan_fields = b->scan_fields.p;
        fa.scan_n = b->scan_n.p;
        fa.max_fields = kCodecScanFields;
        fa.max_ulen = std::max(ncomp ? comp_max : 1u, nhpieces ? hpiece_max : 1u);
        if (rc == 0) rc = LaunchCodecWaves(fa, s);
        g_fused_launches.fetch_add(1, std::memory_order_relaxed);
        ncomp = nhpieces = 0;  // nothing left for the per-stage sequence below but (maybe) the scans
        if (scan_in_kernel) nscan = 0;
    }
    if (rc == 0 && nruns) rc = LaunchPbRunEncode(b->run_jobs.p, (int)nruns, b->run_err.p, s);
    g_run_chunks.fetch_add((int64_t)nruns, std::memory_order_relaxed);
    if (rc == 0 && !h2d.empty()) rc = LaunchBatchedCopy(h2d.data(), (int)h2d.size(), s);
    if (rc == 0 && ncomp) {
        rc = LaunchSnappyCompress(b->comp_jobs.p, (int)ncomp, comp_max, b->scratch, b->comp_len.p, b->comp_err.p, s);
    }
    if (rc == 0 && ndecomp) {
        rc = LaunchSnappyDecompress(b->decomp_jobs.p, (int)ndecomp, decomp_max, b->decomp_len.p, b->decomp_err.p, s);
    }
    if (rc == 0 && nhpieces) {
        rc = LaunchSnappyDecompressPieces(b->piece_jobs.p, (int)nhpieces, 0, std::min(hpiece_max, kSnappyMaxBlock),
                                          b->piece_job_err.p, s);
    }
    if (rc == 0 && nstreams) {
        // cut on the device, then small pieces (many waves per CU) and the
        // 64 KiB fragments of CPU encoders in a second launch
        const uint32_t small = std::min(piece_limit, kSnappyMaxBlock);
        rc = LaunchSnappySplit(b->stream_jobs.p, (int)nstreams, small, b->pieces, b->stream_err.p, s);
        if (rc == 0) rc = LaunchSnappyDecompressPieces(b->pieces, (int)npieces, 0, small, b->piece_err.p, s);
        if (rc == 0 && small < kSnappyMaxBlock) {
            rc = LaunchSnappyDecompressPieces(b->pieces, (int)npieces, small, kSnappyMaxBlock, b->piece_err.p, s);
        }
    }
    if (rc == 0 && nscan) {
        rc = LaunchPbScanPtrs(b->scan_jobs.p, (int64_t)nscan, kCodecScanFields, b->scan_fields.p, b->scan_n.p, s);
    }
    if (rc == 0 && !d2h.empty()) rc = LaunchBatchedCopy(d2h.data(), (int)d2h.size(), s);
    if (rc == 0 && ndec) rc = LaunchPbRunDecode(b->dec_jobs.p, (int)ndec, b->dec_counts.p, b->dec_prefix, b->dec_err.p, s);
    g_dec_chunks.fetch_add((int64_t)ndec, std::memory_order_relaxed);
    if (rc == 0 && hipEventRecord(b->ev, s) != hipSuccess) rc = -1;
    if (prev != device) hipSetDevice(prev);
    g_launches.fetch_add(1, std::memory_order_relaxed);
    if (rc != 0) {
        // kernels already queued may still read the tables: wait them out
        // before anyone frees request buffers
        if (s) SyncStream(s);
        return false;
    }
    b->done_us = 0;
    WatchEvent(b->ev, b->butex, &b->done_us, kEventCodec);
    return true;
}

// Launch the open batch while fewer than -codec_batch_max_inflight batches
// are in flight; one launcher at a time, and nobody waits here. With the
// limit reached the open batch keeps collecting requests until a completion
// frees a place: the requesters of every finished batch pump again, so an
// open batch always has a completion coming that launches it. (A leader that
// kept launching, blocking on the oldest batch, served the whole burst
// while its own RPC, long finished, waited behind it: one call of every
// run timed out at a limit of 1.)
void pump(Engine& e, int device) {
    const int limit = FLAGS_codec_batch_max_inflight;
    for (;;) {
        retire_done(e);
        CBatch* cur;
        {
            std::lock_guard<std::mutex> g(e.mu);
            if (e.launching || !e.open) return;
            if (limit > 0 && (int)e.flying.size() >= limit) return;
            e.launching = true;
            cur = e.open;
            e.open = nullptr;
            // the in-flight list's ref, taken before the launch: the batch can
            // complete, and its requesters drop their refs, before we get back
            cur->refs.fetch_add(1, std::memory_order_relaxed);
        }
        cur->launch_us = monotonic_us();
        const bool ok = launch(cur, device);
        cur->launched_us = monotonic_us();
        if (!ok) {
            LOG_EVERY_SECOND(ERROR) << "codec batch of " << cur->reqs.size() << " requests failed on device " << device;
            cur->butex->store(-1, std::memory_order_release);
            fiber::butex_wake_all(cur->butex);
        } else {
            std::lock_guard<std::mutex> g(e.mu);
            e.flying.push_back(cur);
        }
        if (!ok) release(e, cur);
        std::lock_guard<std::mutex> g(e.mu);
        e.launching = false;
    }
}

}  // namespace

int RunCodecRequest(CodecRequest* r, int device) {
    if (device < 0 || device >= kMaxDev || Init(device) != 0) return -1;
    Engine& e = g_engine[device];
    g_requests.fetch_add(1, std::memory_order_relaxed);
    const int64_t submit_us = monotonic_us();
    CBatch* mine;
    size_t idx = 0;
    {
        std::lock_guard<std::mutex> g(e.mu);
        if (!e.open) {
            e.open = new_batch(e);
            e.open->butex->store(0, std::memory_order_relaxed);
        }
        mine = e.open;
        idx = mine->reqs.size();
        mine->reqs.push_back(r);
        mine->refs.fetch_add(1, std::memory_order_relaxed);
    }
    pump(e, device);
    while (mine->butex->load(std::memory_order_acquire) == 0) fiber::butex_wait(mine->butex, 0);
    const int rc = mine->butex->load(std::memory_order_acquire) == 1 ? 0 : -1;
    if (rc == 0 && mine->done_us > 0) {
        const int64_t woke = monotonic_us();
        g_queue_us.fetch_add(std::max<int64_t>(0, mine->launch_us - submit_us), std::memory_order_relaxed);
        g_api_us.fetch_add(mine->launched_us - mine->launch_us, std::memory_order_relaxed);
        g_gpu_us.fetch_add(std::max<int64_t>(0, mine->done_us - mine->launched_us), std::memory_order_relaxed);
        g_wake_us.fetch_add(std::max<int64_t>(0, woke - mine->done_us), std::memory_order_relaxed);
        g_timed.fetch_add(1, std::memory_order_relaxed);
    }
    if (rc == 0) {
        const size_t c0 = mine->comp_first[idx], d0 = mine->decomp_first[idx];
        r->comp_len.assign(mine->comp_len.p + c0, mine->comp_len.p + c0 + r->comp.size());
        r->comp_err.assign(mine->comp_err.p + c0, mine->comp_err.p + c0 + r->comp.size());
        r->decomp_len.assign(mine->decomp_len.p + d0, mine->decomp_len.p + d0 + r->decomp.size());
        r->decomp_err.assign(mine->decomp_err.p + d0, mine->decomp_err.p + d0 + r->decomp.size());
        const size_t r0 = mine->run_first[idx];
        r->run_err.assign(mine->run_err.p + r0, mine->run_err.p + r0 + r->runs.size());
        const size_t q0 = mine->dec_first[idx];
        r->dec_counts.assign(mine->dec_counts.p + q0, mine->dec_counts.p + q0 + r->dec_runs.size());
        r->dec_err.assign(mine->dec_err.p + q0, mine->dec_err.p + q0 + r->dec_runs.size());
        const size_t p0 = mine->piece_first[idx];
        r->piece_err.assign(mine->piece_job_err.p + p0, mine->piece_job_err.p + p0 + r->pieces.size());
        r->stream_err.assign(r->streams.size(), 0);
        for (size_t j = 0; j < r->streams.size(); ++j) {
            const size_t g = mine->stream_first[idx] + j;
            int code = mine->stream_err.p[g];
            const SnappyStream& st = mine->stream_jobs.p[g];
            for (uint32_t k = 0; code == 0 && k < st.max_pieces; ++k) code = mine->piece_err.p[st.first + k];
            r->stream_err[j] = code;
        }
        if (!r->scans.empty()) {
            const size_t row = mine->scan_row[idx], ns = r->scans.size();
            const uint64_t* f = mine->scan_fields.p + row * 2 * kCodecScanFields;
            r->scan_nfields.assign(mine->scan_n.p + row, mine->scan_n.p + row + ns);
            r->scan_fields.assign(f, f + ns * 2 * kCodecScanFields);
        }
    }
    release(e, mine);
    // retire what finished (an idle engine must not keep events, pinned
    // tables and HBM buffers until the next request) and launch the batch
    // that waited for a place
    pump(e, device);
    return rc;
}

CodecBatchStats GetCodecBatchStats() {
    CodecBatchStats s;
    s.requests = g_requests.load(std::memory_order_relaxed);
    s.launches = g_launches.load(std::memory_order_relaxed);
    s.run_chunks = g_run_chunks.load(std::memory_order_relaxed);
    s.decode_chunks = g_dec_chunks.load(std::memory_order_relaxed);
    s.fused_launches = g_fused_launches.load(std::memory_order_relaxed);
    s.timed = g_timed.load(std::memory_order_relaxed);
    s.queue_us = g_queue_us.load(std::memory_order_relaxed);
    s.api_us = g_api_us.load(std::memory_order_relaxed);
    s.gpu_us = g_gpu_us.load(std::memory_order_relaxed);
    s.wake_us = g_wake_us.load(std::memory_order_relaxed);
    return s;
}

}  // namespace gpu
}  // namespace mrpc
