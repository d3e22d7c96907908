// Cross-request batching of the device body codecs (snappy compress /
// decompress, pb_scan) — the same leader-combining scheme as the copy
// engine (gpu/copy_engine.h): concurrent RPCs submit their codec work, one
// submitter becomes the leader and issues everything that accumulated as ONE
// sequence on one stream (staging copies, one compress launch, one
// stream-split launch, the decompress launches, one pb_scan launch, copies
// back) with ONE event; every
// submitter parks its fiber on that event. At 50 RPCs in flight this turns
// ~4 launches + 1 event per body into a few per batch of bodies.
#pragma once

#include <cstdint>
#include <vector>

#include "gpu/kernels.h"

namespace mrpc {
namespace gpu {

struct CodecRequest {
    // numeric runs encoded first (K2 packed fields / K6 JSON arrays), into
    // buffers the later stages may read (the body the compressor takes)
    std::vector<PbRunChunk> runs;
    // staging copies issued before the codec kernels (host/pinned -> HBM)
    std::vector<Segment> h2d;
    // codec jobs; pointers in the jobs are device-accessible
    std::vector<SnappyJob> comp, decomp;
    uint32_t comp_max_ulen = 0, decomp_max_ulen = 0;
    // whole compressed streams cut into pieces on the device
    // (snappy_split_kernel) and decoded piecewise, no host tag walk;
    // SnappyStream::first is relative to this request (the batch rebases it)
    std::vector<SnappyStream> streams;
    uint32_t stream_piece_limit = 4096;
    // headerless pieces cut on the host (pointers device-accessible)
    std::vector<SnappyPiece> pieces;
    uint32_t pieces_max_ulen = 0;
    // wire scans of decoded messages (kCodecScanFields rows each), run after
    // every decode of the batch
    std::vector<PbScanJob> scans;
    // optional, per scan: the range of `pieces` that decode into its message.
    // When every scan of a batch names its pieces (and the batch holds only
    // compress jobs and pieces of <= kFusedMaxBlock), the batch is ONE fused
    // launch (codec_waves_kernel) and, with -codec_fused_scan_in_kernel,
    // the scan runs as soon as the message's last piece is decoded.
    std::vector<uint32_t> scan_piece_first, scan_piece_count;
    // copies issued after the kernels (HBM -> pinned)
    std::vector<Segment> d2h;
    // packed varint runs decoded last (their bytes are final by then);
    // PbRunDecodeChunk::first is relative to this request (rebased)
    std::vector<PbRunDecodeChunk> dec_runs;

    // results, filled before RunCodecRequest returns 0
    std::vector<uint32_t> comp_len, decomp_len;
    std::vector<int> comp_err, decomp_err;
    std::vector<int> stream_err;  // 0, or the split / piece decode code
    std::vector<int> piece_err;
    std::vector<int32_t> run_err;  // per chunk: 0, or 1 when the device size disagreed (nothing written)
    std::vector<uint32_t> dec_counts;  // per decode chunk: varints ending in it
    std::vector<int32_t> dec_err;      // per decode chunk: 0, or 1 for a malformed varint
    std::vector<uint64_t> scan_fields;  // 2 * kCodecScanFields per scan
    std::vector<int32_t> scan_nfields;  // per scan: field count or a negative code

    // Empty again, keeping every vector's capacity (pooled requests: the
    // device codec path issued ~20 allocations per RPC building fresh ones).
    void Reset() {
        runs.clear();
        h2d.clear();
        comp.clear();
        decomp.clear();
        comp_max_ulen = decomp_max_ulen = 0;
        streams.clear();
        stream_piece_limit = 4096;
        pieces.clear();
        pieces_max_ulen = 0;
        scans.clear();
        scan_piece_first.clear();
        scan_piece_count.clear();
        d2h.clear();
        dec_runs.clear();
        comp_len.clear();
        decomp_len.clear();
        comp_err.clear();
        decomp_err.clear();
        stream_err.clear();
        piece_err.clear();
        run_err.clear();
        dec_counts.clear();
        dec_err.clear();
        scan_fields.clear();
        scan_nfields.clear();
    }
};

constexpr uint32_t kCodecScanFields = 128;

// Blocks the calling fiber until the batch holding `r` completed; 0 on
// success (per-job codes in the result vectors), -1 on a device error.
int RunCodecRequest(CodecRequest* r, int device);

struct CodecBatchStats {
    int64_t requests = 0, launches = 0, run_chunks = 0, decode_chunks = 0, fused_launches = 0;
    // latency breakdown summed over `timed` requests (us): waiting for a
    // launch, launch API, launch -> completion seen, completion -> resumed
    int64_t timed = 0, queue_us = 0, api_us = 0, gpu_us = 0, wake_us = 0;
};
CodecBatchStats GetCodecBatchStats();

}  // namespace gpu
}  // namespace mrpc
