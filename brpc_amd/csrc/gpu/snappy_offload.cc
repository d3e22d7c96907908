// GPU snappy for RPC bodies: the offload behind rpc/compress.h's
// SetSnappyOffload (reference: src/brpc/policy/snappy_compress.cpp:28-64,
// src/brpc/compress.cpp:79-92 — ParseFromCompressedData /
// SerializeAsCompressedData call the registered snappy handler; this is that
// handler's device half).
//
// Wire format is standard raw snappy in both directions, so peers with a
// CPU codec interoperate:
//  * compress: the body is staged into HBM (batched copy kernel reading the
//    pinned socket blocks), cut into gpu_snappy_block_kb blocks (4 KiB: one
//    64 KiB body spreads over 16 waves) that snappy_compress_kernel encodes
//    one wave each straight into pinned host memory; the stream is
//    one varint header + the blocks' element runs (a block never references
//    another, so the concatenation is one valid stream).
//  * decompress: the compressed blocks are copied to HBM as they are (no
//    flattening, no per-piece staging); the stream is cut into pieces of
//    <= 4 KiB (device encoders), else <= 64 KiB (CPU encoders) uncompressed
//    whose copies stay inside the piece, and the headerless piece decoder
//    rebuilds every piece in LDS. The cut is one host walk over the blocks
//    in place (~3 us per 64 KiB body), or with -gpu_snappy_device_split
//    snappy_split_kernel on the device: the walk is a serial chain, and one
//    wave takes ~95 us for the same body (MI355X, kernel trace), so the host
//    walk is the default. A stream that cannot be cut (or is malformed)
//    falls back to the CPU codec.
// Each direction is one stream-ordered sequence (copy, kernel) and ONE
// fiber-friendly event wait, shared with every other RPC's codec work that
// arrived meanwhile (gpu/codec_batch.h: one launch sequence per batch).
// History on MI355X (bench.py gRPC leg, 64 KiB bodies, 50 in flight): one
// launch + wait per call lost to the CPU codec (25k vs 53k QPS); with
// cross-RPC batching the GPU codec wins (63k vs 46k QPS at 152 vs 261 host
// CPU us per RPC, profiles/r3_bench_run7_checkpoint.json). It stays opt-in
// (EnableGpuSnappy) with a body-size threshold: small bodies are faster on
// the CPU than any launch.
#include "gpu/snappy_offload.h"

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "base/logging.h"
#include "gpu/codec_batch.h"
#include "gpu/gpu.h"
#include "gpu/hbm_pool.h"
#include "gpu/kernels.h"
#include "pb/descriptor.h"
#include "pb/message.h"
#include "rpc/compress.h"
#include "var/var.h"
#include "base/flags.h"

DECLARE_uint64(max_body_size);

DEFINE_bool(gpu_snappy_device_split, false,
            "cut received snappy streams on the device (snappy_split_kernel) instead of walking the tags on the "
            "host; measured slower on MI355X: the walk is serial, ~95 us of one wave per 64 KiB body vs ~3 us of "
            "host CPU (profiles/r3_snappy_device_split.txt)");
DEFINE_bool(gpu_snappy_direct_host, true,
            "codec kernels read their host input and write their host output in pinned memory directly (no "
            "staging copy kernels around them): two kernels fewer per decode, one per encode");
DEFINE_int32(gpu_pb_pack_min_elems, 4096,
             "packed varint fields with at least this many elements are encoded on the device (pb_run_encode_kernel) "
             "when their message goes through the GPU snappy codec, in the same batch as the compress kernel; 0: "
             "never");
DEFINE_int32(gpu_pb_unpack_min_bytes, 16384,
             "packed varint fields of at least this many bytes in a body the GPU codec decoded are decoded on the "
             "device too (pb_run_count/decode kernels, one more codec batch per message); 0: never");
DEFINE_bool(gpu_snappy_packed_only, true,
            "with the GPU snappy codec enabled, route only messages with large packed numeric fields to it (their "
            "varints are packed/unpacked on the device in the same batch); plain host bodies (strings, bytes) go to "
            "the CPU codec, which beats a host-memory GPU round trip on them (bench: the *_snappy_64KB_* legs)");
DEFINE_int32(gpu_snappy_block_kb, 4,
             "uncompressed bytes per device snappy block (one wave each): smaller blocks spread one body over more "
             "waves (lower latency) at some cost in ratio; <= 64");

#include "base/time.h"
#include "rpc/span.h"

namespace mrpc {
namespace gpu {

namespace {

int g_device = -1;
std::atomic<int64_t> g_comp_calls{0}, g_decomp_calls{0}, g_fallbacks{0};

void pinned_deleter(void* p, void* arg) { PinnedFree(p, (size_t)reinterpret_cast<uintptr_t>(arg)); }

// A pinned host buffer owned by a Buf block (kind PINNED).
struct PinnedBuf {
    char* p = nullptr;
    size_t n = 0;
    explicit PinnedBuf(size_t bytes) : p(bytes ? static_cast<char*>(PinnedAlloc(bytes)) : nullptr), n(bytes) {}
    ~PinnedBuf() {
        if (p) PinnedFree(p, n);
    }
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(PinnedBuf&& o) noexcept {
        if (this != &o) {
            if (p) PinnedFree(p, n);
            p = o.p;
            n = o.n;
            o.p = nullptr;
        }
        return *this;
    }
    // hand ownership to *b as one block
    void give_to(Buf* b) {
        b->append_user_data(p, n, pinned_deleter, reinterpret_cast<void*>((uintptr_t)n), MemKind::PINNED);
        p = nullptr;
    }
};

struct HbmTmp {
    void* p = nullptr;
    size_t n = 0;
    int dev = -1;
    HbmTmp(size_t bytes, int d) : p(bytes ? HbmAlloc(bytes, d) : nullptr), n(bytes), dev(d) {}
    ~HbmTmp() {
        if (p) HbmFree(p, n, dev);
    }
};

int varint_len(uint64_t v) {
    int n = 1;
    while (v >= 0x80) {
        v >>= 7;
        ++n;
    }
    return n;
}

int put_varint(char* out, uint64_t v) {
    int n = 0;
    while (v >= 0x80) {
        out[n++] = (char)((v & 0x7f) | 0x80);
        v >>= 7;
    }
    out[n++] = (char)v;
    return n;
}

// Gather segments for `in` into HBM at dst (pageable bytes bounced through
// `bounce`, which must hold them).
void gather_segments(const Buf& in, char* dst, char* bounce, std::vector<Segment>* segs) {
    size_t off = 0, boff = 0;
    for (size_t i = 0; i < in.backing_block_num(); ++i) {
        const BlockRef& r = in.ref_at(i);
        const char* src = r.block->data + r.offset;
        if (r.block->kind == MemKind::HOST) {
            memcpy(bounce + boff, src, r.length);
            src = bounce + boff;
            boff += r.length;
        }
        segs->push_back(Segment{src, dst + off, r.length});
        off += r.length;
    }
}

size_t pageable_bytes(const Buf& in) {
    size_t n = 0;
    for (size_t i = 0; i < in.backing_block_num(); ++i) {
        if (in.ref_at(i).block->kind == MemKind::HOST) n += in.ref_at(i).length;
    }
    return n;
}

bool device_blocks_elsewhere(const Buf& in, int device) {
    for (size_t i = 0; i < in.backing_block_num(); ++i) {
        const BufBlock* b = in.ref_at(i).block;
        if (!IsHostAccessible(b->kind) && b->device != device) return true;
    }
    return false;
}

static_assert(kPbRunChunkElems == pb::kPackedRunChunkElems, "serializer and kernel chunking differ");

uint32_t run_kind(pb::FieldType t) {
    switch (t) {
    case pb::FieldType::INT32:
    case pb::FieldType::ENUM: return PB_RUN_INT32;
    case pb::FieldType::UINT32: return PB_RUN_UINT32;
    case pb::FieldType::SINT32: return PB_RUN_SINT32;
    case pb::FieldType::INT64: return PB_RUN_INT64;
    case pb::FieldType::UINT64: return PB_RUN_UINT64;
    case pb::FieldType::SINT64: return PB_RUN_SINT64;
    default: return PB_RUN_BOOL;
    }
}

// Collects the packed runs the serializer skipped (pb::PackedRunSink).
struct RunCollector : public pb::PackedRunSink {
    std::vector<pb::PackedRun> runs;
    size_t value_bytes = 0;
    size_t min_elems() const override { return (size_t)std::max(1, FLAGS_gpu_pb_pack_min_elems); }
    void Take(pb::PackedRun&& r) override {
        value_bytes += r.n * r.elem_bytes;
        runs.push_back(std::move(r));
    }
};

// The runs' values copied into one pinned buffer (the kernel cannot read
// pageable vectors) and cut into device chunks.
bool stage_runs(const RunCollector& col, PinnedBuf* stage, std::vector<PbRunChunk>* chunks) {
    size_t off = 0;
    for (const pb::PackedRun& r : col.runs) {
        char* v = stage->p + off;
        memcpy(v, r.values, r.n * r.elem_bytes);
        uint8_t* d = r.dst;
        for (size_t c = 0, k = 0; c < r.n; c += kPbRunChunkElems, ++k) {
            PbRunChunk ch;
            ch.src = v + c * r.elem_bytes;
            ch.dst = d;
            ch.count = (uint32_t)std::min<size_t>(kPbRunChunkElems, r.n - c);
            ch.kind = run_kind(r.type);
            ch.format = PB_RUN_VARINT;
            ch.last = c + kPbRunChunkElems >= r.n ? 1 : 0;
            ch.bytes = r.chunk_bytes[k];
            ch.pad = 0;
            chunks->push_back(ch);
            d += r.chunk_bytes[k];
        }
        off += (r.n * r.elem_bytes + 15) & ~(size_t)15;
    }
    return true;
}

std::atomic<int64_t> g_unpack_runs{0}, g_unpack_fallbacks{0};

// Decodes packed runs whose bytes are device-readable (pinned) into one
// pinned array per call: chunks of every run in one codec request.
// Returns false when nothing could be decoded on the device.
bool decode_runs(std::vector<pb::PackedRunIn>* runs, PinnedBuf* out, int device) {
    size_t cap = 0;
    for (const pb::PackedRunIn& r : *runs) cap += ((r.len * r.elem_bytes) + 15) & ~(size_t)15;
    *out = PinnedBuf(cap ? cap : 1);
    if (!out->p) return false;
    CodecRequest req;
    std::vector<size_t> first_chunk;
    size_t off = 0;
    for (pb::PackedRunIn& r : *runs) {
        first_chunk.push_back(req.dec_runs.size());
        // a run must end on a varint's last byte (else it is truncated: the
        // host parser reports it)
        if (r.len == 0 || (r.p[r.len - 1] & 0x80) || r.len > 0xFFFFFFFFull) continue;
        const uint32_t first = (uint32_t)req.dec_runs.size();
        for (size_t o = 0; o < r.len; o += kPbRunDecodeChunkBytes) {
            PbRunDecodeChunk c;
            c.run = r.p;
            c.dst = out->p + off;
            c.offset = (uint32_t)o;
            c.len = (uint32_t)std::min<size_t>(kPbRunDecodeChunkBytes, r.len - o);
            c.first = first;
            c.kind = run_kind(r.type);
            req.dec_runs.push_back(c);
        }
        r.values = out->p + off;  // provisional: cleared below on a device error
        off += ((r.len * r.elem_bytes) + 15) & ~(size_t)15;
    }
    first_chunk.push_back(req.dec_runs.size());
    if (req.dec_runs.empty()) return false;
    if (RunCodecRequest(&req, device) != 0) {
        for (pb::PackedRunIn& r : *runs) r.values = nullptr;
        return false;
    }
    for (size_t i = 0; i < runs->size(); ++i) {
        pb::PackedRunIn& r = (*runs)[i];
        if (!r.values) continue;
        size_t count = 0;
        bool ok = true;
        for (size_t k = first_chunk[i]; k < first_chunk[i + 1]; ++k) {
            count += req.dec_counts[k];
            ok = ok && req.dec_err[k] == 0;
        }
        if (!ok) {
            r.values = nullptr;  // malformed: the host parser reports it
            continue;
        }
        r.count = count;
    }
    return true;
}

struct DeviceRunDecoder : public pb::PackedRunDecoder {
    PinnedBuf out{1};
    int calls = 0;  // runs handed to the device by this parse
    size_t min_bytes() const override { return (size_t)std::max(1, FLAGS_gpu_pb_unpack_min_bytes); }
    void Decode(std::vector<pb::PackedRunIn>* runs) override {
        calls += (int)runs->size();
        if (g_device < 0 || !decode_runs(runs, &out, g_device)) {
            g_unpack_fallbacks.fetch_add(1, std::memory_order_relaxed);
            return;
        }
        for (const pb::PackedRunIn& r : *runs) {
            if (r.values) g_unpack_runs.fetch_add(1, std::memory_order_relaxed);
        }
    }
};

bool gpu_compress(const Buf& in, Buf* out, const std::vector<PbRunChunk>* runs = nullptr) {
    const int dev = g_device;
    const size_t n = in.size();
    const size_t blk = (size_t)std::max(1, std::min(64, FLAGS_gpu_snappy_block_kb)) << 10;
    const size_t nblk = (n + blk - 1) / blk;
    const size_t cap = (SnappyMaxCompressedLength(blk) + 15) & ~(size_t)15;
    // direct: the kernel stages its blocks into LDS straight from pinned
    // host memory (the body's own pinned block, or one flat pinned copy);
    // otherwise the body is gathered into HBM first
    const bool direct = FLAGS_gpu_snappy_direct_host && in.all_host_accessible();
    const bool one_pinned = in.backing_block_num() == 1 && in.ref_at(0).block->kind == MemKind::PINNED;
    const size_t pageable = direct ? 0 : pageable_bytes(in);
    HbmTmp raw(direct ? 0 : n, dev);
    PinnedBuf flat(direct && !one_pinned ? n : 1), bounce(pageable ? pageable : 1), comp(nblk * cap);
    if ((!direct && !raw.p) || !flat.p || !bounce.p || !comp.p) return false;
    CodecRequest req;
    const char* src;
    if (!direct) {
        gather_segments(in, static_cast<char*>(raw.p), bounce.p, &req.h2d);
        src = static_cast<const char*>(raw.p);
    } else if (one_pinned) {
        src = in.block_data(0);
    } else {
        in.copy_to(flat.p, n);
        src = flat.p;
    }
    req.comp.resize(nblk);
    for (size_t i = 0; i < nblk; ++i) {
        const size_t off = i * blk;
        req.comp[i] = SnappyJob{src + off, comp.p + i * cap, std::min<size_t>(blk, n - off), cap};
    }
    req.comp_max_ulen = (uint32_t)std::min(blk, n);
    // packed runs of the body are encoded into it first, in the same stream
    // sequence (the compress kernel reads what the run kernel wrote)
    if (runs) req.runs = *runs;
    // batched with the other RPCs' codec work: one launch sequence, one event
    if (RunCodecRequest(&req, dev) != 0) return false;
    for (int32_t e : req.run_err) {
        if (e) return false;
    }
    for (size_t i = 0; i < nblk; ++i) {
        if (req.comp_err[i] || req.comp_len[i] > cap) return false;
    }
    // one stream: total-length varint + each block's elements (its own
    // varint header stripped); the compressed bytes stay in the pinned
    // buffer, referenced zero-copy by the output Buf
    char hdr[10];
    out->append(hdr, put_varint(hdr, n));
    Buf whole;
    comp.give_to(&whole);
    size_t pos = 0;
    for (size_t i = 0; i < nblk; ++i) {
        const size_t h = (size_t)varint_len(req.comp[i].src_len);
        whole.pop_front(i * cap + h - pos);
        whole.cutn(out, req.comp_len[i] - h);
        pos = i * cap + req.comp_len[i];
    }
    return true;
}

// Cuts a raw snappy stream into pieces of <= limit uncompressed bytes whose
// copies stay inside the piece. False when malformed or not cuttable at
// this limit.
struct Piece {
    size_t comp_off, comp_len, ulen;
};
bool split_stream(const uint8_t* p, size_t n, size_t limit, size_t* total, std::vector<Piece>* pieces) {
    uint64_t ulen = 0;
    size_t i = 0;
    for (int shift = 0; shift <= 35; shift += 7) {
        if (i >= n) return false;
        const uint8_t c = p[i++];
        ulen |= (uint64_t)(c & 0x7f) << shift;
        if (!(c & 0x80)) break;
        if (shift == 35) return false;
    }
    *total = ulen;
    size_t piece_start_comp = i, piece_start_u = 0, upos = 0;
    while (i < n) {
        const size_t elem_start = i;
        const uint8_t tag = p[i++];
        size_t len = 0, off = 0;
        bool literal = false;
        switch (tag & 3) {
        case 0: {
            literal = true;
            size_t l = tag >> 2;
            if (l >= 60) {
                const int nb = (int)l - 59;
                if (i + nb > n) return false;
                l = 0;
                for (int k = 0; k < nb; ++k) l |= (size_t)p[i + k] << (8 * k);
                i += nb;
            }
            len = l + 1;
            if (len > n - i) return false;
            break;
        }
        case 1:
            if (i + 1 > n) return false;
            len = 4 + ((tag >> 2) & 7);
            off = ((size_t)(tag >> 5) << 8) | p[i];
            i += 1;
            break;
        case 2:
            if (i + 2 > n) return false;
            len = 1 + (tag >> 2);
            off = (size_t)p[i] | ((size_t)p[i + 1] << 8);
            i += 2;
            break;
        default:
            if (i + 4 > n) return false;
            len = 1 + (tag >> 2);
            off = (size_t)p[i] | ((size_t)p[i + 1] << 8) | ((size_t)p[i + 2] << 16) | ((size_t)p[i + 3] << 24);
            i += 4;
            break;
        }
        if (upos + len > ulen) return false;
        // start a new piece when this element would overflow the current one
        if (upos - piece_start_u + len > limit) {
            if (upos == piece_start_u) return false;  // one element larger than a piece
            pieces->push_back(Piece{piece_start_comp, elem_start - piece_start_comp, upos - piece_start_u});
            piece_start_comp = elem_start;
            piece_start_u = upos;
        }
        if (!literal && (off == 0 || off > upos - piece_start_u)) return false;  // crosses the piece start
        if (literal) i += len;
        upos += len;
    }
    if (upos != ulen) return false;
    if (upos > piece_start_u) pieces->push_back(Piece{piece_start_comp, n - piece_start_comp, upos - piece_start_u});
    return true;
}

// Uncompressed length from the stream's varint preamble (the first <= 5
// bytes, wherever the Buf's blocks are); false when malformed.
bool read_preamble(const Buf& in, uint64_t* ulen) {
    uint8_t h[5];
    const size_t n = in.copy_to(h, std::min<size_t>(sizeof(h), in.size()));
    uint64_t v = 0;
    for (size_t i = 0; i < n; ++i) {
        v |= (uint64_t)(h[i] & 0x7f) << (7 * i);
        if (!(h[i] & 0x80)) {
            *ulen = v;
            return true;
        }
    }
    return false;
}

// Top-level field table of a decompressed message (pb_scan layout).
struct PbIndex {
    std::vector<uint64_t> fields;
    int nfields = -1;  // pb_scan's count or negative code
};

// Decodes a raw snappy stream on the device into a pinned Buf. With `index`
// the output is decoded into HBM instead, pb_scan indexes it there, and one
// copy brings the bytes to pinned memory. The work joins the cross-RPC codec
// batch (gpu/codec_batch.h): one launch sequence and one event per batch.
bool gpu_decompress(const Buf& in, Buf* out, PbIndex* index = nullptr) {
    const int dev = g_device;
    uint64_t total = 0;
    if (!read_preamble(in, &total) || total > 0xFFFFFFFFull || in.size() > 0xFFFFFFFFull) return false;
    if (total == 0) return in.size() == 1;
    if (index && total > FLAGS_max_body_size) return false;
    // the compressed blocks go to HBM as they are (pinned socket blocks read
    // by the copy kernel, pageable ones bounced), cut into pieces either by
    // one host walk over the blocks in place or on the device
    const uint32_t limit = (uint32_t)std::max(1, std::min(64, FLAGS_gpu_snappy_block_kb)) << 10;
    std::vector<Piece> cuts;
    // compressed bytes already in HBM are cut on the device
    const bool host_cut = !FLAGS_gpu_snappy_device_split && in.all_host_accessible();
    if (host_cut) {
        // the walk needs contiguous bytes: the block itself, or a flat copy
        // of a stream spread over several blocks (host memory, only read)
        std::string flat;
        const uint8_t* bytes;
        if (in.backing_block_num() == 1) {
            bytes = reinterpret_cast<const uint8_t*>(in.block_data(0));
        } else {
            flat = in.to_string();
            bytes = reinterpret_cast<const uint8_t*>(flat.data());
        }
        // small pieces first (streams from device encoders: more waves, less
        // latency), then the 64 KiB fragments every host encoder respects
        size_t t = 0;
        if (!split_stream(bytes, in.size(), limit, &t, &cuts)) {
            cuts.clear();
            if (!split_stream(bytes, in.size(), kSnappyMaxBlock, &t, &cuts)) return false;
        }
    }
    // direct (host cut only): pieces are read from the pinned block (or one
    // flat pinned copy) and decoded straight into the pinned output, which
    // pb_scan reads in place; otherwise compressed bytes go to HBM and the
    // body comes back with a copy after the scan
    const bool direct = host_cut && FLAGS_gpu_snappy_direct_host;
    const bool one_pinned = in.backing_block_num() == 1 && in.ref_at(0).block->kind == MemKind::PINNED;
    const size_t pageable = direct ? 0 : pageable_bytes(in);
    PinnedBuf bounce(pageable ? pageable : 1), dst(total), cflat(direct && !one_pinned ? in.size() : 1);
    HbmTmp dcomp(direct ? 0 : in.size(), dev), dbody(index && !direct ? total : 0, dev);
    if (!bounce.p || !dst.p || !cflat.p || (!direct && !dcomp.p) || (index && !direct && !dbody.p)) return false;
    char* out_base = index && !direct ? static_cast<char*>(dbody.p) : dst.p;
    CodecRequest req;
    const char* comp_base;
    if (!direct) {
        gather_segments(in, static_cast<char*>(dcomp.p), bounce.p, &req.h2d);
        comp_base = static_cast<const char*>(dcomp.p);
    } else if (one_pinned) {
        comp_base = in.block_data(0);
    } else {
        in.copy_to(cflat.p, in.size());
        comp_base = cflat.p;
    }
    if (host_cut) {
        size_t upos = 0;
        for (const Piece& c : cuts) {
            req.pieces.push_back(SnappyPiece{comp_base + c.comp_off, out_base + upos,
                                             (uint32_t)c.comp_len, (uint32_t)c.ulen});
            req.pieces_max_ulen = std::max(req.pieces_max_ulen, (uint32_t)c.ulen);
            upos += c.ulen;
        }
    } else {
        req.streams.push_back(SnappyStream{dcomp.p, out_base, (uint32_t)in.size(), (uint32_t)total, 0,
                                           SnappyMaxPieces(total, limit)});
        req.stream_piece_limit = limit;
    }
    if (index) {
        req.scans.push_back(PbScanJob{reinterpret_cast<const uint8_t*>(out_base), total});
        if (host_cut) {
            // every piece decodes into this message: a fused batch scans it
            // as soon as its last piece is done
            req.scan_piece_first.push_back(0);
            req.scan_piece_count.push_back((uint32_t)req.pieces.size());
        }
        if (out_base != dst.p) req.d2h.push_back(Segment{dbody.p, dst.p, total});
    }
    if (RunCodecRequest(&req, dev) != 0) return false;
    for (int e : req.stream_err) {
        if (e) return false;
    }
    for (int e : req.piece_err) {
        if (e) return false;
    }
    if (index) {
        index->nfields = req.scan_nfields.empty() ? -1 : req.scan_nfields[0];
        index->fields.swap(req.scan_fields);
    }
    Buf whole;
    dst.give_to(&whole);
    out->append(std::move(whole));
    return true;
}

std::atomic<int64_t> g_indexed_parses{0}, g_index_fallbacks{0}, g_packs{0}, g_pack_runs{0}, g_pack_run_chunks{0},
    g_plain_routed{0};



// -gpu_snappy_packed_only on the receive side: whether a body carries a
// large packed run is only known once it is decoded, so the route adapts per
// message type (and worker). Types without packed numeric fields never go to
// the device; for the others, a device decode that found no run to unpack
// sends the next kPlainSkip bodies of the type to the CPU codec before the
// device probes again (the same adaptive skip as incompressible device
// payloads).
const uint32_t kPlainSkip = 31;
struct TypeRoute {
    bool packable = false;
    uint32_t skip = 0;
};
TypeRoute& route_of(const pb::Descriptor* d) {
    static thread_local std::unordered_map<const pb::Descriptor*, TypeRoute> routes;
    auto it = routes.find(d);
    if (it != routes.end()) return it->second;
    TypeRoute r;
    for (int i = 0; i < d->field_count() && !r.packable; ++i) {
        const pb::FieldDescriptor* f = d->field(i);
        r.packable = f->is_repeated() && f->packed && f->is_packable();
    }
    return routes.emplace(d, r).first->second;
}

// SetPbParseOffload hook: snappy decode + pb_scan in one device pass; the
// host merges the top-level fields from the table (bytes fields become one
// assign each, nested messages parse from their ranges).
int parse_offload(const Buf& in, CompressType type, pb::Message* msg) {
    if (type != COMPRESS_TYPE_SNAPPY || g_device < 0 || device_blocks_elsewhere(in, g_device)) return 0;
    TypeRoute* route = nullptr;
    if (FLAGS_gpu_snappy_packed_only) {
        route = &route_of(msg->GetDescriptor());
        if (!route->packable) return 0;
        if (route->skip > 0) {
            --route->skip;
            g_plain_routed.fetch_add(1, std::memory_order_relaxed);
            return 0;
        }
    }
    Span* span = IsRpczEnabled() ? Span::tls_parent() : nullptr;
    const int64_t t0 = span ? monotonic_us() : 0;
    PbIndex index;
    Buf raw;
    if (!gpu_decompress(in, &raw, &index)) {
        g_fallbacks.fetch_add(1, std::memory_order_relaxed);
        return 0;  // the CPU codec and parser take over
    }
    g_decomp_calls.fetch_add(1, std::memory_order_relaxed);
    bool ok;
    msg->Clear();
    const bool contiguous = raw.backing_block_num() <= 1;
    DeviceRunDecoder decoder;
    if (index.nfields >= 0 && contiguous &&
        msg->MergeFromFieldTable(raw.empty() ? nullptr : reinterpret_cast<const uint8_t*>(raw.block_data(0)),
                                 raw.size(), index.fields.data(), index.nfields,
                                 FLAGS_gpu_pb_unpack_min_bytes > 0 ? &decoder : nullptr)) {
        ok = msg->IsInitialized();
        g_indexed_parses.fetch_add(1, std::memory_order_relaxed);
        if (route && decoder.calls == 0) route->skip = kPlainSkip;  // a plain body: CPU for a while
    } else {
        // too many fields for the table, unknown fields, ...: the bytes are
        // already decoded, so only the parse runs on the host
        g_index_fallbacks.fetch_add(1, std::memory_order_relaxed);
        ok = msg->ParseFromBuf(raw);
    }
    if (span) {
        span->AnnotateDevice(string_printf("snappy decompress + pb_scan %zu -> %zu B, %d fields dev%d", in.size(),
                                           raw.size(), index.nfields, g_device),
                             (float)(monotonic_us() - t0) / 1000.0f);
    }
    return ok ? 1 : -1;
}

bool offload(const Buf& in, Buf* out, bool compress) {
    if (g_device < 0 || FLAGS_gpu_snappy_packed_only || device_blocks_elsewhere(in, g_device)) return false;
    Buf result;
    Span* span = IsRpczEnabled() ? Span::tls_parent() : nullptr;
    const int64_t t0 = span ? monotonic_us() : 0;
    const bool ok = compress ? gpu_compress(in, &result) : gpu_decompress(in, &result);
    if (span) {
        span->AnnotateDevice(string_printf("snappy %s %zu -> %zu B dev%d%s", compress ? "compress" : "decompress",
                                           in.size(), result.size(), g_device, ok ? "" : " (fell back to CPU)"),
                             (float)(monotonic_us() - t0) / 1000.0f);
    }
    if (!ok) {
        g_fallbacks.fetch_add(1, std::memory_order_relaxed);
        return false;  // the CPU codec takes over
    }
    (compress ? g_comp_calls : g_decomp_calls).fetch_add(1, std::memory_order_relaxed);
    out->append(std::move(result));
    return true;
}

// SetSnappyPackOffload hook: the message is serialized once, straight into
// a pinned block the compress kernel reads in place (no serialize-then-copy)
// Large packed varint fields are not encoded by the host at all: the
// serializer leaves their payload to pb_run_encode_kernel, which writes it
// into the pinned body in the same codec batch, right before the compress
// kernel reads the body (SURVEY K2 on the path).
bool pack_offload(const pb::Message& msg, size_t n, Buf* out) {
    if (g_device < 0 || n == 0 || !FLAGS_gpu_snappy_direct_host) return false;
    PinnedBuf body(n);
    if (!body.p) return false;
    RunCollector col;
    pb::PackedRunSink* prev = pb::SetThreadPackedRunSink(FLAGS_gpu_pb_pack_min_elems > 0 ? &col : nullptr);
    uint8_t* e = msg.SerializeWithCachedSizesToArray(reinterpret_cast<uint8_t*>(body.p));
    pb::SetThreadPackedRunSink(prev);
    if ((size_t)(e - reinterpret_cast<uint8_t*>(body.p)) != n) return false;
    std::vector<PbRunChunk> chunks;
    bool device_runs = !col.runs.empty();
    PinnedBuf stage(0);  // values of the runs, only when there are any
    if (device_runs) stage = PinnedBuf(col.value_bytes + 16 * col.runs.size());
    if (device_runs && (!stage.p || !stage_runs(col, &stage, &chunks))) {
        for (const pb::PackedRun& r : col.runs) pb::EncodePackedRunOnHost(r);
        device_runs = false;
    }
    Buf raw;
    body.give_to(&raw);
    if (FLAGS_gpu_snappy_packed_only && !device_runs) {
        // no packed run large enough for the device: the CPU codec compresses
        // the body we already serialized
        g_plain_routed.fetch_add(1, std::memory_order_relaxed);
        return CompressBuf(COMPRESS_TYPE_SNAPPY, raw, out);
    }
    Buf result;
    bool ok;
    {
        Span* span = IsRpczEnabled() ? Span::tls_parent() : nullptr;
        const int64_t t0 = span ? monotonic_us() : 0;
        ok = gpu_compress(raw, &result, device_runs ? &chunks : nullptr);
        if (span) {
            span->AnnotateDevice(string_printf("pb pack (%zu packed runs, %zu chunks) + snappy compress %zu -> %zu B dev%d%s",
                                               col.runs.size(), chunks.size(), n, result.size(), g_device,
                                               ok ? "" : " (fell back to CPU)"),
                                 (float)(monotonic_us() - t0) / 1000.0f);
        }
    }
    if (!ok) {
        // the device did not finish: the host encodes what it skipped and
        // the CPU codec compresses the same bytes
        g_fallbacks.fetch_add(1, std::memory_order_relaxed);
        if (device_runs) {
            for (const pb::PackedRun& r : col.runs) pb::EncodePackedRunOnHost(r);
        }
        return CompressBuf(COMPRESS_TYPE_SNAPPY, raw, out);
    }
    g_comp_calls.fetch_add(1, std::memory_order_relaxed);
    if (device_runs) {
        g_pack_runs.fetch_add((int64_t)col.runs.size(), std::memory_order_relaxed);
        g_pack_run_chunks.fetch_add((int64_t)chunks.size(), std::memory_order_relaxed);
    }
    g_packs.fetch_add(1, std::memory_order_relaxed);
    out->append(std::move(result));
    return true;
}

}  // namespace

namespace {

size_t run_elem_bytes(uint32_t kind) {
    switch (kind) {
    case PB_RUN_BOOL: return 1;
    case PB_RUN_INT32:
    case PB_RUN_UINT32:
    case PB_RUN_SINT32: return 4;
    default: return 8;
    }
}

// Output bytes of element p under kind/format (the host size pass; the
// kernel checks it chunk by chunk).
size_t run_elem_len(const char* p, uint32_t kind, uint32_t format) {
    int64_t sv = 0;
    uint64_t uv = 0;
    bool is_signed = false;
    switch (kind) {
    case PB_RUN_BOOL: return format == PB_RUN_VARINT ? 1 : (*(const uint8_t*)p ? 4 : 5);
    case PB_RUN_INT32: sv = *(const int32_t*)p; is_signed = true; break;
    case PB_RUN_SINT32: sv = *(const int32_t*)p; is_signed = true; break;
    case PB_RUN_UINT32: uv = *(const uint32_t*)p; break;
    case PB_RUN_INT64:
    case PB_RUN_SINT64: sv = *(const int64_t*)p; is_signed = true; break;
    default: uv = *(const uint64_t*)p; break;
    }
    if (format == PB_RUN_VARINT) {
        uint64_t w;
        if (kind == PB_RUN_SINT32) w = (uint32_t)(((uint32_t)sv << 1) ^ (uint32_t)((int32_t)sv >> 31));
        else if (kind == PB_RUN_SINT64) w = ((uint64_t)sv << 1) ^ (uint64_t)(sv >> 63);
        else w = is_signed ? (uint64_t)sv : uv;
        return (size_t)varint_len(w);
    }
    const bool neg = is_signed && sv < 0;
    const uint64_t mag = is_signed ? (neg ? (uint64_t)0 - (uint64_t)sv : (uint64_t)sv) : uv;
    size_t d = 1;
    for (uint64_t p = 10; d < 20 && mag >= p; p *= 10) ++d;
    return d + (neg ? 1 : 0);
}

}  // namespace

int EncodeRunOnDevice(const void* values, size_t n, uint32_t kind, uint32_t format, std::string* out, int device) {
    out->clear();
    if (n == 0) return 0;
    if (kind > PB_RUN_BOOL || format > PB_RUN_DECIMAL || device < 0) return -1;
    if (Init(device) != 0) return -1;
    const size_t eb = run_elem_bytes(kind);
    const char* v = static_cast<const char*>(values);
    std::vector<PbRunChunk> chunks;
    size_t total = 0;
    for (size_t c = 0; c < n; c += kPbRunChunkElems) {
        const size_t e = std::min(n, c + kPbRunChunkElems);
        size_t cb = 0;
        for (size_t i = c; i < e; ++i) cb += run_elem_len(v + i * eb, kind, format) + (format == PB_RUN_DECIMAL && i + 1 < n);
        PbRunChunk ch;
        ch.src = nullptr;
        ch.dst = nullptr;
        ch.count = (uint32_t)(e - c);
        ch.kind = kind;
        ch.format = format;
        ch.last = e == n ? 1 : 0;
        ch.bytes = (uint32_t)cb;
        ch.pad = 0;
        chunks.push_back(ch);
        total += cb;
    }
    PinnedBuf stage(n * eb), dst(total ? total : 1);
    if (!stage.p || !dst.p) return -1;
    memcpy(stage.p, values, n * eb);
    size_t off = 0;
    for (size_t k = 0; k < chunks.size(); ++k) {
        chunks[k].src = stage.p + k * kPbRunChunkElems * eb;
        chunks[k].dst = reinterpret_cast<uint8_t*>(dst.p) + off;
        off += chunks[k].bytes;
    }
    CodecRequest req;
    req.runs = chunks;
    if (RunCodecRequest(&req, device) != 0) return -1;
    for (int32_t e : req.run_err) {
        if (e) return -1;
    }
    out->assign(dst.p, total);
    return 0;
}

int DecodeRunOnDevice(const void* bytes, size_t len, uint32_t kind, std::string* out, int device) {
    out->clear();
    if (kind > PB_RUN_BOOL || device < 0 || Init(device) != 0) return -1;
    if (len == 0) return 0;
    PinnedBuf in(len);
    if (!in.p) return -1;
    memcpy(in.p, bytes, len);
    std::vector<pb::PackedRunIn> runs(1);
    runs[0].p = reinterpret_cast<const uint8_t*>(in.p);
    runs[0].len = len;
    runs[0].elem_bytes = run_elem_bytes(kind);
    // run_kind() maps field types; here the kind is given directly
    static const pb::FieldType kTypes[] = {pb::FieldType::INT32,  pb::FieldType::UINT32, pb::FieldType::SINT32,
                                           pb::FieldType::INT64,  pb::FieldType::UINT64, pb::FieldType::SINT64,
                                           pb::FieldType::BOOL};
    runs[0].type = kTypes[kind];
    PinnedBuf dec(1);
    if (!decode_runs(&runs, &dec, device) || !runs[0].values) return -1;
    out->assign(static_cast<const char*>(runs[0].values), runs[0].count * runs[0].elem_bytes);
    return 0;
}

int EnableGpuSnappy(int device, size_t min_bytes, std::string* error) {
    if (Init(device, error) != 0 || InitHbmPool(device, error) != 0) return -1;
    g_device = device;
    SetSnappyOffload(offload, min_bytes);
    SetPbParseOffload(parse_offload, min_bytes);
    SetSnappyPackOffload(pack_offload, min_bytes);
    static var::PassiveStatus<int64_t> v6("gpu_snappy_packs", [] { return g_packs.load(); });
    static var::PassiveStatus<int64_t> v7("gpu_pb_pack_runs", [] { return g_pack_runs.load(); });
    static var::PassiveStatus<int64_t> v8("gpu_pb_unpack_runs", [] { return g_unpack_runs.load(); });
    static var::PassiveStatus<int64_t> v1("gpu_snappy_compress_calls", [] { return g_comp_calls.load(); });
    static var::PassiveStatus<int64_t> v2("gpu_snappy_decompress_calls", [] { return g_decomp_calls.load(); });
    static var::PassiveStatus<int64_t> v3("gpu_snappy_fallbacks", [] { return g_fallbacks.load(); });
    static var::PassiveStatus<int64_t> v4("gpu_pb_indexed_parses", [] { return g_indexed_parses.load(); });
    static var::PassiveStatus<int64_t> v5("gpu_pb_index_fallbacks", [] { return g_index_fallbacks.load(); });
    return 0;
}

void DisableGpuSnappy() {
    SetSnappyOffload(nullptr, (size_t)-1);
    SetPbParseOffload(nullptr, (size_t)-1);
    SetSnappyPackOffload(nullptr, (size_t)-1);
}

GpuSnappyStats GetGpuSnappyStats() {
    GpuSnappyStats s;
    s.compress_calls = g_comp_calls.load();
    s.decompress_calls = g_decomp_calls.load();
    s.fallbacks = g_fallbacks.load();
    s.indexed_parses = g_indexed_parses.load();
    s.index_fallbacks = g_index_fallbacks.load();
    s.packs = g_packs.load();
    s.pack_runs = g_pack_runs.load();
    s.plain_routed = g_plain_routed.load();
    s.pack_run_chunks = g_pack_run_chunks.load();
    s.unpack_runs = g_unpack_runs.load();
    s.unpack_fallbacks = g_unpack_fallbacks.load();
    return s;
}

}  // namespace gpu
}  // namespace mrpc
