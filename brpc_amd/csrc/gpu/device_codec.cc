#include "gpu/device_codec.h"

#include <algorithm>
#include <atomic>
#include <vector>

#include "base/flags.h"
#include "base/pool.h"
#include "gpu/codec_batch.h"
#include "gpu/hbm_pool.h"
#include "gpu/kernels.h"
#include "policy/device_payload.h"

DEFINE_int32(device_payload_block_kb, 2,
             "uncompressed KiB per device snappy block of a compressed device payload (one wave each); 1..64. "
             "Smaller blocks spread a payload over more waves: on MI355X the 64 KiB text leg runs 121k QPS at 2 KiB "
             "(ratio 1.96) against 80k at 4 KiB (ratio 2.24)");

namespace mrpc {
namespace gpu {

namespace {

std::atomic<int64_t> g_encodes{0}, g_enc_bytes{0}, g_enc_out{0}, g_decodes{0}, g_dec_bytes{0}, g_bad_tables{0},
    g_dec_err{0}, g_scans{0}, g_runs{0}, g_run_bytes{0}, g_run_elems{0}, g_run_err{0};

uint32_t varint_len(uint64_t v) {
    uint32_t n = 1;
    while (v >= 0x80) {
        v >>= 7;
        ++n;
    }
    return n;
}

uint32_t block_len(const DeviceSnappyLayout& lay, uint64_t len, uint32_t i) {
    const uint64_t off = (uint64_t)i * lay.block_ulen;
    return (uint32_t)std::min<uint64_t>(lay.block_ulen, len - off);
}

// A table that cannot describe `len` bytes inside the region is refused
// before anything runs on the device: every block lies inside the region,
// holds at least its header, and the blocks cover the payload exactly.
bool table_ok(const DeviceSnappyBlocks& j) {
    const DeviceSnappyLayout& l = j.lay;
    if (!j.region || !j.dst || !j.clen || j.len == 0 || l.block_ulen == 0 || l.block_ulen > kSnappyMaxBlock ||
        l.nblocks == 0 || l.stride == 0) {
        return false;
    }
    if ((uint64_t)l.nblocks != (j.len + l.block_ulen - 1) / l.block_ulen) return false;
    for (uint32_t i = 0; i < l.nblocks; ++i) {
        const uint64_t c = j.clen[i];
        const uint32_t ul = block_len(l, j.len, i);
        if (c <= varint_len(ul) || c > l.stride || (uint64_t)i * l.stride + c > j.region_len) return false;
    }
    return true;
}

void fill_index(const CodecRequest& req, size_t row, DevicePayloadIndex* out) {
    out->nfields = req.scan_nfields[row];
    const uint64_t* f = req.scan_fields.data() + row * 2 * kCodecScanFields;
    const int n = std::max(0, std::min<int>(out->nfields, (int)kCodecScanFields));
    out->fields.assign(f, f + 2 * n);
}

// A CodecRequest from the object pool, emptied but with its vectors'
// capacity (the encode and decode of every device-body RPC build one).
struct PooledRequest {
    CodecRequest* r;
    PooledRequest() : r(get_object<CodecRequest>()) { r->Reset(); }
    ~PooledRequest() { return_object(r); }
    PooledRequest(const PooledRequest&) = delete;
    PooledRequest& operator=(const PooledRequest&) = delete;
};

}  // namespace

DeviceSnappyLayout DeviceSnappyLayoutFor(size_t len) {
    DeviceSnappyLayout l;
    l.block_ulen = (uint32_t)std::max(1, std::min(64, FLAGS_device_payload_block_kb)) << 10;
    l.stride = (uint32_t)((SnappyMaxCompressedLength(l.block_ulen) + 15) & ~15ull);
    l.nblocks = (uint32_t)((len + l.block_ulen - 1) / l.block_ulen);
    return l;
}

int DeviceSnappyEncode(const void* src, size_t len, void* dst, const DeviceSnappyLayout& lay, uint32_t* clen,
                       int device) {
    if (!src || !dst || len == 0 || lay.nblocks == 0) return -1;
    const char* s = static_cast<const char*>(src);
    char* d = static_cast<char*>(dst);
    PooledRequest pooled;
    CodecRequest& req = *pooled.r;
    req.comp.resize(lay.nblocks);
    for (uint32_t i = 0; i < lay.nblocks; ++i) {
        req.comp[i] = SnappyJob{s + (size_t)i * lay.block_ulen, d + (size_t)i * lay.stride, block_len(lay, len, i),
                                lay.stride};
    }
    req.comp_max_ulen = (uint32_t)std::min<uint64_t>(lay.block_ulen, len);
    if (RunCodecRequest(&req, device) != 0) return -1;
    uint64_t out = 0;
    for (uint32_t i = 0; i < lay.nblocks; ++i) {
        if (req.comp_err[i] || req.comp_len[i] > lay.stride || req.comp_len[i] == 0) return -1;
        clen[i] = req.comp_len[i];
        out += clen[i];
    }
    g_encodes.fetch_add(1, std::memory_order_relaxed);
    g_enc_bytes.fetch_add((int64_t)len, std::memory_order_relaxed);
    g_enc_out.fetch_add((int64_t)out, std::memory_order_relaxed);
    return 0;
}

int DeviceSnappyDecode(const DeviceSnappyBlocks* jobs, int n, int* err, DevicePayloadIndex* index, int device) {
    PooledRequest pooled;
    CodecRequest& req = *pooled.r;
    std::vector<size_t> first(n, 0), count(n, 0), scan_row(n, (size_t)-1);
    for (int k = 0; k < n; ++k) {
        const DeviceSnappyBlocks& j = jobs[k];
        err[k] = 0;
        if (!table_ok(j)) {
            err[k] = 1;
            g_bad_tables.fetch_add(1, std::memory_order_relaxed);
            continue;
        }
        first[k] = req.pieces.size();
        count[k] = j.lay.nblocks;
        char* d = static_cast<char*>(j.dst);
        for (uint32_t i = 0; i < j.lay.nblocks; ++i) {
            const uint32_t ul = block_len(j.lay, j.len, i);
            const uint32_t h = varint_len(ul);
            // headerless pieces: the block's varint length is known from the
            // table, the decoder starts at its first element
            req.pieces.push_back(SnappyPiece{j.region + (size_t)i * j.lay.stride + h, d + (size_t)i * j.lay.block_ulen,
                                             j.clen[i] - h, ul});
        }
        req.pieces_max_ulen = std::max(req.pieces_max_ulen, std::min<uint32_t>(j.lay.block_ulen, (uint32_t)j.len));
        if (j.scan && index) {
            scan_row[k] = req.scans.size();
            req.scans.push_back(PbScanJob{static_cast<const uint8_t*>(j.dst), j.len});
            req.scan_piece_first.push_back((uint32_t)first[k]);
            req.scan_piece_count.push_back(j.lay.nblocks);
        }
    }
    if (req.pieces.empty()) return 0;
    if (RunCodecRequest(&req, device) != 0) return -1;
    for (int k = 0; k < n; ++k) {
        if (err[k]) continue;
        for (size_t p = first[k]; p < first[k] + count[k]; ++p) {
            if (req.piece_err[p]) {
                err[k] = 2;
                g_dec_err.fetch_add(1, std::memory_order_relaxed);
                break;
            }
        }
        if (err[k]) continue;
        g_decodes.fetch_add(1, std::memory_order_relaxed);
        g_dec_bytes.fetch_add((int64_t)jobs[k].len, std::memory_order_relaxed);
        if (scan_row[k] != (size_t)-1) {
            fill_index(req, scan_row[k], &index[k]);
            g_scans.fetch_add(1, std::memory_order_relaxed);
        }
    }
    return 0;
}

int DevicePbScan(const void* const* bufs, const uint64_t* lens, int n, DevicePayloadIndex* index, int device) {
    if (n <= 0) return 0;
    CodecRequest req;
    for (int k = 0; k < n; ++k) req.scans.push_back(PbScanJob{static_cast<const uint8_t*>(bufs[k]), lens[k]});
    if (RunCodecRequest(&req, device) != 0) return -1;
    for (int k = 0; k < n; ++k) fill_index(req, (size_t)k, &index[k]);
    g_scans.fetch_add(n, std::memory_order_relaxed);
    return 0;
}

bool DevicePayloadField(const DevicePayloadIndex& index, uint32_t number, uint64_t* off, uint64_t* len) {
    const int n = std::min<int>(index.nfields, (int)(index.fields.size() / 2));
    for (int k = 0; k < n; ++k) {
        const uint64_t key = index.fields[2 * k];
        if ((key >> 3) != number || (key & 7) != 2) continue;
        const uint64_t v = index.fields[2 * k + 1];
        *off = v >> 32;
        *len = v & 0xFFFFFFFFull;
        return true;
    }
    return false;
}

int DeviceDecodePackedRuns(DevicePackedRun* runs, int n, int device) {
    if (n <= 0) return 0;
    CodecRequest req;
    std::vector<size_t> first(n + 1, 0);
    for (int i = 0; i < n; ++i) {
        DevicePackedRun& r = runs[i];
        first[i] = req.dec_runs.size();
        r.count = 0;
        r.err = 0;
        if (!r.src || !r.dst || r.kind > PB_RUN_BOOL || r.len > 0xFFFFFFFFull) {
            r.err = 2;
            continue;
        }
        if (r.len == 0) continue;
        const uint32_t head = (uint32_t)req.dec_runs.size();
        for (uint64_t o = 0; o < r.len; o += kPbRunDecodeChunkBytes) {
            PbRunDecodeChunk c;
            c.run = static_cast<const uint8_t*>(r.src);
            c.dst = r.dst;
            c.offset = (uint32_t)o;
            c.len = (uint32_t)std::min<uint64_t>(kPbRunDecodeChunkBytes, r.len - o);
            c.first = head;
            c.kind = r.kind;
            req.dec_runs.push_back(c);
        }
    }
    first[n] = req.dec_runs.size();
    if (req.dec_runs.empty()) return 0;
    // every run's final byte comes back with the batch (the host cannot read
    // HBM): one still carrying a continuation bit ends inside a varint
    uint8_t* tail = static_cast<uint8_t*>(PinnedAlloc((size_t)n));
    if (!tail) return -1;
    for (int i = 0; i < n; ++i) {
        tail[i] = 0;
        if (first[i + 1] > first[i]) {
            req.d2h.push_back(Segment{static_cast<const uint8_t*>(runs[i].src) + runs[i].len - 1, tail + i, 1});
        }
    }
    if (RunCodecRequest(&req, device) != 0) {
        PinnedFree(tail, (size_t)n);
        return -1;
    }
    for (int i = 0; i < n; ++i) {
        DevicePackedRun& r = runs[i];
        if (r.err || r.len == 0) continue;
        uint64_t count = 0;
        for (size_t k = first[i]; k < first[i + 1]; ++k) {
            count += req.dec_counts[k];
            if (req.dec_err[k]) r.err = 1;
        }
        if (tail[i] & 0x80) r.err = 1;
        if (r.err) {
            g_run_err.fetch_add(1, std::memory_order_relaxed);
            continue;
        }
        r.count = count;
        g_runs.fetch_add(1, std::memory_order_relaxed);
        g_run_bytes.fetch_add((int64_t)r.len, std::memory_order_relaxed);
        g_run_elems.fetch_add((int64_t)count, std::memory_order_relaxed);
    }
    PinnedFree(tail, (size_t)n);
    return 0;
}

DeviceCodecStats GetDeviceCodecStats() {
    DeviceCodecStats s;
    s.encodes = g_encodes.load();
    s.encoded_bytes = g_enc_bytes.load();
    s.encoded_out_bytes = g_enc_out.load();
    s.decodes = g_decodes.load();
    s.decoded_bytes = g_dec_bytes.load();
    s.bad_tables = g_bad_tables.load();
    s.decode_errors = g_dec_err.load();
    s.scans = g_scans.load();
    s.packed_runs = g_runs.load();
    s.packed_bytes = g_run_bytes.load();
    s.packed_elems = g_run_elems.load();
    s.packed_errors = g_run_err.load();
    return s;
}

}  // namespace gpu
}  // namespace mrpc
