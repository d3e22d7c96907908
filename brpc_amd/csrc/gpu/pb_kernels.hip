// Batched protobuf wire scan on CDNA4 (gfx950): the device half of the pb
// "unpack" (SURVEY K1 — the per-message tag/varint walk of
// ParsePbFromIOBuf, protocol.h:207, and of RpcMeta at
// baidu_rpc_protocol.cpp:323,563). Many small messages (RpcMeta-sized,
// 20-200 bytes) are packed back to back in HBM with an int64 offset table;
// one launch decodes every top-level field of every message into a
// fixed-width table:
//   fields[i][k] = { (field_number << 3) | wire_type, value }
// where value is the varint (wire 0), the little-endian fixed64/fixed32
// (wires 1/5), or (offset_in_message << 32) | length for length-delimited
// fields (wire 2), which a second pass (or the host) can descend into.
// nfields[i] = number of fields, or a negative code: -1 truncated/malformed,
// -2 more than max_fields fields, -3 field number 0, -4 unsupported wire
// type (proto2 groups), -5 offsets outside the buffer or descending (the
// message is not read at all).
//
// Layout: one lane per message. Messages are tiny and independent, so the
// serial tag walk of one message costs one lane, not one wave; a lane reads
// its message sequentially (the 128-byte lines it touches stay in L1 while
// the lane walks them) and writes its field rows with 16-byte stores.
#include <hip/hip_runtime.h>

#include "gpu/kernels.h"
#include "gpu/device_pb.h"

namespace mrpc {
namespace gpu {

namespace {

typedef const __attribute__((address_space(1))) uint8_t gbyte_c;

__global__ void __launch_bounds__(256) pb_scan_kernel(const uint8_t* __restrict__ buf_,
                                                      uint64_t buf_len, const int64_t* __restrict__ offsets,
                                                      int64_t n, uint32_t max_fields, uint64_t* __restrict__ fields,
                                                      int32_t* __restrict__ nfields) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    gbyte_c* b = (gbyte_c*)buf_;
    const int64_t so = offsets[i], eo = offsets[i + 1];
    // never trust the offset table: a message must lie inside the buffer
    if (so < 0 || eo < so || (uint64_t)eo > buf_len) {
        nfields[i] = -5;
        return;
    }
    const uint64_t start = (uint64_t)so;
    const uint64_t end = (uint64_t)eo;
    nfields[i] = devpb::scan_message(b, start, end, fields + (uint64_t)i * max_fields * 2, max_fields);
}

// Messages in separate buffers (one per job): the batched codec path, where
// every request decoded its body into its own HBM block.
__global__ void __launch_bounds__(256) pb_scan_ptrs_kernel(const PbScanJob* __restrict__ jobs, int64_t n,
                                                           uint32_t max_fields, uint64_t* __restrict__ fields,
                                                           int32_t* __restrict__ nfields) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const PbScanJob job = jobs[i];
    nfields[i] = devpb::scan_message((gbyte_c*)job.buf, 0, job.len, fields + (uint64_t)i * max_fields * 2, max_fields);
}

// ------------------------------------------------------------ run encoder
// The device half of body encode (the reference serializes every
// body on the host: SerializeAsCompressedData, src/brpc/compress.cpp:92,
// called from baidu_rpc_protocol.cpp's response path) and of pb2json's
// number printing (src/json2pb/pb_to_json.cpp, K6).
// One workgroup (4 waves) per PbRunChunk. The chunk is walked in 8 rounds
// of 256 consecutive elements: lane t of round r takes element 256r + t
// (a coalesced 1/4/8-byte load from the source, pinned host or HBM), the
// encoded lengths are block-scanned (wave shuffles + 4 wave totals in LDS)
// and every lane writes its bytes into the chunk's output image in LDS
// (<= 21 B per element: 43 KiB). The image then leaves with byte stores
// that are contiguous across the lanes of each instruction, so a host
// destination sees full-line PCIe writes instead of one small write per
// varint.
constexpr int kRunThreads = 256;
constexpr uint32_t kRunMaxElemBytes = 21;  // "-9223372036854775808" + ','

// Raw element bits: signed 32-bit kinds sign-extended, bools as 0/1.
__device__ __forceinline__ uint64_t run_load(const void* src, uint32_t i, uint32_t kind) {
    switch (kind) {
    case PB_RUN_INT32:
    case PB_RUN_SINT32: return (uint64_t)(int64_t)static_cast<const int32_t*>(src)[i];
    case PB_RUN_UINT32: return static_cast<const uint32_t*>(src)[i];
    case PB_RUN_BOOL: return static_cast<const uint8_t*>(src)[i] ? 1 : 0;
    default: return static_cast<const uint64_t*>(src)[i];
    }
}

// Wire value of an element (zigzag for sint kinds).
__device__ __forceinline__ uint64_t run_value(uint64_t raw, uint32_t kind) {
    switch (kind) {
    case PB_RUN_SINT32: {
        const int32_t v = (int32_t)raw;
        return (uint32_t)(((uint32_t)v << 1) ^ (uint32_t)(v >> 31));
    }
    case PB_RUN_SINT64: return (raw << 1) ^ (uint64_t)((int64_t)raw >> 63);
    default: return raw;
    }
}

// For decimal output the value is printed as its field type says: signed
// kinds as two's complement of their width (zigzag undone: the JSON shows
// the number, not its wire form).
__device__ __forceinline__ bool run_negative(uint64_t raw, uint32_t kind, uint64_t* mag) {
    const bool is_signed = kind == PB_RUN_INT32 || kind == PB_RUN_SINT32 || kind == PB_RUN_INT64 ||
                           kind == PB_RUN_SINT64;
    const bool neg = is_signed && (int64_t)raw < 0;
    *mag = neg ? (uint64_t)0 - raw : raw;
    return neg;
}

__device__ __forceinline__ uint32_t run_varint_len(uint64_t v) {
    const int bits = v ? 64 - __clzll(v) : 1;
    return (uint32_t)((bits + 6) / 7);
}

__device__ __forceinline__ uint32_t run_digits(uint64_t v) {
    uint32_t d = 1;
    uint64_t p = 10;
    while (d < 20 && v >= p) {
        ++d;
        p *= 10;
    }
    return d;
}

// Copies an LDS image to dst (any alignment) with 16-byte stores for the
// aligned middle: over PCIe to pinned host memory a wave's byte stores make
// 64-byte writes, its 16-byte stores 1 KiB ones.
__device__ __forceinline__ void copy_out(uint8_t* dst, const uint8_t* image, uint32_t total) {
    const uint32_t t = threadIdx.x;
    uint32_t head = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15);
    if (head > total) head = total;
    if (t < head) dst[t] = image[t];
    const uint32_t nv = (total - head) / 16;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4* body = reinterpret_cast<u32x4*>(dst + head);
    for (uint32_t w = t; w < nv; w += kRunThreads) {
        const uint8_t* q = image + head + 16 * w;
        u32x4 v;
        v.x = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
        v.y = (uint32_t)q[4] | ((uint32_t)q[5] << 8) | ((uint32_t)q[6] << 16) | ((uint32_t)q[7] << 24);
        v.z = (uint32_t)q[8] | ((uint32_t)q[9] << 8) | ((uint32_t)q[10] << 16) | ((uint32_t)q[11] << 24);
        v.w = (uint32_t)q[12] | ((uint32_t)q[13] << 8) | ((uint32_t)q[14] << 16) | ((uint32_t)q[15] << 24);
        body[w] = v;
    }
    for (uint32_t j = head + 16 * nv + t; j < total; j += kRunThreads) dst[j] = image[j];
}

__global__ void __launch_bounds__(kRunThreads) pb_run_encode_kernel(const PbRunChunk* __restrict__ chunks,
                                                                    int32_t* __restrict__ err) {
    __shared__ uint8_t image[kPbRunChunkElems * kRunMaxElemBytes];
    __shared__ uint32_t wave_tot[kRunThreads / 64];
    __shared__ uint32_t round_base;
    const PbRunChunk c = chunks[blockIdx.x];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const bool decimal = c.format == PB_RUN_DECIMAL;
    if (t == 0) round_base = 0;
    __syncthreads();
    const uint32_t count = c.count < kPbRunChunkElems ? c.count : kPbRunChunkElems;
    // every round's element is loaded before any is used: from pinned host
    // memory each load is a PCIe round trip, so the 8 go out together
    // instead of one per round behind the scan's barriers
    constexpr int kRounds = kPbRunChunkElems / kRunThreads;
    uint64_t raws[kRounds];
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t i = (uint32_t)r * kRunThreads + t;
        raws[r] = i < count ? run_load(c.src, i, c.kind) : 0;
    }
#pragma unroll
    for (int r = 0; r < kRounds; ++r) {
        const uint32_t r0 = (uint32_t)r * kRunThreads;
        if (r0 >= count) break;
        const uint32_t i = r0 + t;
        uint32_t len = 0;
        uint64_t v = 0;
        bool neg = false;
        if (i < count) {
            if (!decimal) {
                v = run_value(raws[r], c.kind);
                len = run_varint_len(v);
            } else if (c.kind == PB_RUN_BOOL) {
                v = raws[r];
                len = v ? 4 : 5;
            } else {
                neg = run_negative(raws[r], c.kind, &v);
                len = run_digits(v) + (neg ? 1 : 0);
            }
            if (decimal && !(c.last && i + 1 == count)) len += 1;  // ','
        }
        // block exclusive scan of len in element order
        uint32_t incl = len;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wave_tot[wave] = incl;
        __syncthreads();
        uint32_t pos = round_base + incl - len;
        for (int w = 0; w < wave; ++w) pos += wave_tot[w];
        const uint32_t round_total = wave_tot[0] + wave_tot[1] + wave_tot[2] + wave_tot[3];
        if (i < count) {
            uint8_t* o = image + pos;
            if (!decimal) {
                for (uint32_t j = 0; j < len; ++j) {
                    o[j] = (uint8_t)((v & 0x7f) | (j + 1 < len ? 0x80 : 0));
                    v >>= 7;
                }
            } else if (c.kind == PB_RUN_BOOL) {
                const char* s = v ? "true" : "false";
                const uint32_t n = v ? 4 : 5;
                for (uint32_t j = 0; j < n; ++j) o[j] = (uint8_t)s[j];
                if (len > n) o[n] = ',';
            } else {
                const uint32_t nd = run_digits(v);
                uint32_t k = 0;
                if (neg) o[k++] = '-';
                for (uint32_t j = 0; j < nd; ++j) {
                    const uint64_t q = v / 10;
                    o[k + nd - 1 - j] = (uint8_t)('0' + (uint32_t)(v - q * 10));
                    v = q;
                }
                k += nd;
                if (len > k) o[k] = ',';
            }
        }
        __syncthreads();  // wave_tot is rewritten by the next round
        if (t == 0) round_base += round_total;
        __syncthreads();
    }
    const uint32_t total = round_base;
    if (total != c.bytes) {
        if (t == 0) err[blockIdx.x] = 1;
        return;
    }
    copy_out(c.dst, image, total);
    if (t == 0) err[blockIdx.x] = 0;
}

// ------------------------------------------------------------ run decoder
// Packed fields of a decoded body (the reference's ParsePbFromIOBuf walks
// them element by element on the host, src/brpc/protocol.cpp).
// Both passes read the chunk (plus up to 16 bytes of the run before it)
// with 16-byte loads of the aligned span around it (a byte outside the run
// shares its aligned 16 bytes with a byte inside, so with its page): a
// wave's load moves 1 KiB instead of the 64 bytes of per-lane byte loads,
// which held the count pass to ~1 TB/s on HBM. Lane t then owns chunk bytes
// [16t, 16t + 16) of the staged copy.
constexpr int kHalo = 16;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// staged at raw + kPad: every lane's 32-byte window (16 bytes before its
// own 16) stays inside the array
constexpr int kPad = 16;
constexpr int kStage16 = (kPad + kHalo + kPbRunDecodeChunkBytes + 64) / 16;

// Stages [p, p + n) into lds (n <= kHalo + chunk); returns the LDS byte
// offset of p.
__device__ __forceinline__ uint32_t stage_aligned(const uint8_t* p, uint32_t n, u32x4* lds) {
    const uint32_t a = (uint32_t)((uintptr_t)p & 15);
    const u32x4* src = reinterpret_cast<const u32x4*>(p - a);
    const uint32_t n16 = (a + n + 15) >> 4;
    u32x4 v[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t i = threadIdx.x + (uint32_t)k * kRunThreads;
        if (i < n16) v[k] = src[i];
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const uint32_t i = threadIdx.x + (uint32_t)k * kRunThreads;
        if (i < n16) lds[i] = v[k];
    }
    return a;
}

// Bits 0..3 of each nibble k: byte k of w ends a varint (top bit clear).
__device__ __forceinline__ uint32_t ends_of(uint32_t w) {
    const uint32_t m = ~w & 0x80808080u;
    return ((m >> 7) & 1) | ((m >> 14) & 2) | ((m >> 21) & 4) | ((m >> 28) & 8);
}

__global__ void __launch_bounds__(kRunThreads) pb_run_count_kernel(const PbRunDecodeChunk* __restrict__ chunks,
                                                                   int nchunks, uint32_t* __restrict__ counts,
                                                                   uint32_t* __restrict__ prefix) {
    // one wave per chunk, straight from the loads (no LDS, no barriers):
    // varint ends are bytes with the top bit clear, counted 16 at a time
    // inside [0, len). Every lane issues its (up to 5) 16-byte loads before
    // using any, so a wave keeps a whole 4 KiB chunk in flight; one load per
    // lane and a block-wide reduction per chunk held this pass to ~1 TB/s
    constexpr int kUnits = (kPbRunDecodeChunkBytes + 16 + 63 * 16) / (64 * 16);  // 16 B units per lane
    const int lane = threadIdx.x & 63;
    const int nwaves = (int)gridDim.x * (kRunThreads / 64);
    for (int ci = (int)blockIdx.x * (kRunThreads / 64) + (int)(threadIdx.x >> 6); ci < nchunks; ci += nwaves) {
        const PbRunDecodeChunk c = chunks[ci];
        const uint32_t len = c.len < kPbRunDecodeChunkBytes ? c.len : kPbRunDecodeChunkBytes;
        const uint8_t* p = c.run + c.offset;
        const int a = (int)((uintptr_t)p & 15);
        const u32x4* src = reinterpret_cast<const u32x4*>(p - a);
        const uint32_t n16 = ((uint32_t)a + len + 15) >> 4;
        u32x4 v[kUnits];
#pragma unroll
        for (int k = 0; k < kUnits; ++k) {
            const uint32_t i = (uint32_t)lane + 64u * k;
            if (i < n16) v[k] = src[i];
        }
        uint32_t n = 0;
#pragma unroll
        for (int k = 0; k < kUnits; ++k) {
            const uint32_t i = (uint32_t)lane + 64u * k;
            if (i < n16) {
                const uint32_t bits =
                    ends_of(v[k].x) | (ends_of(v[k].y) << 4) | (ends_of(v[k].z) << 8) | (ends_of(v[k].w) << 12);
                const int lo = max(a - (int)(i * 16), 0), hi = min(a + (int)len - (int)(i * 16), 16);
                if (hi > lo) n += __popc(bits & (((1u << hi) - 1) & ~((1u << lo) - 1)));
            }
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) n += __shfl_xor(n, off, 64);
        if (lane == 0) {
            counts[ci] = n;  // the host's copy (pinned)
            prefix[ci] = n;  // scanned in HBM by pb_run_prefix_kernel
        }
    }
}

// One workgroup turns the per-chunk counts into their exclusive prefix sum
// over the whole table (mod 2^32), so every chunk of every run finds its
// first element index as prefix[chunk] - prefix[run's first chunk] with two
// loads: summing the earlier chunks' counts in each workgroup instead grows
// with the square of a run's length (16 K chunks for a 64 MiB run).
constexpr int kPrefixThreads = 1024, kPrefixPer = 4;
__global__ void __launch_bounds__(kPrefixThreads) pb_run_prefix_kernel(uint32_t* __restrict__ prefix, int n) {
    __shared__ uint32_t wave_tot[kPrefixThreads / 64];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint32_t carry = 0;
    for (int base = 0; base < n; base += kPrefixThreads * kPrefixPer) {
        const int i0 = base + t * kPrefixPer;
        uint32_t v[kPrefixPer], mine = 0;
#pragma unroll
        for (int j = 0; j < kPrefixPer; ++j) {
            v[j] = i0 + j < n ? prefix[i0 + j] : 0;
            mine += v[j];
        }
        uint32_t incl = mine;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wave_tot[wave] = incl;
        __syncthreads();
        uint32_t run = carry + incl - mine, tile = 0;
        for (int w = 0; w < kPrefixThreads / 64; ++w) {
            const uint32_t x = wave_tot[w];
            if (w < wave) run += x;
            tile += x;
        }
#pragma unroll
        for (int j = 0; j < kPrefixPer; ++j) {
            if (i0 + j < n) prefix[i0 + j] = run;
            run += v[j];
        }
        carry += tile;
        __syncthreads();  // wave_tot is rewritten by the next tile
    }
}

__device__ __forceinline__ void store_elem(uint8_t* o, uint32_t kind, uint64_t raw) {
    switch (kind) {
    case PB_RUN_INT32:
    case PB_RUN_UINT32: *reinterpret_cast<uint32_t*>(o) = (uint32_t)raw; break;
    case PB_RUN_SINT32: {
        const uint32_t u = (uint32_t)raw;
        *reinterpret_cast<int32_t*>(o) = (int32_t)(u >> 1) ^ -(int32_t)(u & 1);
        break;
    }
    case PB_RUN_SINT64: *reinterpret_cast<int64_t*>(o) = (int64_t)(raw >> 1) ^ -(int64_t)(raw & 1); break;
    case PB_RUN_BOOL: *o = raw ? 1 : 0; break;
    default: *reinterpret_cast<uint64_t*>(o) = raw; break;
    }
}

// dst gets image[sh, sh + total) where dst = sh (mod 16): the aligned body
// moves as 16-byte LDS reads and 16-byte stores.
__device__ __forceinline__ void copy_out_aligned(uint8_t* dst, const uint8_t* image, uint32_t sh, uint32_t total) {
    const uint32_t t = threadIdx.x;
    uint32_t head = (16 - sh) & 15;
    if (head > total) head = total;
    if (t < head) dst[t] = image[sh + t];
    const uint32_t nv = (total - head) / 16;
    const u32x4* from = reinterpret_cast<const u32x4*>(image + sh + head);
    u32x4* body = reinterpret_cast<u32x4*>(dst + head);
    for (uint32_t w = t; w < nv; w += kRunThreads) body[w] = from[w];
    for (uint32_t j = head + 16 * nv + t; j < total; j += kRunThreads) dst[j] = image[sh + j];
}

__global__ void __launch_bounds__(kRunThreads) pb_run_decode_kernel(const PbRunDecodeChunk* __restrict__ chunks,
                                                                    int nchunks,
                                                                    const uint32_t* __restrict__ prefix,
                                                                    int32_t* __restrict__ err) {
    __shared__ u32x4 raw[kStage16];
    __shared__ __attribute__((aligned(16))) uint8_t image[kPbRunDecodeChunkBytes * 8 + 16];
    __shared__ uint32_t wave_tot[kRunThreads / 64];
    __shared__ int bad;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    PbRunDecodeChunk c = chunks[blockIdx.x];
    // grid-stride over the chunks; the next descriptor (pinned host memory)
    // is fetched while this chunk decodes
    for (int ci = blockIdx.x; ci < nchunks; ci += gridDim.x) {
        PbRunDecodeChunk next = c;
        if (ci + (int)gridDim.x < nchunks) next = chunks[ci + gridDim.x];
        const uint32_t len = c.len < kPbRunDecodeChunkBytes ? c.len : kPbRunDecodeChunkBytes;
        const uint32_t halo = c.offset < (uint32_t)kHalo ? c.offset : (uint32_t)kHalo;
        if (t == 0) bad = 0;
        // chunk byte x (x in [-halo, len)) is at LDS byte x + o
        const uint32_t o = kPad + stage_aligned(c.run + c.offset - halo, halo + len, raw + kPad / 16) + halo;
        // first element index: the earlier chunks of the run
        const uint32_t base = prefix[ci] - prefix[c.first];
        const uint32_t eb = c.kind == PB_RUN_BOOL ? 1 : (c.kind <= PB_RUN_SINT32 ? 4 : 8);
        uint8_t* dst = static_cast<uint8_t*>(c.dst) + (size_t)base * eb;
        // the image sits at dst's alignment so copy-out is 16-byte both sides;
        // element stores stay naturally aligned only when dst is
        const uint32_t sh0 = (uint32_t)((uintptr_t)dst & 15);
        const uint32_t sh = sh0 % eb == 0 ? sh0 : 0;
        __syncthreads();  // the staging is complete
        // lane t decodes the varints ending in chunk bytes [j0, j0 + 16), from a
        // register window of bytes [j0 - 16, j0 + 16): 9 aligned LDS words
        // funnel-shifted into 8, then fixed-position bit work only (no
        // byte-serial LDS walks)
        const uint32_t j0 = (uint32_t)t * 16;
        const uint32_t wb = o + j0 - 16;  // >= 0: o >= kPad
        const uint32_t* words = reinterpret_cast<const uint32_t*>(raw) + (wb >> 2);
        const uint32_t fs = (wb & 3) * 8;
        uint32_t W[8];
        {
            uint32_t w9[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) w9[k] = words[k];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                W[k] = fs ? (uint32_t)((((uint64_t)w9[k + 1] << 32) | w9[k]) >> fs) : w9[k];
            }
        }
        uint32_t cont = 0;  // bit i: window byte i carries a continuation bit
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t m = W[k] & 0x80808080u;
            cont |= (((m >> 7) & 1) | ((m >> 14) & 2) | ((m >> 21) & 4) | ((m >> 28) & 8)) << (4 * k);
        }
        // bytes before the run's staged part end the lookback (the first lane of
        // a run's first chunk)
        const int first_valid = 16 - (int)j0 - (int)halo;  // window index of chunk byte -halo
        if (first_valid > 0) cont &= ~((1u << first_valid) - 1);
        const int mine_n = (int)len - (int)j0;
        const uint32_t own = mine_n >= 16 ? 0xFFFFu : (mine_n <= 0 ? 0u : ((1u << mine_n) - 1));
        const uint32_t term = (~cont >> 16) & own;
        const uint32_t mine = __popc(term);
        uint32_t incl = mine;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        if (lane == 63) wave_tot[wave] = incl;
        __syncthreads();
        uint32_t rank = incl - mine;
        for (int w = 0; w < wave; ++w) rank += wave_tot[w];
        const uint32_t total = wave_tot[0] + wave_tot[1] + wave_tot[2] + wave_tot[3];
#define WBYTE(i) ((W[(i) >> 2] >> (8 * ((i) & 3))) & 0xFFu)
#pragma unroll
        for (int p = 16; p < 32; ++p) {
            if (!((term >> (p - 16)) & 1)) continue;
            const uint32_t below = ~cont & ((1u << p) - 1);
            const int n = p - (below ? 31 - __clz(below) : -1);  // varint bytes
            if (n > 10 || (n == 10 && WBYTE(p) > 1)) bad = 1;
            uint64_t v = 0;
#pragma unroll
            for (int k = 0; k < 10; ++k) {
                if (k < n) v = (v << 7) | (WBYTE(p - k) & 0x7F);
            }
            store_elem(image + sh + (size_t)rank * eb, c.kind, v);
            ++rank;
        }
#undef WBYTE
        __syncthreads();
        if (bad) {
            if (t == 0) err[ci] = 1;
        } else {
            const uint32_t nbytes = total * eb;
            if (sh == sh0) {
                copy_out_aligned(dst, image, sh, nbytes);
            } else {
                copy_out(dst, image, nbytes);
            }
            if (t == 0) err[ci] = 0;
        }
        __syncthreads();  // raw, image, wave_tot and bad are reused
        c = next;
    }
}

}  // namespace

int LaunchPbRunDecode(const PbRunDecodeChunk* chunks, int n, uint32_t* counts, uint32_t* prefix, int32_t* err,
                      hipStream_t s) {
    if (n <= 0) return 0;
    if (!prefix) return -1;
    // a wave per chunk, 8 workgroups (32 waves) per CU at most; the waves
    // stride over the rest
    const int count_wgs = (n + kRunThreads / 64 - 1) / (kRunThreads / 64);
    const int count_grid = count_wgs < 2048 ? count_wgs : 2048;
    const int decode_grid = n < 1024 ? n : 1024;  // 4 resident per CU (37 KiB of LDS each)
    hipLaunchKernelGGL(pb_run_count_kernel, dim3((unsigned)count_grid), dim3(kRunThreads), 0, s, chunks, n, counts,
                       prefix);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(pb_run_prefix_kernel, dim3(1), dim3(kPrefixThreads), 0, s, prefix, n);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(pb_run_decode_kernel, dim3((unsigned)decode_grid), dim3(kRunThreads), 0, s, chunks, n, prefix,
                       err);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int LaunchPbRunEncode(const PbRunChunk* chunks, int n, int32_t* err, hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(pb_run_encode_kernel, dim3((unsigned)n), dim3(kRunThreads), 0, s, chunks, err);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int LaunchPbScan(const uint8_t* buf, uint64_t buf_len, const int64_t* offsets_dev, int64_t n, uint32_t max_fields,
                 uint64_t* fields, int32_t* nfields, hipStream_t s) {
    if (n <= 0) return 0;
    if (max_fields == 0) return -1;
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(pb_scan_kernel, dim3((unsigned)blocks), dim3(256), 0, s, buf, buf_len, offsets_dev, n,
                       max_fields, fields, nfields);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int LaunchPbScanPtrs(const PbScanJob* jobs, int64_t n, uint32_t max_fields, uint64_t* fields, int32_t* nfields,
                     hipStream_t s) {
    if (n <= 0) return 0;
    if (max_fields == 0) return -1;
    const int64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(pb_scan_ptrs_kernel, dim3((unsigned)blocks), dim3(256), 0, s, jobs, n, max_fields, fields,
                       nfields);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace gpu
}  // namespace mrpc
