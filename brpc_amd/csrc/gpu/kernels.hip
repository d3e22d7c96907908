// Hand-written CDNA4 (gfx950) kernels for the RPC data path.
//
//  * crc32c_kernel — batched CRC32C of HBM buffers. Each 256-lane
//    workgroup owns a 16 KiB chunk; each lane folds 64 contiguous bytes
//    (4 x 16 B global loads) with slicing-by-8 tables staged in LDS. Chunk
//    and lane blocks are aligned to the END of the segment so every
//    partial CRC is shifted by a fixed, table-resident power of x
//    (leading zero bytes do not change a zero-initialised CRC register),
//    wave XOR-reduction via DPP shuffles, and one atomicXor per
//    workgroup folds chunks in any completion order — CRC over GF(2) is
//    linear, so the combine is order-free.
//  * batched_copy_kernel — one launch for many (src,dst,len) segments
//    (Buf blocks -> contiguous HBM), 16 B vector path.
//  * varint count/scan/decode/encode — packed protobuf varints decoded and
//    encoded on device: per-tile terminator counts, a single-workgroup
//    scan, then a decode pass that places each value by a block prefix sum.
//
// The reference has no device code; these are the MI355X-native
// equivalents of butil/crc32c.cc (src/butil/crc32c.cc:25-349) and the
// protobuf wire codec used by src/brpc/policy/baidu_rpc_protocol.cpp.
#include <hip/hip_runtime.h>

#include <cstring>

#include "gpu/kernels.h"

namespace mrpc {
namespace gpu {

namespace {

constexpr uint32_t kPoly = 0x82F63B78u;  // reflected Castagnoli
constexpr int kThreads = 256;
constexpr int kLaneBytes = 64;

struct CrcTables {
    uint32_t t8[8][256];       // slicing-by-8 tables
    uint32_t lane_shift[256];  // x^(8*64*j) mod P
    uint32_t x2n[64];          // x^(2^k) mod P
};

__constant__ uint32_t c_lane_shift[256];
__constant__ uint32_t c_x2n[64];

__device__ __forceinline__ uint32_t mult_mod_p(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {  // fixed trip count: no data-dependent exit
        const uint32_t m = 1u << (31 - i);
        p ^= (a & m) ? b : 0u;
        b = (b & 1u) ? (b >> 1) ^ kPoly : (b >> 1);
    }
    return p;
}

// x^(8n) mod P
__device__ uint32_t shift_bytes_poly(uint64_t n) {
    uint32_t r = 1u << 31;
    uint64_t bits = n;
    int k = 3;  // 8 = 2^3
    while (bits && k < 64) {
        if (bits & 1) r = mult_mod_p(c_x2n[k], r);
        bits >>= 1;
        ++k;
    }
    return r;
}

struct SegBatch {
    int nseg;
    int pad;
    const void* src[kInlineSegments];
    void* dst[kInlineSegments];
    uint64_t len[kInlineSegments];
    uint32_t chunk_start[kInlineSegments + 1];  // exclusive prefix of chunk counts
};

__device__ __forceinline__ int find_segment(const SegBatch& b, uint32_t chunk) {
    int lo = 0, hi = b.nseg - 1;
    while (lo < hi) {  // last seg with chunk_start <= chunk
        const int mid = (lo + hi + 1) >> 1;
        if (b.chunk_start[mid] <= chunk) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ uint32_t crc_word8(uint32_t crc, uint32_t lo, uint32_t hi, const uint32_t (*t)[256]) {
    lo ^= crc;
    return t[7][lo & 0xff] ^ t[6][(lo >> 8) & 0xff] ^ t[5][(lo >> 16) & 0xff] ^ t[4][lo >> 24] ^
           t[3][hi & 0xff] ^ t[2][(hi >> 8) & 0xff] ^ t[1][(hi >> 16) & 0xff] ^ t[0][hi >> 24];
}

__global__ void __launch_bounds__(kThreads) crc32c_kernel(SegBatch b, const uint32_t* __restrict__ tables,
                                                          uint32_t* __restrict__ out) {
    __shared__ uint32_t t[8][256];
    __shared__ uint32_t wave_acc[kThreads / 64];
    // stage the 8 KiB of tables into LDS: 2048 dwords, 8 per lane, 16 B loads
    {
        const uint4* src = reinterpret_cast<const uint4*>(tables);
        uint4* dst = reinterpret_cast<uint4*>(&t[0][0]);
        dst[threadIdx.x] = src[threadIdx.x];
        dst[threadIdx.x + kThreads] = src[threadIdx.x + kThreads];
    }
    const uint32_t chunk = blockIdx.x;
    const int seg = find_segment(b, chunk);
    const uint64_t len = b.len[seg];
    const uint8_t* base = static_cast<const uint8_t*>(b.src[seg]);
    const uint32_t seg_chunks = b.chunk_start[seg + 1] - b.chunk_start[seg];
    const uint32_t k = chunk - b.chunk_start[seg];          // chunk index from the front
    const uint32_t after = seg_chunks - 1 - k;                 // chunks after this one
    // chunk covers [end - (after+1)*C, end - after*C) clipped at 0
    const int64_t chunk_end = (int64_t)len - (int64_t)after * (int64_t)kChunkBytes;
    // lane j covers [chunk_end - (256-j)*64, chunk_end - (255-j)*64)
    const int64_t lane_end = chunk_end - (int64_t)(kThreads - 1 - threadIdx.x) * kLaneBytes;
    const int64_t lane_beg = lane_end - kLaneBytes;
    __syncthreads();

    uint32_t crc = 0;
    if (lane_end > 0) {
        if (lane_beg >= 0 && ((reinterpret_cast<uintptr_t>(base) + (uint64_t)lane_beg) & 15) == 0) {
            const uint4* p = reinterpret_cast<const uint4*>(base + lane_beg);
            uint4 v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = p[i];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                crc = crc_word8(crc, v[i].x, v[i].y, t);
                crc = crc_word8(crc, v[i].z, v[i].w, t);
            }
        } else {
            const int64_t s = lane_beg < 0 ? 0 : lane_beg;
            for (int64_t i = s; i < lane_end; ++i) crc = t[0][(crc ^ base[i]) & 0xff] ^ (crc >> 8);
        }
        // shift by the bytes that follow this lane inside the chunk
        crc = mult_mod_p(c_lane_shift[kThreads - 1 - threadIdx.x], crc);
    }
    // XOR-reduce the wave (64 lanes)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) crc ^= __shfl_xor(crc, off, 64);
    if ((threadIdx.x & 63) == 0) wave_acc[threadIdx.x >> 6] = crc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = wave_acc[0] ^ wave_acc[1] ^ wave_acc[2] ^ wave_acc[3];
        if (after) acc = mult_mod_p(shift_bytes_poly((uint64_t)after * kChunkBytes), acc);
        if (after == seg_chunks - 1) {
            // first chunk also folds the ~0 init and final inversion:
            // std = raw0(M) ^ shift(~0, len) ^ ~0
            acc ^= mult_mod_p(shift_bytes_poly(len), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
        }
        atomicXor(out + seg, acc);
    }
}

__global__ void __launch_bounds__(kThreads) batched_copy_kernel(SegBatch b) {
    const uint32_t chunk = blockIdx.x;
    const int seg = find_segment(b, chunk);
    const uint64_t len = b.len[seg];
    const uint64_t k = chunk - b.chunk_start[seg];
    const uint8_t* src = static_cast<const uint8_t*>(b.src[seg]);
    uint8_t* dst = static_cast<uint8_t*>(b.dst[seg]);
    const uint64_t cbeg = k * kChunkBytes;
    const uint64_t cend = cbeg + kChunkBytes < len ? cbeg + kChunkBytes : len;
    const bool aligned = (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0);
    if (aligned) {
        // coalesced: lane i moves 16 B at i*16 within each 4 KiB stripe
        for (uint64_t off = cbeg + threadIdx.x * 16; off < cend; off += kThreads * 16) {
            if (off + 16 <= cend) {
                uint4 v = *reinterpret_cast<const uint4*>(src + off);
                *reinterpret_cast<uint4*>(dst + off) = v;
            } else {
                for (uint64_t i = off; i < cend; ++i) dst[i] = src[i];
            }
        }
    } else {
        for (uint64_t off = cbeg + threadIdx.x; off < cend; off += kThreads) dst[off] = src[off];
    }
}

// ---------------------------------------------------------------- varint
constexpr int kVTile = kThreads * 16;  // 4 KiB of bytes (or 4096 values) per tile

__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* total, uint32_t* smem) {
    // wave inclusive scan
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) smem[wave] = x;
    __syncthreads();
    uint32_t wave_prefix = 0, sum = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) {
        const uint32_t s = smem[w];
        if (w < wave) wave_prefix += s;
        sum += s;
    }
    __syncthreads();
    *total = sum;
    return wave_prefix + x - v;
}

__global__ void __launch_bounds__(kThreads) varint_count_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                                uint64_t* __restrict__ tile_counts) {
    __shared__ uint32_t smem[kThreads / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kVTile + threadIdx.x * 16;
    uint32_t c = 0;
    if (base + 16 <= n && (reinterpret_cast<uintptr_t>(in + base) & 15) == 0) {
        const uint4 v = *reinterpret_cast<const uint4*>(in + base);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) c += __popc(~w[i] & 0x80808080u);  // bytes with MSB clear
    } else {
        for (uint64_t i = base; i < base + 16 && i < n; ++i) c += (in[i] & 0x80) ? 0 : 1;
    }
    uint32_t total;
    block_exclusive_scan(c, &total, smem);
    if (threadIdx.x == 0) tile_counts[blockIdx.x] = total;
}

// Exclusive scan of `counts` in place (single workgroup, any length);
// writes the grand total to *total.
__global__ void __launch_bounds__(1024) scan_tiles_kernel(uint64_t* counts, uint64_t ntiles, uint64_t* total) {
    __shared__ uint64_t part[1024];
    const uint64_t per = (ntiles + 1023) / 1024;
    const uint64_t b = threadIdx.x * per;
    const uint64_t e = b + per < ntiles ? b + per : ntiles;
    uint64_t s = 0;
    for (uint64_t i = b; i < e; ++i) s += counts[i];
    part[threadIdx.x] = s;
    __syncthreads();
    // Hillis-Steele over 1024 partial sums
    for (int off = 1; off < 1024; off <<= 1) {
        const uint64_t y = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += y;
        __syncthreads();
    }
    uint64_t run = threadIdx.x ? part[threadIdx.x - 1] : 0;
    for (uint64_t i = b; i < e; ++i) {
        const uint64_t c = counts[i];
        counts[i] = run;
        run += c;
    }
    if (threadIdx.x == 1023) *total = part[1023];
}

__global__ void __launch_bounds__(kThreads) varint_decode_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                                 const uint64_t* __restrict__ tile_offsets,
                                                                 uint64_t* __restrict__ out, uint64_t max_out,
                                                                 int zigzag, int* __restrict__ err) {
    __shared__ uint32_t smem[kThreads / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kVTile + threadIdx.x * 16;
    union {
        uint4 v;
        uint8_t b[16];
    } u;
    uint8_t* bytes = u.b;
    int nb = 0;
    if (base < n) {
        nb = (int)(n - base < 16 ? n - base : 16);
        if (nb == 16 && (reinterpret_cast<uintptr_t>(in + base) & 15) == 0) {
            u.v = *reinterpret_cast<const uint4*>(in + base);
        } else {
            for (int i = 0; i < nb; ++i) bytes[i] = in[base + i];
        }
    }
    uint32_t c = 0;
    for (int i = 0; i < nb; ++i) c += (bytes[i] & 0x80) ? 0 : 1;
    uint32_t total;
    uint64_t idx = tile_offsets[blockIdx.x] + block_exclusive_scan(c, &total, smem);
    for (int i = 0; i < nb; ++i) {
        if (bytes[i] & 0x80) continue;
        // terminator at base+i: walk back over continuation bytes
        const uint64_t p = base + i;
        uint64_t start = p;
        int len = 1;
        while (start > 0 && len <= 10 && (in[start - 1] & 0x80)) {
            --start;
            ++len;
        }
        if (len > 10) {
            atomicOr(err, 1);
            ++idx;
            continue;
        }
        uint64_t v = 0;
        for (int j = 0; j < len; ++j) v |= (uint64_t)(in[start + j] & 0x7f) << (7 * j);
        if (zigzag) v = (v >> 1) ^ (~(v & 1) + 1);
        if (idx < max_out) out[idx] = v;
        else atomicOr(err, 2);
        ++idx;
    }
    // a trailing continuation byte means truncated input
    if (base + nb == n && nb > 0 && (bytes[nb - 1] & 0x80)) atomicOr(err, 1);
}

__device__ __forceinline__ uint32_t varint_len(uint64_t v) {
    // 1 + floor(bit_width(v)-1)/7, with v=0 -> 1
    const int bits = v ? 64 - __clzll(v) : 1;
    return (uint32_t)((bits + 6) / 7);
}

__global__ void __launch_bounds__(kThreads) varint_len_kernel(const uint64_t* __restrict__ in, uint64_t n,
                                                              int zigzag, uint64_t* __restrict__ tile_counts) {
    __shared__ uint32_t smem[kThreads / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kVTile + threadIdx.x * 16;
    uint32_t c = 0;
    for (uint64_t i = base; i < base + 16 && i < n; ++i) {
        uint64_t v = in[i];
        if (zigzag) v = (v << 1) ^ (uint64_t)((int64_t)v >> 63);
        c += varint_len(v);
    }
    uint32_t total;
    block_exclusive_scan(c, &total, smem);
    if (threadIdx.x == 0) tile_counts[blockIdx.x] = total;
}

__global__ void __launch_bounds__(kThreads) varint_encode_kernel(const uint64_t* __restrict__ in, uint64_t n,
                                                                 int zigzag,
                                                                 const uint64_t* __restrict__ tile_offsets,
                                                                 uint8_t* __restrict__ out) {
    __shared__ uint32_t smem[kThreads / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kVTile + threadIdx.x * 16;
    uint64_t vals[16];
    uint32_t c = 0;
    int nv = 0;
    for (uint64_t i = base; i < base + 16 && i < n; ++i) {
        uint64_t v = in[i];
        if (zigzag) v = (v << 1) ^ (uint64_t)((int64_t)v >> 63);
        vals[nv++] = v;
        c += varint_len(v);
    }
    uint32_t total;
    uint64_t pos = tile_offsets[blockIdx.x] + block_exclusive_scan(c, &total, smem);
    for (int k = 0; k < nv; ++k) {
        uint64_t v = vals[k];
        while (v >= 0x80) {
            out[pos++] = (uint8_t)(v | 0x80);
            v >>= 7;
        }
        out[pos++] = (uint8_t)v;
    }
}

// ---------------------------------------------------------------- host side
uint32_t host_mult_mod_p(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int i = 0; i < 32; ++i) {
        if (a & (1u << (31 - i))) p ^= b;
        b = (b & 1u) ? (b >> 1) ^ kPoly : (b >> 1);
    }
    return p;
}

struct DeviceTables {
    uint32_t* t8 = nullptr;  // device copy of the slicing tables
    bool ready = false;
};

DeviceTables g_tables[64];

int ensure_tables() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
    DeviceTables& dt = g_tables[dev];
    if (dt.ready) return 0;
    static CrcTables h;
    static bool built = false;
    if (!built) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
            h.t8[0][i] = c;
        }
        for (int s = 1; s < 8; ++s) {
            for (int i = 0; i < 256; ++i) h.t8[s][i] = (h.t8[s - 1][i] >> 8) ^ h.t8[0][h.t8[s - 1][i] & 0xff];
        }
        // x2n[k] = x^(2^k) mod P; x^1 reflected = 1<<30
        uint32_t p = 1u << 30;
        for (int k = 0; k < 64; ++k) {
            h.x2n[k] = p;
            p = host_mult_mod_p(p, p);
        }
        // lane_shift[j] = x^(8*64*j)
        uint32_t step = 1u << 31;
        {
            // x^(512) = product of x2n bits of 512 = 2^9
            step = h.x2n[9];
        }
        uint32_t acc = 1u << 31;
        for (int j = 0; j < 256; ++j) {
            h.lane_shift[j] = acc;
            acc = host_mult_mod_p(step, acc);
        }
        built = true;
    }
    if (hipMalloc(&dt.t8, sizeof(h.t8)) != hipSuccess) return -1;
    if (hipMemcpy(dt.t8, h.t8, sizeof(h.t8), hipMemcpyHostToDevice) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_lane_shift), h.lane_shift, sizeof(h.lane_shift)) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_x2n), h.x2n, sizeof(h.x2n)) != hipSuccess) return -1;
    dt.ready = true;
    return 0;
}

// Fill a SegBatch with up to kInlineSegments segments; returns chunk count.
uint32_t fill_batch(SegBatch* b, const Segment* segs, int n) {
    memset(b, 0, sizeof(*b));
    b->nseg = n;
    uint32_t c = 0;
    for (int i = 0; i < n; ++i) {
        b->src[i] = segs[i].src;
        b->dst[i] = segs[i].dst;
        b->len[i] = segs[i].len;
        b->chunk_start[i] = c;
        uint64_t nc = (segs[i].len + kChunkBytes - 1) / kChunkBytes;
        if (nc == 0) nc = 1;  // empty segment still gets a workgroup (writes crc 0)
        c += (uint32_t)nc;
    }
    b->chunk_start[n] = c;
    return c;
}

}  // namespace

int LaunchCrc32c(const Segment* segs, int nseg, uint32_t* out_dev, hipStream_t s) {
    if (nseg <= 0) return 0;
    if (ensure_tables() != 0) return -1;
    int dev = 0;
    hipGetDevice(&dev);
    if (hipMemsetAsync(out_dev, 0, sizeof(uint32_t) * nseg, s) != hipSuccess) return -1;
    for (int i = 0; i < nseg; i += kInlineSegments) {
        const int n = nseg - i < kInlineSegments ? nseg - i : kInlineSegments;
        SegBatch b;
        const uint32_t chunks = fill_batch(&b, segs + i, n);
        hipLaunchKernelGGL(crc32c_kernel, dim3(chunks), dim3(kThreads), 0, s, b, g_tables[dev].t8, out_dev + i);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    return 0;
}

int LaunchBatchedCopy(const Segment* segs, int nseg, hipStream_t s) {
    for (int i = 0; i < nseg; i += kInlineSegments) {
        const int n = nseg - i < kInlineSegments ? nseg - i : kInlineSegments;
        SegBatch b;
        const uint32_t chunks = fill_batch(&b, segs + i, n);
        hipLaunchKernelGGL(batched_copy_kernel, dim3(chunks), dim3(kThreads), 0, s, b);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    return 0;
}

size_t VarintScratchBytes(uint64_t n) {
    const uint64_t tiles = (n + kVTile - 1) / kVTile;
    return (tiles + 1) * sizeof(uint64_t);
}

int LaunchVarintDecode(const uint8_t* in, uint64_t n, uint64_t* out, uint64_t max_out, bool zigzag,
                       uint64_t* count_dev, int* err_dev, void* scratch, hipStream_t s) {
    if (hipMemsetAsync(err_dev, 0, sizeof(int), s) != hipSuccess) return -1;
    if (n == 0) return hipMemsetAsync(count_dev, 0, sizeof(uint64_t), s) == hipSuccess ? 0 : -1;
    const uint64_t tiles = (n + kVTile - 1) / kVTile;
    uint64_t* tile = static_cast<uint64_t*>(scratch);
    hipLaunchKernelGGL(varint_count_kernel, dim3((uint32_t)tiles), dim3(kThreads), 0, s, in, n, tile);
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(1), dim3(1024), 0, s, tile, tiles, count_dev);
    hipLaunchKernelGGL(varint_decode_kernel, dim3((uint32_t)tiles), dim3(kThreads), 0, s, in, n,
                       (const uint64_t*)tile, out, max_out, zigzag ? 1 : 0, err_dev);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int LaunchVarintEncode(const uint64_t* in, uint64_t n, bool zigzag, uint8_t* out, uint64_t* bytes_dev,
                       void* scratch, hipStream_t s) {
    if (n == 0) return hipMemsetAsync(bytes_dev, 0, sizeof(uint64_t), s) == hipSuccess ? 0 : -1;
    const uint64_t tiles = (n + kVTile - 1) / kVTile;
    uint64_t* tile = static_cast<uint64_t*>(scratch);
    hipLaunchKernelGGL(varint_len_kernel, dim3((uint32_t)tiles), dim3(kThreads), 0, s, in, n, zigzag ? 1 : 0, tile);
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(1), dim3(1024), 0, s, tile, tiles, bytes_dev);
    hipLaunchKernelGGL(varint_encode_kernel, dim3((uint32_t)tiles), dim3(kThreads), 0, s, in, n, zigzag ? 1 : 0,
                       (const uint64_t*)tile, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace gpu
}  // namespace mrpc
