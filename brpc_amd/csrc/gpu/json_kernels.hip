// JSON structural index on gfx950 (K6 of SURVEY §3, the device half of
// json2pb for large http+json bodies): the positions of every structural
// character ({ } [ ] : ,) outside strings and of every unescaped quote, plus
// validation that all strings are terminated — the stage-1 index a parser
// walks instead of scanning bytes (the reference's json2pb tokenizes on the
// CPU, src/json2pb/json_to_pb.cpp via rapidjson).
//
// Each lane owns 64 input bytes and turns them into 64-bit masks (quote,
// backslash, structural) with SWAR byte compares; the bytes are read once,
// everything after works on masks. The two sequential dependencies of
// tokenizing are carried with scans instead of a serial walk:
//  * escapes: whether byte i is escaped depends on the parity of the
//    backslash run before it, which may start in an earlier lane or tile.
//    A lane maps its carry-in (byte 0 escaped?) to a carry-out; the map is
//    composable, so lanes and tiles scan it.
//  * strings: inside/outside flips at every unescaped quote, so the state
//    at a byte is the XOR of the quote parities before it (prefix XOR in a
//    lane), and a lane's parity depends on its escape carry-in.
// A lane therefore has 4 possible start states (carry, in-string), and so
// does a tile (256 lanes x 64 B = 16 KiB). Three launches:
//  1. per tile: masks, the tile's transfer table T(c) = (carry-out, quote
//     parity), each lane's prefix table and its exclusive position offset
//     for each of the 4 tile start states (4 x u16 packed in one u64 and
//     scanned with plain 64-bit adds) and the tile's 4 counts;
//  2. one block: scan the tile tables to each tile's actual start state,
//     pick its count, scan the counts to output offsets;
//  3. per tile: each lane resolves its position mask with no further scan
//     and writes positions through an LDS window, so global stores are
//     contiguous 1 KiB rows instead of 64 scattered lanes.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gpu/kernels.h"

namespace mrpc {
namespace gpu {

namespace {

constexpr int kJThreads = 256;
constexpr int kJWaves = kJThreads / 64;
constexpr uint64_t kLaneBytes = 64;
constexpr uint64_t kJTile = kJThreads * kLaneBytes;  // 16 KiB
constexpr uint32_t kEmitWindow = 4096;               // positions staged in LDS per round (16 KiB)

// Transfer table for escape carry-in c in {0,1}, packed in 4 bits:
// bit c = carry-out for carry-in c, bit 2+c = quote parity for carry-in c.
__device__ __forceinline__ uint32_t xf_next(uint32_t x, int c) { return (x >> c) & 1; }
__device__ __forceinline__ uint32_t xf_flip(uint32_t x, int c) { return (x >> (2 + c)) & 1; }
__device__ __forceinline__ uint32_t xf_make(uint32_t n0, uint32_t n1, uint32_t f0, uint32_t f1) {
    return n0 | (n1 << 1) | (f0 << 2) | (f1 << 3);
}
constexpr uint32_t kXfIdentity = 0x2;  // next = c, no flips

// a then b
__device__ __forceinline__ uint32_t xf_compose(uint32_t a, uint32_t b) {
    const uint32_t m0 = xf_next(a, 0), m1 = xf_next(a, 1);
    return xf_make(xf_next(b, m0), xf_next(b, m1), xf_flip(a, 0) ^ xf_flip(b, m0), xf_flip(a, 1) ^ xf_flip(b, m1));
}

// Start state k = carry | in_string << 1 after applying prefix table x to
// start state k0.
__device__ __forceinline__ int xf_apply(uint32_t x, int k0) {
    const int c = k0 & 1;
    return (int)xf_next(x, c) | ((((k0 >> 1) & 1) ^ (int)xf_flip(x, c)) << 1);
}

// High bit of each byte of w set iff that byte equals the byte broadcast in
// pat (exact, no cross-byte carries).
__device__ __forceinline__ uint32_t bytes_eq(uint32_t w, uint32_t pat) {
    const uint32_t t = w ^ pat;
    return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
}
// Gather the 4 byte-high-bits into bits 0..3.
__device__ __forceinline__ uint32_t gather4(uint32_t m) { return ((m >> 7) & 0x01010101u) * 0x01020408u >> 24; }

struct LaneMasks {
    uint64_t quote, backslash, structural;
};

__device__ __forceinline__ void word_masks(uint32_t w, int shift, LaneMasks& m) {
    const uint32_t lw = w | 0x20202020u;  // '[' -> '{', ']' -> '}'
    const uint32_t q = bytes_eq(w, 0x22222222u);
    const uint32_t b = bytes_eq(w, 0x5C5C5C5Cu);
    const uint32_t s = bytes_eq(lw, 0x7B7B7B7Bu) | bytes_eq(lw, 0x7D7D7D7Du) | bytes_eq(w, 0x3A3A3A3Au) |
                       bytes_eq(w, 0x2C2C2C2Cu);
    m.quote |= (uint64_t)gather4(q) << shift;
    m.backslash |= (uint64_t)gather4(b) << shift;
    m.structural |= (uint64_t)gather4(s) << shift;
}

// Masks of the lane's 64 bytes (zero past the end: neither quote nor
// backslash nor structural).
__device__ __forceinline__ LaneMasks lane_masks(const uint8_t* __restrict__ in, uint64_t n, uint64_t base) {
    LaneMasks m{0, 0, 0};
    if (base + kLaneBytes <= n && ((reinterpret_cast<uintptr_t>(in) + base) & 15) == 0) {
        const uint4* p = reinterpret_cast<const uint4*>(in + base);
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = p[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            word_masks(v[k].x, 16 * k + 0, m);
            word_masks(v[k].y, 16 * k + 4, m);
            word_masks(v[k].z, 16 * k + 8, m);
            word_masks(v[k].w, 16 * k + 12, m);
        }
    } else if (base < n) {
        for (int j = 0; j < (int)kLaneBytes; j += 4) {
            uint32_t w = 0;
            for (int t = 0; t < 4; ++t)
                if (base + j + t < n) w |= (uint32_t)in[base + j + t] << (8 * t);
            word_masks(w, j, m);
        }
    }
    return m;
}

// Escaped-byte mask of a lane for carry-in c (byte 0 escaped), walking the
// backslash runs (JSON has few); *carry_out = whether the next lane's byte 0
// is escaped.
__device__ __forceinline__ uint64_t escaped_mask(uint64_t bs, int c, int* carry_out) {
    uint64_t esc = 0;
    int co = 0;
    if (c) {
        esc = 1;
        bs &= ~1ull;  // an escaped backslash escapes nothing
    }
    while (bs) {
        const int s = __builtin_ctzll(bs);
        const uint64_t rest = ~(bs >> s);
        const int len = rest ? __builtin_ctzll(rest) : 64 - s;
        const int e = s + len;
        if (len & 1) {
            if (e < 64) esc |= 1ull << e;
            else co = 1;
        }
        bs = e >= 64 ? 0 : bs & (~0ull << e);
    }
    *carry_out = co;
    return esc;
}

// Inclusive prefix XOR of the bits of x (bit i = XOR of bits 0..i).
__device__ __forceinline__ uint64_t prefix_xor(uint64_t x) {
    x ^= x << 1;
    x ^= x << 2;
    x ^= x << 4;
    x ^= x << 8;
    x ^= x << 16;
    x ^= x << 32;
    return x;
}

// Reported positions of a lane given its unescaped quotes q and start
// in-string flag: quotes always, structurals outside strings. The in-string
// mask (inclusive prefix XOR) runs from an opening quote to the byte before
// its closing quote.
__device__ __forceinline__ uint64_t position_mask(uint64_t q, uint64_t structural, int in_string) {
    const uint64_t inside = (prefix_xor(q) ^ (in_string ? ~0ull : 0ull)) & ~q;
    return (structural & ~inside) | q;
}

// Block-wide scans: 64-lane shuffle scans, then the 4 wave totals through
// LDS. `wtot` is a kJWaves-entry LDS array owned by the caller.
__device__ __forceinline__ uint32_t block_xf_scan(uint32_t v, uint32_t* wtot, uint32_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off, 64);
        if (lane >= off) inc = xf_compose(y, inc);
    }
    if (lane == 63) wtot[wave] = inc;
    __syncthreads();
    uint32_t before = kXfIdentity, all = kXfIdentity;
#pragma unroll
    for (int w = 0; w < kJWaves; ++w) {
        if (w < wave) before = xf_compose(before, wtot[w]);
        all = xf_compose(all, wtot[w]);
    }
    uint32_t ex = __shfl_up(inc, 1, 64);
    if (lane == 0) ex = kXfIdentity;
    *total = all;
    return xf_compose(before, ex);
}

__device__ __forceinline__ uint64_t block_sum_scan(uint64_t v, uint64_t* wtot, uint64_t* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t inc = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint64_t y = __shfl_up(inc, off, 64);
        if (lane >= off) inc += y;
    }
    if (lane == 63) wtot[wave] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kJWaves; ++w) {
        if (w < wave) before += wtot[w];
        all += wtot[w];
    }
    *total = all;
    return before + inc - v;
}

// Scratch layout (lanes = tiles * 256):
//   u64 quote0[lanes], quote1[lanes], structural[lanes]  unescaped quotes for carry-in 0/1
//   u64 lane_off[lanes]       exclusive offset in the tile, u16 per tile start state
//   u8  lane_prefix[lanes]    prefix transfer table of the lanes before it in the tile
//   u32 tile_xfer[tiles]      then, after pass 2, tile start state
//   u64 tile_cnt[tiles]       u16 x 4 counts by start state; after pass 2, output offset
struct Scratch {
    uint64_t *q0, *q1, *st, *lane_off, *tile_cnt;
    uint8_t* lane_prefix;
    uint32_t* tile_xfer;
};

__host__ __device__ inline Scratch carve(void* p, uint64_t tiles) {
    const uint64_t lanes = tiles * kJThreads;
    Scratch s;
    uint64_t* u = static_cast<uint64_t*>(p);
    s.q0 = u;
    s.q1 = u + lanes;
    s.st = u + 2 * lanes;
    s.lane_off = u + 3 * lanes;
    s.tile_cnt = u + 4 * lanes;
    s.tile_xfer = reinterpret_cast<uint32_t*>(s.tile_cnt + tiles);
    s.lane_prefix = reinterpret_cast<uint8_t*>(s.tile_xfer + tiles);
    return s;
}

// Pass 1.
__global__ void __launch_bounds__(kJThreads) json_tile_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                              Scratch sc, int* err) {
    __shared__ uint32_t xf_wtot[kJWaves];
    __shared__ uint64_t sum_wtot[kJWaves];
    const uint64_t lane = (uint64_t)blockIdx.x * kJThreads + threadIdx.x;
    const LaneMasks m = lane_masks(in, n, lane * kLaneBytes);
    int c0, c1;
    const uint64_t e0 = escaped_mask(m.backslash, 0, &c0);
    uint64_t e1;
    if (m.backslash & 1) {
        e1 = escaped_mask(m.backslash, 1, &c1);
    } else {  // byte 0 is no backslash: an escape carried in only escapes byte 0
        e1 = e0 | 1;
        c1 = c0;
    }
    const uint64_t q0 = m.quote & ~e0;
    const uint64_t q1 = m.quote & ~e1;
    if (blockIdx.x == 0 && threadIdx.x == 0) *err = 0;  // pass 2 is the first to set it
    const uint32_t mine = xf_make((uint32_t)c0, (uint32_t)c1, (uint32_t)(__popcll(q0) & 1),
                                  (uint32_t)(__popcll(q1) & 1));
    uint32_t tile_xf;
    const uint32_t before = block_xf_scan(mine, xf_wtot, &tile_xf);
    // the lane's position count for each tile start state k
    uint64_t packed = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int ls = xf_apply(before, k);
        const uint64_t pos = position_mask(ls & 1 ? q1 : q0, m.structural, ls >> 1);
        packed |= (uint64_t)__popcll(pos) << (16 * k);
    }
    uint64_t tile_cnt;
    const uint64_t off = block_sum_scan(packed, sum_wtot, &tile_cnt);  // no u16 field exceeds 16384
    sc.q0[lane] = q0;
    sc.q1[lane] = q1;
    sc.st[lane] = m.structural;
    sc.lane_off[lane] = off;
    sc.lane_prefix[lane] = (uint8_t)before;
    if (threadIdx.x == 0) {
        sc.tile_xfer[blockIdx.x] = tile_xf;
        sc.tile_cnt[blockIdx.x] = tile_cnt;
    }
}

// Pass 2 (one block): tile start states from (carry 0, outside strings),
// output offsets, total count; err |= 1 for a string open at the end. The
// tile arrays stream through LDS in coalesced chunks of kScanPer tiles per
// thread; the state and the running offset carry from chunk to chunk.
constexpr int kScanThreads = 1024;
constexpr int kScanPer = 4;
constexpr int kScanChunk = kScanThreads * kScanPer;

__global__ void __launch_bounds__(kScanThreads) json_scan_kernel(Scratch sc, uint64_t ntiles, uint64_t* total,
                                                                 int* err) {
    __shared__ uint32_t sx[kScanChunk];
    __shared__ uint64_t scnt[kScanChunk];
    __shared__ uint32_t xpart[kScanThreads];
    __shared__ uint64_t cpart[kScanThreads];
    const int t = threadIdx.x;
    int k_carry = 0;
    uint64_t off_carry = 0;
    for (uint64_t base = 0; base < ntiles; base += kScanChunk) {
        const uint64_t m = ntiles - base < (uint64_t)kScanChunk ? ntiles - base : (uint64_t)kScanChunk;
        for (int j = t; j < kScanChunk; j += kScanThreads) {
            sx[j] = (uint64_t)j < m ? sc.tile_xfer[base + j] : kXfIdentity;
            scnt[j] = (uint64_t)j < m ? sc.tile_cnt[base + j] : 0;
        }
        __syncthreads();
        uint32_t acc = kXfIdentity;
#pragma unroll
        for (int i = 0; i < kScanPer; ++i) acc = xf_compose(acc, sx[t * kScanPer + i]);
        xpart[t] = acc;
        __syncthreads();
        for (int off = 1; off < kScanThreads; off <<= 1) {
            const uint32_t y = t >= off ? xpart[t - off] : kXfIdentity;
            __syncthreads();
            xpart[t] = xf_compose(y, xpart[t]);
            __syncthreads();
        }
        int k = xf_apply(t ? xpart[t - 1] : kXfIdentity, k_carry);
        uint64_t sum = 0;
#pragma unroll
        for (int i = 0; i < kScanPer; ++i) {
            const int j = t * kScanPer + i;
            const uint32_t x = sx[j];
            const uint64_t cnt = (scnt[j] >> (16 * k)) & 0xFFFF;
            sx[j] = (uint32_t)k;  // now: the tile's start state
            scnt[j] = cnt;
            sum += cnt;
            k = xf_apply(x, k);
        }
        cpart[t] = sum;
        __syncthreads();
        for (int off = 1; off < kScanThreads; off <<= 1) {
            const uint64_t y = t >= off ? cpart[t - off] : 0;
            __syncthreads();
            cpart[t] += y;
            __syncthreads();
        }
        uint64_t run = off_carry + (t ? cpart[t - 1] : 0);
#pragma unroll
        for (int i = 0; i < kScanPer; ++i) {
            const int j = t * kScanPer + i;
            const uint64_t c = scnt[j];
            scnt[j] = run;
            run += c;
        }
        __syncthreads();
        for (int j = t; (uint64_t)j < m; j += kScanThreads) {
            sc.tile_xfer[base + j] = sx[j];
            sc.tile_cnt[base + j] = scnt[j];
        }
        k_carry = xf_apply(xpart[kScanThreads - 1], k_carry);
        off_carry += cpart[kScanThreads - 1];
        __syncthreads();  // the next chunk reuses the LDS arrays
    }
    if (t == 0) {
        *total = off_carry;
        if (k_carry >> 1) atomicOr(err, 1);
    }
}

// Pass 3: positions through an LDS window, written as contiguous rows.
__global__ void __launch_bounds__(kJThreads) json_emit_kernel(Scratch sc, uint64_t ntiles, const uint64_t* total_dev,
                                                              uint32_t* __restrict__ out, uint64_t max_out, int* err) {
    __shared__ uint32_t win[kEmitWindow];
    const uint64_t lane = (uint64_t)blockIdx.x * kJThreads + threadIdx.x;
    const int tk = (int)sc.tile_xfer[blockIdx.x];
    const int ls = xf_apply(sc.lane_prefix[lane], tk);
    uint64_t m = position_mask(ls & 1 ? sc.q1[lane] : sc.q0[lane], sc.st[lane], ls >> 1);
    uint32_t idx = (uint32_t)((sc.lane_off[lane] >> (16 * tk)) & 0xFFFF);
    const uint64_t tile_off = sc.tile_cnt[blockIdx.x];
    const uint64_t tile_end = blockIdx.x + 1 < ntiles ? sc.tile_cnt[blockIdx.x + 1] : *total_dev;
    const uint32_t count = (uint32_t)(tile_end - tile_off);
    const uint32_t base = (uint32_t)(lane * kLaneBytes);
    for (uint32_t w0 = 0; w0 < count; w0 += kEmitWindow) {  // uniform trip count
        const uint32_t wend = w0 + kEmitWindow;
        while (m && idx < wend) {
            const int i = __builtin_ctzll(m);
            m &= m - 1;
            win[idx - w0] = base + (uint32_t)i;
            ++idx;
        }
        __syncthreads();
        const uint32_t nwin = count - w0 < kEmitWindow ? count - w0 : kEmitWindow;
        for (uint32_t j = threadIdx.x; j < nwin; j += kJThreads) {
            const uint64_t g = tile_off + w0 + j;
            if (g < max_out) out[g] = win[j];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0 && tile_end > max_out && tile_off < tile_end) atomicOr(err, 2);
}

// json2pb integer arrays (the reference converts them element by element
// from rapidjson values, src/json2pb/json_to_pb.cpp).
// One lane per element; a workgroup's 256 elements are one contiguous span
// of text, staged into LDS with loads that are all issued before any is
// used (the text is pinned host memory: a lane walking its element byte by
// byte would pay a PCIe round trip per character). Spans longer than the
// LDS window (long runs of whitespace) are read from memory directly.
constexpr uint32_t kIntSpan = 16384;

__device__ __forceinline__ bool json_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

__global__ void __launch_bounds__(256) json_int_array_kernel(const char* __restrict__ text,
                                                             const uint32_t* __restrict__ seps, uint32_t n,
                                                             int64_t* __restrict__ out, int32_t* __restrict__ bad) {
    __shared__ char span[kIntSpan];
    __shared__ uint32_t lo_s, hi_s;
    const uint32_t first = blockIdx.x * blockDim.x;
    const uint32_t i = first + threadIdx.x;
    const uint32_t last = min(first + blockDim.x, n);  // elements [first, last)
    uint32_t b = 0, e = 0;
    if (i < n) {
        b = seps[i] + 1;
        e = seps[i + 1];
    }
    if (threadIdx.x == 0) lo_s = seps[first] + 1;
    if (i + 1 == last) hi_s = e;
    __syncthreads();
    const uint32_t lo = lo_s, hi = hi_s;
    const bool staged = hi - lo <= kIntSpan;
    if (staged) {
        constexpr int kPer = kIntSpan / 256;
        char v[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const uint32_t j = threadIdx.x + (uint32_t)k * 256;
            v[k] = lo + j < hi ? text[lo + j] : 0;
        }
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const uint32_t j = threadIdx.x + (uint32_t)k * 256;
            if (lo + j < hi) span[j] = v[k];
        }
    }
    __syncthreads();
    if (i >= n) return;
    // positions stay absolute; an LDS pointer must never be offset below the
    // array (a flat address below the LDS aperture is a global address)
    auto at = [&](uint32_t k) -> char { return staged ? span[k - lo] : text[k]; };
    while (b < e && json_ws(at(b))) ++b;
    while (e > b && json_ws(at(e - 1))) --e;
    bool neg = false;
    if (b < e && at(b) == '-') {
        neg = true;
        ++b;
    }
    bool ok = b < e && e - b <= 20;
    uint64_t v = 0;
    for (uint32_t k = b; ok && k < e; ++k) {
        const uint32_t d = (uint32_t)(unsigned char)at(k) - '0';
        if (d > 9 || v > (0xFFFFFFFFFFFFFFFFull - d) / 10) {
            ok = false;
            break;
        }
        v = v * 10 + d;
    }
    if (ok) ok = neg ? v <= 0x8000000000000000ull : v <= 0x7FFFFFFFFFFFFFFFull;
    if (!ok) {
        *bad = 1;
        return;
    }
    out[i] = neg ? (int64_t)((uint64_t)0 - v) : (int64_t)v;
}

}  // namespace

int LaunchJsonIntArray(const char* text, const uint32_t* seps, uint32_t n, int64_t* out, int32_t* bad,
                       hipStream_t s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(json_int_array_kernel, dim3((n + 255) / 256), dim3(256), 0, s, text, seps, n, out, bad);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t JsonIndexScratchBytes(uint64_t n) {
    const uint64_t tiles = (n + kJTile - 1) / kJTile;
    const uint64_t lanes = tiles * kJThreads;
    return (size_t)(lanes * (4 * sizeof(uint64_t) + 1) + tiles * (sizeof(uint64_t) + sizeof(uint32_t)) + 64);
}

int LaunchJsonIndex(const uint8_t* in, uint64_t n, uint32_t* out_pos, uint64_t max_out, uint64_t* count_dev,
                    int* err_dev, void* scratch, hipStream_t s) {
    if (n > 0xFFFFFFFFull) return -1;  // positions are 32-bit
    if (n == 0) {
        if (hipMemsetAsync(err_dev, 0, sizeof(int), s) != hipSuccess) return -1;
        return hipMemsetAsync(count_dev, 0, sizeof(uint64_t), s) == hipSuccess ? 0 : -1;
    }
    const uint64_t tiles = (n + kJTile - 1) / kJTile;
    const Scratch sc = carve(scratch, tiles);
    const dim3 grid((uint32_t)tiles), block(kJThreads);
    hipLaunchKernelGGL(json_tile_kernel, grid, block, 0, s, in, n, sc, err_dev);
    hipLaunchKernelGGL(json_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, sc, tiles, count_dev, err_dev);
    hipLaunchKernelGGL(json_emit_kernel, grid, block, 0, s, sc, tiles, (const uint64_t*)count_dev, out_pos, max_out,
                       err_dev);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace gpu
}  // namespace mrpc
