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
#include <map>
#include <mutex>
#include <vector>

#include "base/crc32c.h"
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
constexpr int kChunkPows = 128;             // chunks after a chunk inside its segment (2 MiB)
__constant__ uint32_t c_chunk_pow[kChunkPows];  // x^(8*kChunkBytes*a)

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
    // CRC kernels: consecutive segments may form one MESSAGE whose CRC32C is
    // folded on the device (the concatenation of its segments), so the host
    // never combines per-segment CRCs
    uint64_t tail[kInlineSegments];       // bytes after the segment inside its message
    uint64_t msg_len[kInlineSegments];    // by message slot
    uint32_t msg_chunks[kInlineSegments]; // by message slot: chunks of all its segments
    uint8_t msg[kInlineSegments];         // message slot of the segment
    uint8_t first_of_msg[kInlineSegments];
    // CRC batches: x^(8*tail) per segment and each message's init/final term
    // (x^(8*len)*~0 ^ ~0), computed on the host by fill_batch so the one
    // lane that folds a chunk does two multiplies, not a log-time power
    uint32_t tail_poly[kInlineSegments];
    uint32_t msg_init[kInlineSegments];
    // completion word (DoneWord in kernels.h); null: the launch has none
    uint32_t* done_ctr;
    unsigned long long* done_word;
    unsigned long long done_seq;
    unsigned long long done_pad;  // keeps sizeof a multiple of 16 (LDS staging of the resident ring)
};

// End of a workgroup of a launch with a completion word: after every lane's
// stores, release them at agent scope and count the workgroup; the last one
// resets the counter for the next launch and publishes the sequence number
// to the host (system scope). Uniform per launch: no divergence without a word.
// Each workgroup's first lane does the agent-scope release (an L2
// write-back of ITS XCD) after every wave's stores were acknowledged by L2
// (s_waitcnt 0 before the barrier), so the word implies every XCD that ran
// a workgroup wrote its part back.
__device__ __forceinline__ void signal_done(const SegBatch& b) {
    if (!b.done_word) return;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t before = __hip_atomic_fetch_add(b.done_ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (before + 1 == gridDim.x) {
            __hip_atomic_store(b.done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            b.done_word[2] = wall_clock64();
            __hip_atomic_store(b.done_word, b.done_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

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

// Per-launch-group fold of the chunk CRCs of each message, with no
// zero-initialised output (so no memset launch per batch): every chunk
// folds into its message's 64-bit slot of a per-stream scratch with ONE
// compare-and-swap that both XORs its CRC into the low half and counts it
// in the high half, so the chunk that completes the count holds the final
// CRC in its own CAS result — no fences, no second read. It resets the slot
// for the next launch on the stream and stores the CRC straight into `out`
// (device memory, or pinned host memory the CPU reads after the batch's
// event: no D2H copy).
__device__ __forceinline__ void fold_segment_crc(uint32_t* __restrict__ scratch, int m, uint32_t chunks,
                                                 uint32_t acc, uint32_t* __restrict__ out, uint32_t count = 1) {
    if (chunks == count) {  // this fold carries every chunk of the message
        out[m] = acc;
        return;
    }
    // XOR is order-free: one atomic XOR into the message's CRC word, then one
    // counter increment that releases it; the chunk that brings the count to
    // `chunks` acquires every other chunk's XOR, takes the CRC and resets the
    // slot. Two single-shot L2 atomics per chunk (a CAS loop on one 64-bit
    // word serialized the 64 chunks of a 1 MiB message behind retries).
    uint32_t* crc_word = scratch + 2 * m;
    uint32_t* cnt_word = scratch + 2 * m + 1;
    __hip_atomic_fetch_xor(crc_word, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t before = __hip_atomic_fetch_add(cnt_word, count, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (before + count == chunks) {
        const uint32_t v = __hip_atomic_exchange(crc_word, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(cnt_word, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        out[m] = v;
    }
}

// x^(8*kChunkBytes*a): a table lookup for the chunk counts of segments up
// to 2 MiB, the log-time power beyond.
__device__ __forceinline__ uint32_t chunk_shift_poly(uint32_t a) {
    return a < (uint32_t)kChunkPows ? c_chunk_pow[a] : shift_bytes_poly((uint64_t)a * kChunkBytes);
}

// One chunk's raw CRC: shift it by the bytes that follow the chunk inside its
// MESSAGE (the rest of its segment plus the segments after it), add the ~0
// init / final inversion once per message (std = raw0(M) ^ shift(~0,
// len(M)) ^ ~0), and fold it into the message's slot.
__device__ __forceinline__ void fold_chunk(const SegBatch& b, int seg, uint32_t after, uint32_t seg_chunks,
                                           uint32_t acc, uint32_t* __restrict__ scratch,
                                           uint32_t* __restrict__ out) {
    if (after) acc = mult_mod_p(chunk_shift_poly(after), acc);
    if (b.tail[seg]) acc = mult_mod_p(b.tail_poly[seg], acc);
    const int m = b.msg[seg];
    if (after == seg_chunks - 1 && b.first_of_msg[seg]) acc ^= b.msg_init[m];
    fold_segment_crc(scratch, m, b.msg_chunks[m], acc, out);
}

__global__ void __launch_bounds__(kThreads) crc32c_kernel(SegBatch b, const uint32_t* __restrict__ tables,
                                                          uint32_t* __restrict__ scratch, uint32_t* __restrict__ out) {
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
        fold_chunk(b, seg, after, seg_chunks, acc, scratch, out);
    }
}

__device__ __forceinline__ void stamp_start(const SegBatch& b) {
    if (b.done_word && blockIdx.x == 0 && threadIdx.x == 0) b.done_word[1] = wall_clock64();
}

__global__ void __launch_bounds__(kThreads) batched_copy_kernel(SegBatch b) {
    stamp_start(b);
    const uint32_t chunk = blockIdx.x;
    const int seg = find_segment(b, chunk);
    const uint64_t len = b.len[seg];
    const uint64_t k = chunk - b.chunk_start[seg];
    const uint8_t* src = static_cast<const uint8_t*>(b.src[seg]);
    uint8_t* dst = static_cast<uint8_t*>(b.dst[seg]);
    const uint64_t cbeg = k * kChunkBytes;
    const uint64_t cend = cbeg + kChunkBytes < len ? cbeg + kChunkBytes : len;
    const bool aligned = (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0);
    if (aligned && cend - cbeg == kChunkBytes) {
        // full 16 KiB chunk: each lane issues all four 16 B loads before any
        // store (4 KiB stripes, coalesced), so 64 B per lane are in flight —
        // what a pull across xGMI needs to cover the remote-read latency
        const uint4* __restrict__ s4 = reinterpret_cast<const uint4*>(src + cbeg) + threadIdx.x;
        uint4* __restrict__ d4 = reinterpret_cast<uint4*>(dst + cbeg) + threadIdx.x;
        uint4 v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = s4[i * kThreads];
#pragma unroll
        for (int i = 0; i < 4; ++i) d4[i * kThreads] = v[i];
    } else if (aligned) {
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
    signal_done(b);
}

// Fused pull + checksum: the batched copy and the LDS CRC32C in ONE pass
// over the bytes (the data is read once — from local HBM, a peer GPU's HBM
// across xGMI, or pinned host memory — stored to dst and folded into the
// CRC while in registers). Same end-aligned chunk/lane geometry as
// crc32c_kernel, so every partial CRC is shifted by a table-resident power
// of x and chunks fold with one atomicXor per workgroup. Misaligned
// segments (an attachment that starts mid-block after the RPC meta) use
// unaligned 16 B accesses, which gfx950 serves natively.
typedef uint32_t u32x4_unaligned __attribute__((ext_vector_type(4), aligned(1)));

__global__ void __launch_bounds__(kThreads) copy_crc32c_kernel(SegBatch b, const uint32_t* __restrict__ tables,
                                                               uint32_t* __restrict__ scratch,
                                                               uint32_t* __restrict__ out) {
    stamp_start(b);
    __shared__ uint32_t t[8][256];
    __shared__ uint32_t wave_acc[kThreads / 64];
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
    uint8_t* dbase = static_cast<uint8_t*>(b.dst[seg]);
    const uint32_t seg_chunks = b.chunk_start[seg + 1] - b.chunk_start[seg];
    const uint32_t k = chunk - b.chunk_start[seg];
    const uint32_t after = seg_chunks - 1 - k;
    const int64_t chunk_end = (int64_t)len - (int64_t)after * (int64_t)kChunkBytes;
    const int64_t lane_end = chunk_end - (int64_t)(kThreads - 1 - threadIdx.x) * kLaneBytes;
    const int64_t lane_beg = lane_end - kLaneBytes;
    __syncthreads();

    uint32_t crc = 0;
    if (lane_end > 0) {
        if (lane_beg >= 0) {
            const u32x4_unaligned* p = reinterpret_cast<const u32x4_unaligned*>(base + lane_beg);
            u32x4_unaligned* q = reinterpret_cast<u32x4_unaligned*>(dbase + lane_beg);
            u32x4_unaligned v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = p[i];
            if (dbase) {  // null destination: checksum only (uniform per segment)
#pragma unroll
                for (int i = 0; i < 4; ++i) q[i] = v[i];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                crc = crc_word8(crc, v[i].x, v[i].y, t);
                crc = crc_word8(crc, v[i].z, v[i].w, t);
            }
        } else {
            for (int64_t i = 0; i < lane_end; ++i) {
                const uint8_t c = base[i];
                if (dbase) dbase[i] = c;
                crc = t[0][(crc ^ c) & 0xff] ^ (crc >> 8);
            }
        }
        crc = mult_mod_p(c_lane_shift[kThreads - 1 - threadIdx.x], crc);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) crc ^= __shfl_xor(crc, off, 64);
    if ((threadIdx.x & 63) == 0) wave_acc[threadIdx.x >> 6] = crc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = wave_acc[0] ^ wave_acc[1] ^ wave_acc[2] ^ wave_acc[3];
        fold_chunk(b, seg, after, seg_chunks, acc, scratch, out);
    }
    signal_done(b);
}

// ---------------------------------------------------------------- CRC32C on MFMA
//
// CRC32C over GF(2) is linear in the message bits, so the CRC of a 64-byte
// block is a 32x512 bit-matrix times the block's bits. That product runs on
// the int8 matrix cores: v_mfma_i32_32x32x32_i8 with
//   A[r][k] = bit r of the CRC contribution of block-bit k   (constant)
//   B[k][c] = block-bit k of column c (0/1 bytes expanded from the data)
//   D[r][c] = number of set bits whose contribution has bit r
// and the CRC bit is the parity of D. One wave owns a 2 KiB group = 32
// columns x 64 B per pass (16 MFMAs, K = 512 bits). Lane (c, h) holds column
// c's bytes [32h, 32h+32), loaded as two 16 B vectors; because A and B share
// the same k order inside a lane half, the bit->k assignment never needs the
// exact fragment layout. Columns are folded across the wave-chunk (32
// groups = 64 KiB) with a Horner step whose constant (x^(8*2048)) is applied
// through four LDS byte tables, then each lane applies its column shift
// x^(512*(31-c)) once per chunk and the wave XOR-reduces. Chunks fold into
// the segment result with one atomicXor (order-free, like the LDS kernel).
typedef signed char i8x16 __attribute__((ext_vector_type(16)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int kGroupBytes = 2048;                       // 32 columns x 64 B
static_assert(kChunkBytes == 2 * kGroupBytes * (kThreads / 64), "copy_crc32c_mfma_kernel: 2 groups per wave");
static_assert(kChunkBytes == (1u << 14), "copy_crc32c_mfma_kernel: Horner constant x^(8*kChunkBytes) = c_x2n[17]");
constexpr int kGroupsPerChunk = 32;
constexpr uint64_t kMfmaChunk = (uint64_t)kGroupBytes * kGroupsPerChunk;  // 64 KiB per wave

struct CrcMfmaConsts {
    i8x16 afrag[16][64];     // A fragments, [mfma j][lane]
    uint32_t t2k[4][256];    // byte tables of "multiply by x^(8*2048)"
    uint32_t lane_shift[32]; // x^(512*(31-c))
    uint32_t xl[256];        // x^(8r), r < 256
    uint32_t xm[256];        // x^(8*256*q), q < 256
};

__device__ __forceinline__ i8x16 expand16(uint32_t bits) {
    union {
        uint32_t u[4];
        i8x16 v;
    } r;
#pragma unroll
    for (int q = 0; q < 4; ++q) r.u[q] = (((bits >> (4 * q)) & 0xFu) * 0x00204081u) & 0x01010101u;
    return r.v;
}

// Rare path (leading partial group / unaligned segment end). Inlined with
// w[] by reference so the array stays in registers: an out-of-line helper
// taking a pointer forced it into 80 bytes of per-lane scratch.
__device__ __forceinline__ void fetch_bytes_slow(const uint8_t* base, int64_t lbeg, uint32_t (&w)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = 0;
#pragma unroll
    for (int b = 0; b < 32; ++b) {
        const int64_t off = lbeg + b;
        if (off >= 0) w[b >> 2] |= (uint32_t)base[off] << (8 * (b & 3));
    }
}

__global__ void __launch_bounds__(kThreads) crc32c_mfma_kernel(
    const uint64_t* __restrict__ starts, const uint64_t* __restrict__ lens, const uint64_t* __restrict__ chunk_start,
    int64_t nseg, const CrcMfmaConsts* __restrict__ K, const uint32_t* __restrict__ xc, uint32_t* __restrict__ out) {
    // A fragments (16 KiB) and the Horner tables (4 KiB) live in LDS: the
    // fragments would otherwise pin 64 VGPRs per lane and cap occupancy at
    // 3 waves/SIMD; ds_read_b128 of consecutive lanes is conflict-free.
    __shared__ i8x16 sa[16][64];
    __shared__ uint32_t t2k[4][256];
    for (int i = threadIdx.x; i < 16 * 64; i += kThreads) (&sa[0][0])[i] = (&K->afrag[0][0])[i];
    for (int i = threadIdx.x; i < 1024; i += kThreads) (&t2k[0][0])[i] = (&K->t2k[0][0])[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int c = lane & 31;
    const int h = lane >> 5;
    const uint32_t lshift = K->lane_shift[c];
    const uint64_t total = chunk_start[nseg];
    const uint64_t nwaves = (uint64_t)gridDim.x * (kThreads / 64);
    for (uint64_t chunk = (uint64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6); chunk < total;
         chunk += nwaves) {
        int64_t lo = 0, hi = nseg - 1;
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) >> 1;
            if (chunk_start[mid] <= chunk) lo = mid;
            else hi = mid - 1;
        }
        const int64_t seg = lo;
        const uint64_t len = lens[seg];
        const uint8_t* base = reinterpret_cast<const uint8_t*>(starts[seg]);
        const uint64_t nch = chunk_start[seg + 1] - chunk_start[seg];
        const uint64_t k = chunk - chunk_start[seg];
        const uint64_t after = nch - 1 - k;
        const int64_t chunk_end = (int64_t)len - (int64_t)(after * kMfmaChunk);
        const bool aligned = ((reinterpret_cast<uintptr_t>(base) + len) & 15) == 0;
        // lane's 32 bytes of group gg; bytes before the segment read as zero
        // (a zero prefix leaves the CRC register unchanged)
        auto fetch = [&](int gg, uint32_t(&w)[8]) {
            const int64_t gend = chunk_end - (int64_t)(kGroupsPerChunk - 1 - gg) * kGroupBytes;
            const int64_t lbeg = gend - kGroupBytes + 64 * c + 32 * h;
            if (lbeg >= 0 && aligned) {
                const uint4* p = reinterpret_cast<const uint4*>(base + lbeg);
                const uint4 v0 = p[0], v1 = p[1];
                w[0] = v0.x; w[1] = v0.y; w[2] = v0.z; w[3] = v0.w;
                w[4] = v1.x; w[5] = v1.y; w[6] = v1.z; w[7] = v1.w;
            } else {
                fetch_bytes_slow(base, lbeg, w);
            }
        };
        // first group that overlaps the segment (wave-uniform)
        int g0 = 0;
        while (g0 < kGroupsPerChunk && chunk_end - (int64_t)(kGroupsPerChunk - 1 - g0) * kGroupBytes <= 0) ++g0;
        uint32_t acc = 0;
        uint32_t cur[8], nxt[8];
        if (g0 < kGroupsPerChunk) fetch(g0, cur);
        for (int g = g0; g < kGroupsPerChunk; ++g) {
            // issue the next group's loads before this group's MFMA work so a
            // wave keeps 4 KiB in flight (Little's law at ~2 us HBM latency)
            if (g + 1 < kGroupsPerChunk) fetch(g + 1, nxt);
            i32x16 d = {0};
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t bits = (cur[j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                d = __builtin_amdgcn_mfma_i32_32x32x32_i8(sa[j][lane], expand16(bits), d, 0, 0, 0);
                // keep fragment reads / bit expansion within a window of 4
                // MFMAs instead of letting the scheduler hoist all 16 (VGPRs)
                if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) cur[i] = nxt[i];
            // D layout: col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
            uint32_t part = 0;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
                part |= ((uint32_t)d[reg] & 1u) << row;
            }
            const uint32_t crc_c = part | __shfl_xor(part, 32, 64);
            acc = t2k[0][acc & 0xff] ^ t2k[1][(acc >> 8) & 0xff] ^ t2k[2][(acc >> 16) & 0xff] ^ t2k[3][acc >> 24] ^
                  crc_c;
        }
        uint32_t v = mult_mod_p(lshift, acc);
#pragma unroll
        for (int off = 16; off > 0; off >>= 1) v ^= __shfl_xor(v, off, 64);
        if (lane == 0) {
            if (after) v = mult_mod_p(xc[after], v);
            if (k == 0) {
                // fold the ~0 initial register and the final inversion
                const uint32_t x8len = mult_mod_p(mult_mod_p(xc[len / kMfmaChunk], K->xm[(len % kMfmaChunk) >> 8]),
                                                  K->xl[len & 0xff]);
                v ^= mult_mod_p(x8len, 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
            }
            atomicXor(out + seg, v);
        }
    }
}

// Fused pull + checksum with the CRC on the matrix cores: the batched
// copy's 16 KiB end-aligned chunks (fill_batch / fold_chunk geometry, so the
// message folding is shared with copy_crc32c_kernel), 4 KiB per wave, two
// 2 KiB MFMA groups per wave. Lane (c, h) of a wave loads the 32 bytes
// [64c + 32h, +32) of each group — exactly the B-fragment bytes of the MFMA
// CRC — stores them to dst, and expands them into the 16 MFMAs of the group.
// Each column's 64-byte CRC is shifted straight to the chunk end with one
// multiply by x^(8*64*j), j = 64-byte blocks after it in the chunk (the
// c_lane_shift table), so no Horner chain links the groups. The byte-table
// kernel's per-lane serial table lookups ran at ~230 GB/s (3% of HBM) and
// held the 1 MiB verified leg GPU-bound; the A fragments come from LDS,
// staged once per workgroup, and a workgroup walks several chunks so the
// staging amortises.
// A lane's 32 bytes that start before the segment: bytes at offsets < 0
// read as zero and are not stored. Fully unrolled so w[] stays in registers
// (an out-of-line helper taking w by pointer put every lane's w[] in
// scratch memory: 80 bytes of private segment per lane, ~230 GB/s).
__device__ __forceinline__ void copy_bytes_slow(const uint8_t* base, uint8_t* dbase, int64_t lbeg, uint32_t (&w)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = 0;
#pragma unroll
    for (int b = 0; b < 32; ++b) {
        const int64_t off = lbeg + b;
        if (off >= 0) {
            const uint32_t c = base[off];
            if (dbase) dbase[off] = (uint8_t)c;
            w[b >> 2] |= c << (8 * (b & 3));
        }
    }
}

// A run of consecutive chunks of one segment: each wave Horner-folds its
// own 4 KiB slab of every chunk of the run (each new chunk follows the
// previous one by 16 KiB), and only where the run ends — a segment change
// or the end of the workgroup's range, the same chunk for all four waves —
// the waves combine through LDS and one lane shifts the run to the message
// end and folds it with ONE atomic. A barrier per chunk (to combine there)
// waited for the wave's global stores every chunk (272 GB/s on 256 MiB);
// one atomic fold per wave instead of per workgroup contended on the
// message's fold words (50k vs 125k QPS on the 1 MiB verified leg).
struct ChunkRun {
    int seg = -1;
    uint32_t acc = 0, n = 0, after_last = 0;
    bool has_first = false;  // the run holds the segment's first chunk
};

__device__ __forceinline__ void flush_run(const SegBatch& b, ChunkRun& r, uint32_t* wave_acc,
                                          uint32_t* __restrict__ scratch, uint32_t* __restrict__ out) {
    if (r.seg < 0) return;  // uniform: every wave ran the same chunks
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) wave_acc[wave] = r.acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (int w = 0; w < kThreads / 64; ++w) acc ^= wave_acc[w];
        if (r.after_last) acc = mult_mod_p(chunk_shift_poly(r.after_last), acc);
        if (b.tail[r.seg]) acc = mult_mod_p(b.tail_poly[r.seg], acc);
        const int m = b.msg[r.seg];
        if (r.has_first && b.first_of_msg[r.seg]) acc ^= b.msg_init[m];
        fold_segment_crc(scratch, m, b.msg_chunks[m], acc, out, r.n);
    }
    __syncthreads();  // wave_acc is reused by the next run
    r = ChunkRun();
}

__global__ void __launch_bounds__(kThreads) copy_crc32c_mfma_kernel(SegBatch b, const CrcMfmaConsts* __restrict__ K,
                                                                    uint32_t* __restrict__ scratch,
                                                                    uint32_t* __restrict__ out, uint32_t nchunks) {
    stamp_start(b);
    __shared__ i8x16 sa[16][64];
    __shared__ uint32_t wave_acc[kThreads / 64];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int c = lane & 31;
    const int h = lane >> 5;
    // a contiguous range of chunks per workgroup (one per workgroup up to
    // the grid cap), so runs of one segment fold locally
    const uint32_t per = (nchunks + gridDim.x - 1) / gridDim.x;
    const uint32_t c0 = blockIdx.x * per;
    const uint32_t c1 = min(nchunks, c0 + per);
    ChunkRun run;  // this wave's slab accumulator (uniform across its lanes)
    for (uint32_t chunk = c0; chunk < c1; ++chunk) {
        const int seg = find_segment(b, chunk);
        const uint64_t len = b.len[seg];
        const uint8_t* base = static_cast<const uint8_t*>(b.src[seg]);
        uint8_t* dbase = static_cast<uint8_t*>(b.dst[seg]);
        const uint32_t seg_chunks = b.chunk_start[seg + 1] - b.chunk_start[seg];
        const uint32_t k = chunk - b.chunk_start[seg];
        const uint32_t after = seg_chunks - 1 - k;
        const int64_t chunk_end = (int64_t)len - (int64_t)after * (int64_t)kChunkBytes;
        const int64_t wave_end = chunk_end - (int64_t)(kThreads / 64 - 1 - wave) * 4096;
        // both groups' loads first: 64 B per lane in flight, as in the copy kernel
        uint32_t w[2][8];
        bool any[2];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            const int64_t lbeg = wave_end - (int64_t)(2 - g) * 2048 + 64 * c + 32 * h;
            any[g] = lbeg + 32 > 0;
            if (lbeg >= 0) {
                const u32x4_unaligned* p = reinterpret_cast<const u32x4_unaligned*>(base + lbeg);
                const u32x4_unaligned v0 = p[0], v1 = p[1];
                w[g][0] = v0.x; w[g][1] = v0.y; w[g][2] = v0.z; w[g][3] = v0.w;
                w[g][4] = v1.x; w[g][5] = v1.y; w[g][6] = v1.z; w[g][7] = v1.w;
            } else if (any[g]) {
                copy_bytes_slow(base, dbase, lbeg, w[g]);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) w[g][i] = 0;
            }
        }
        if (chunk == c0) {
            // stage the A fragments (16 KiB from L2) behind the first
            // chunk's loads, so a one-chunk workgroup (the RPC batches)
            // waits for both latencies at once, not one after the other;
            // the workgroup's only barrier
            for (int i = threadIdx.x; i < 16 * 64; i += kThreads) (&sa[0][0])[i] = (&K->afrag[0][0])[i];
            __syncthreads();
        }
        if (dbase) {  // null destination: checksum only (uniform per segment)
#pragma unroll
            for (int g = 0; g < 2; ++g) {
                const int64_t lbeg = wave_end - (int64_t)(2 - g) * 2048 + 64 * c + 32 * h;
                if (lbeg >= 0) {
                    u32x4_unaligned* q = reinterpret_cast<u32x4_unaligned*>(dbase + lbeg);
                    u32x4_unaligned v0, v1;
                    v0.x = w[g][0]; v0.y = w[g][1]; v0.z = w[g][2]; v0.w = w[g][3];
                    v1.x = w[g][4]; v1.y = w[g][5]; v1.z = w[g][6]; v1.w = w[g][7];
                    q[0] = v0;
                    q[1] = v1;
                }
            }
        }
        uint32_t v = 0;
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            // a group wholly before the segment adds nothing (wave-uniform)
            if (!__ballot(any[g])) continue;
            i32x16 d = {0};
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const uint32_t bits = (w[g][j >> 1] >> (16 * (j & 1))) & 0xFFFFu;
                d = __builtin_amdgcn_mfma_i32_32x32x32_i8(sa[j][lane], expand16(bits), d, 0, 0, 0);
                if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
            uint32_t part = 0;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
                part |= ((uint32_t)d[reg] & 1u) << row;
            }
            const uint32_t crc_c = part | __shfl_xor(part, 32, 64);
            // 64-byte blocks after column c of group g inside the chunk
            const int blocks_after = 64 * (kThreads / 64 - 1 - wave) + 32 * (1 - g) + (31 - c);
            v ^= mult_mod_p(c_lane_shift[blocks_after], crc_c);
        }
        // the 32 columns (each present twice, once per lane half): every
        // lane ends with the slab's CRC, shifted to the chunk end
#pragma unroll
        for (int off = 16; off > 0; off >>= 1) v ^= __shfl_xor(v, off, 64);
        if (run.seg != seg) {
            flush_run(b, run, wave_acc, scratch, out);
            run.seg = seg;
            run.has_first = k == 0;
        }
        // Horner: everything folded so far precedes this chunk by 16 KiB
        run.acc = run.n ? mult_mod_p(c_x2n[17], run.acc) ^ v : v;  // x^(8*16384) = x^(2^17)
        run.n += 1;
        run.after_last = after;
    }
    flush_run(b, run, wave_acc, scratch, out);
    signal_done(b);
}

__global__ void crc_chunk_count_kernel(const uint64_t* __restrict__ lens, int64_t nseg, uint64_t* __restrict__ cs) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nseg) {
        const uint64_t n = (lens[i] + kMfmaChunk - 1) / kMfmaChunk;
        cs[i] = n ? n : 1;
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

// Decode: lane owns 16 input bytes (one coalesced 16 B load) and sees the
// previous lane's 16 bytes through a DPP shuffle (lane 0 of a wave loads
// them), so every varint ending in its bytes (<= 10 bytes long) is decoded
// from registers: a terminator mask locates the start, a 128-bit funnel
// shift brings the bytes into two words and the 7-bit groups are packed
// with shifts and masks. No data-dependent loops over global memory.
__device__ __forceinline__ uint32_t term_mask16(uint4 v) {
    // bit i set <=> byte i has its MSB clear (ends a varint)
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t t = ~w[i] & 0x80808080u;
        m |= (((t >> 7) & 1u) | ((t >> 14) & 2u) | ((t >> 21) & 4u) | ((t >> 28) & 8u)) << (4 * i);
    }
    return m;
}

__device__ __forceinline__ uint64_t pack7(uint64_t a, uint64_t b) {
    // bytes a[0..7], b[0..1] -> 70 bits of payload, low 64 kept
    uint64_t v = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) v |= ((a >> (8 * j)) & 0x7full) << (7 * j);
    v |= (b & 0x7full) << 56;
    v |= ((b >> 8) & 0x01ull) << 63;
    return v;
}

__global__ void __launch_bounds__(kThreads) varint_decode_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                                 const uint64_t* __restrict__ tile_offsets,
                                                                 uint64_t* __restrict__ out, uint64_t max_out,
                                                                 int zigzag, int* __restrict__ err) {
    __shared__ uint32_t smem[kThreads / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kVTile + threadIdx.x * 16;
    const int lane = threadIdx.x & 63;
    uint4 cur = make_uint4(0, 0, 0, 0);
    int nb = 0;
    if (base < n) {
        nb = (int)(n - base < 16 ? n - base : 16);
        if (nb == 16 && (reinterpret_cast<uintptr_t>(in + base) & 15) == 0) {
            cur = *reinterpret_cast<const uint4*>(in + base);
        } else {
            uint32_t w[4] = {0, 0, 0, 0};
            for (int i = 0; i < nb; ++i) w[i >> 2] |= (uint32_t)in[base + i] << (8 * (i & 3));
            cur = make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
    // previous 16 bytes: neighbour lane, or memory for lane 0 (zeros before
    // the stream start act as terminators)
    uint4 prev;
    prev.x = __shfl_up(cur.x, 1, 64);
    prev.y = __shfl_up(cur.y, 1, 64);
    prev.z = __shfl_up(cur.z, 1, 64);
    prev.w = __shfl_up(cur.w, 1, 64);
    if (lane == 0) {
        if (base >= 16) {
            if ((reinterpret_cast<uintptr_t>(in + base - 16) & 15) == 0) {
                prev = *reinterpret_cast<const uint4*>(in + base - 16);
            } else {
                uint32_t w[4] = {0, 0, 0, 0};
                for (int i = 0; i < 16; ++i) w[i >> 2] |= (uint32_t)in[base - 16 + i] << (8 * (i & 3));
                prev = make_uint4(w[0], w[1], w[2], w[3]);
            }
        } else {
            prev = make_uint4(0, 0, 0, 0);
        }
    }
    uint32_t tcur = term_mask16(cur);
    if (nb < 16) tcur &= (1u << nb) - 1;  // bytes past the end are not terminators
    const uint32_t window_terms = term_mask16(prev) | (tcur << 16);
    uint32_t total;
    uint64_t idx = tile_offsets[blockIdx.x] + block_exclusive_scan(__popc(tcur), &total, smem);
    const uint64_t W[4] = {((uint64_t)prev.y << 32) | prev.x, ((uint64_t)prev.w << 32) | prev.z,
                           ((uint64_t)cur.y << 32) | cur.x, ((uint64_t)cur.w << 32) | cur.z};
    uint32_t t = tcur;
    while (t) {
        const int i = __ffs(t) - 1;  // terminator at window position 16+i
        t &= t - 1;
        const int end = 16 + i;
        const uint32_t below = window_terms & ((1u << end) - 1);
        const int start = below ? 32 - __clz(below) : 0;  // after the previous terminator
        const int len = end - start + 1;
        if (len > 10 || (!below && base >= 16)) {
            atomicOr(err, 1);
            ++idx;
            continue;
        }
        // 16 bytes from window position `start` (start <= 31): funnel shift
        const int wi = start >> 3, sh = (start & 7) * 8;
        const uint64_t w0 = W[wi];
        const uint64_t w1 = wi + 1 < 4 ? W[wi + 1] : 0;
        const uint64_t w2 = wi + 2 < 4 ? W[wi + 2] : 0;
        const uint64_t a = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
        const uint64_t b = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
        uint64_t v = pack7(a, b);
        if (len < 10) v &= (1ull << (7 * len)) - 1;
        if (zigzag) v = (v >> 1) ^ (~(v & 1) + 1);
        if (idx < max_out) out[idx] = v;
        else atomicOr(err, 2);
        ++idx;
    }
    // a trailing continuation byte means truncated input
    if (nb > 0 && base + nb == n && !((tcur >> (nb - 1)) & 1)) atomicOr(err, 1);
}

__device__ __forceinline__ uint32_t varint_len(uint64_t v) {
    // 1 + floor(bit_width(v)-1)/7, with v=0 -> 1
    const int bits = v ? 64 - __clzll(v) : 1;
    return (uint32_t)((bits + 6) / 7);
}

__device__ __forceinline__ uint64_t zz(uint64_t v, int zigzag) {
    return zigzag ? (v << 1) ^ (uint64_t)((int64_t)v >> 63) : v;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    return x;
}

// Encode: a tile is 4096 values; wave w owns values [1024w, 1024w+1024) and
// walks them 64 at a time with coalesced 8 B loads. Pass 1 of the kernel
// sums the wave's encoded length, the 4 wave totals are scanned in LDS,
// pass 2 re-reads the (cache-resident) values and writes each varint at
// tile_offset + wave_prefix + in-wave scan.
__global__ void __launch_bounds__(kThreads) varint_len_kernel(const uint64_t* __restrict__ in, uint64_t n,
                                                              int zigzag, uint64_t* __restrict__ tile_counts) {
    __shared__ uint32_t smem[kThreads / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kVTile + (threadIdx.x >> 6) * 1024 + (threadIdx.x & 63);
    uint32_t c = 0;
#pragma unroll 4
    for (int k = 0; k < 16; ++k) {
        const uint64_t i = base + (uint64_t)k * 64;
        if (i < n) c += varint_len(zz(in[i], zigzag));
    }
    uint32_t total;
    block_exclusive_scan(c, &total, smem);
    if (threadIdx.x == 0) tile_counts[blockIdx.x] = total;
}

__global__ void __launch_bounds__(kThreads) varint_encode_kernel(const uint64_t* __restrict__ in, uint64_t n,
                                                                 int zigzag,
                                                                 const uint64_t* __restrict__ tile_offsets,
                                                                 uint8_t* __restrict__ out) {
    __shared__ uint32_t wave_tot[kThreads / 64];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * kVTile + (uint64_t)wave * 1024 + lane;
    uint32_t c = 0;
#pragma unroll 4
    for (int k = 0; k < 16; ++k) {
        const uint64_t i = base + (uint64_t)k * 64;
        if (i < n) c += varint_len(zz(in[i], zigzag));
    }
    const uint32_t wt = wave_incl_scan(c);
    if (lane == 63) wave_tot[wave] = wt;
    __syncthreads();
    uint64_t pos = tile_offsets[blockIdx.x];
    for (int w = 0; w < wave; ++w) pos += wave_tot[w];
    for (int k = 0; k < 16; ++k) {
        const uint64_t i = base + (uint64_t)k * 64;
        uint64_t v = i < n ? zz(in[i], zigzag) : 0;
        const uint32_t L = i < n ? varint_len(v) : 0;
        const uint32_t incl = wave_incl_scan(L);
        const uint32_t wsum = __shfl(incl, 63, 64);
        uint8_t* dst = out + pos + (incl - L);
        for (uint32_t j = 0; j < L; ++j) {
            dst[j] = (uint8_t)((v & 0x7f) | (j + 1 < L ? 0x80 : 0));
            v >>= 7;
        }
        pos += wsum;
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

const CrcTables& host_tables() {
    static CrcTables h;
    static std::once_flag once;
    std::call_once(once, [] {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
            h.t8[0][i] = c;
        }
        for (int s = 1; s < 8; ++s) {
            for (int i = 0; i < 256; ++i) h.t8[s][i] = (h.t8[s - 1][i] >> 8) ^ h.t8[0][h.t8[s - 1][i] & 0xff];
        }
        // x2n[k] = x^(2^k) mod P (reflected: x^0 = 1<<31, x^1 = 1<<30)
        uint32_t p = 1u << 30;
        for (int k = 0; k < 64; ++k) {
            h.x2n[k] = p;
            p = host_mult_mod_p(p, p);
        }
        // lane_shift[j] = x^(8*64*j) = (x^512)^j
        uint32_t acc = 1u << 31;
        for (int j = 0; j < 256; ++j) {
            h.lane_shift[j] = acc;
            acc = host_mult_mod_p(h.x2n[9], acc);
        }
    });
    return h;
}

// x^e mod P for an arbitrary bit exponent e
uint32_t host_xpow(uint64_t e) {
    const CrcTables& h = host_tables();
    uint32_t r = 1u << 31;
    for (int k = 0; e && k < 64; ++k, e >>= 1) {
        if (e & 1) r = host_mult_mod_p(h.x2n[k], r);
    }
    return r;
}

struct DeviceTables {
    uint32_t* t8 = nullptr;           // slicing tables (LDS kernel)
    CrcMfmaConsts* mfma = nullptr;    // MFMA kernel constants
    uint32_t* xc = nullptr;           // x^(8*64KiB*m), m < xc_len
    uint64_t xc_len = 0;
    bool ready = false;
};

DeviceTables g_tables[64];
std::mutex g_tables_mu;

int ensure_tables_locked(int dev) {
    DeviceTables& dt = g_tables[dev];
    if (dt.ready) return 0;
    const CrcTables& h = host_tables();
    if (hipMalloc(&dt.t8, sizeof(h.t8)) != hipSuccess) return -1;
    if (hipMemcpy(dt.t8, h.t8, sizeof(h.t8), hipMemcpyHostToDevice) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_lane_shift), h.lane_shift, sizeof(h.lane_shift)) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_x2n), h.x2n, sizeof(h.x2n)) != hipSuccess) return -1;
    {
        uint32_t pows[kChunkPows];
        for (int a = 0; a < kChunkPows; ++a) pows[a] = host_xpow((uint64_t)8 * kChunkBytes * a);
        if (hipMemcpyToSymbol(HIP_SYMBOL(c_chunk_pow), pows, sizeof(pows)) != hipSuccess) return -1;
    }
    // ---- MFMA constants
    static CrcMfmaConsts m;
    static std::once_flag once;
    std::call_once(once, [&h] {
        // contribution of each of the 512 bits of a 64-byte block (zero-init
        // register, no final inversion) = crc_raw0(block with that bit set)
        static uint32_t contrib[512];
        for (int b = 0; b < 512; ++b) {
            uint8_t blk[64] = {0};
            blk[b >> 3] = (uint8_t)(1u << (b & 7));
            uint32_t reg = 0;
            for (int i = 0; i < 64; ++i) reg = h.t8[0][(reg ^ blk[i]) & 0xff] ^ (reg >> 8);
            contrib[b] = reg;
        }
        for (int j = 0; j < 16; ++j) {
            for (int lane = 0; lane < 64; ++lane) {
                const int r = lane & 31, hh = lane >> 5;
                union {
                    signed char c[16];
                    i8x16 v;
                } u;
                for (int e = 0; e < 16; ++e) u.c[e] = (signed char)((contrib[256 * hh + 16 * j + e] >> r) & 1u);
                m.afrag[j][lane] = u.v;
            }
        }
        const uint32_t x2k = h.x2n[14];  // x^(8*2048) = x^(2^14)
        for (int byte = 0; byte < 4; ++byte) {
            for (int v = 0; v < 256; ++v) m.t2k[byte][v] = host_mult_mod_p(x2k, (uint32_t)v << (8 * byte));
        }
        for (int c = 0; c < 32; ++c) m.lane_shift[c] = host_xpow((uint64_t)512 * (31 - c));
        for (int r = 0; r < 256; ++r) m.xl[r] = host_xpow((uint64_t)8 * r);
        for (int q = 0; q < 256; ++q) m.xm[q] = host_xpow((uint64_t)8 * 256 * q);
    });
    if (hipMalloc(&dt.mfma, sizeof(m)) != hipSuccess) return -1;
    if (hipMemcpy(dt.mfma, &m, sizeof(m), hipMemcpyHostToDevice) != hipSuccess) return -1;
    dt.ready = true;
    return 0;
}

int ensure_tables() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -1;
    std::lock_guard<std::mutex> g(g_tables_mu);
    return ensure_tables_locked(dev);
}

// Grow the per-device x^(8*64KiB*m) table to cover m < need. The old table
// is kept alive (leaked) since in-flight kernels may still read it.
const uint32_t* ensure_xc(uint64_t need) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> g(g_tables_mu);
    if (ensure_tables_locked(dev) != 0) return nullptr;
    DeviceTables& dt = g_tables[dev];
    if (dt.xc_len >= need) return dt.xc;
    uint64_t n = 1024;
    while (n < need) n <<= 1;
    std::vector<uint32_t> x(n);
    const uint32_t step = host_tables().x2n[19];  // x^(8*65536) = x^(2^19)
    uint32_t acc = 1u << 31;
    for (uint64_t i = 0; i < n; ++i) {
        x[i] = acc;
        acc = host_mult_mod_p(step, acc);
    }
    uint32_t* d = nullptr;
    if (hipMalloc(&d, n * sizeof(uint32_t)) != hipSuccess) return nullptr;
    if (hipMemcpy(d, x.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    dt.xc = d;
    dt.xc_len = n;
    return d;
}

// The fold scratch of a stream (fold_segment_crc): launches on one stream
// run in order and every launch leaves its slots zeroed, so one zeroed
// allocation per (device, stream) serves them all.
uint32_t* stream_scratch(int dev, hipStream_t s) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, uint32_t*>* m = new std::map<std::pair<int, hipStream_t>, uint32_t*>;
    std::lock_guard<std::mutex> g(mu);
    auto it = m->find({dev, s});
    if (it != m->end()) return it->second;
    uint32_t* p = nullptr;
    const size_t bytes = 2 * kInlineSegments * sizeof(uint32_t);
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    // hipMemset is asynchronous to the host and runs on the null stream,
    // which non-blocking streams do not wait for: without the sync the first
    // launch on `s` could fold into the allocation's old bytes (a wrong CRC
    // once per stream; seen as one GPU-handler CRC mismatch with 8 ranks
    // sharing a GPU, profiles/r5_rehearse8_one_gpu.json)
    if (hipMemset(p, 0, bytes) != hipSuccess || hipStreamSynchronize(nullptr) != hipSuccess) return nullptr;
    (*m)[{dev, s}] = p;
    return p;
}

// Fill a SegBatch with up to kInlineSegments segments; returns chunk count.
// msg_of (optional, non-decreasing): the message each segment belongs to;
// without it every segment is its own message.
// x^(8n) mod P on the host, memoised per thread: RPC batches repeat a few
// lengths (whole payloads, the bytes after a payload's head block).
uint32_t host_shift_poly(uint64_t n) {
    struct Entry {
        uint64_t n = ~0ull;
        uint32_t p = 0;
    };
    static thread_local Entry cache[64];
    Entry& e = cache[(n ^ (n >> 13) ^ (n >> 29)) & 63];
    if (e.n != n) {
        e.n = n;
        e.p = crc32c::ShiftBytesPoly((size_t)n);
    }
    return e.p;
}

uint32_t fill_batch(SegBatch* b, const Segment* segs, int n, const int* msg_of = nullptr, bool crc = false) {
    memset(b, 0, sizeof(*b));
    b->nseg = n;
    uint32_t c = 0;
    const int m0 = msg_of ? msg_of[0] : 0;
    for (int i = 0; i < n; ++i) {
        b->src[i] = segs[i].src;
        b->dst[i] = segs[i].dst;
        b->len[i] = segs[i].len;
        b->chunk_start[i] = c;
        uint64_t nc = (segs[i].len + kChunkBytes - 1) / kChunkBytes;
        if (nc == 0) nc = 1;  // empty segment still gets a workgroup (writes crc 0)
        c += (uint32_t)nc;
        const int m = msg_of ? msg_of[i] - m0 : i;
        b->msg[i] = (uint8_t)m;
        b->first_of_msg[i] = (uint8_t)(i == 0 || (msg_of ? msg_of[i] != msg_of[i - 1] : true));
        b->msg_len[m] += segs[i].len;
        b->msg_chunks[m] += (uint32_t)nc;
    }
    b->chunk_start[n] = c;
    // bytes after each segment inside its message
    uint64_t after = 0;
    for (int i = n - 1; i >= 0; --i) {
        if (i == n - 1 || b->msg[i] != b->msg[i + 1]) after = 0;
        b->tail[i] = after;
        after += segs[i].len;
    }
    if (crc) {
        for (int i = 0; i < n; ++i) {
            if (b->tail[i]) b->tail_poly[i] = host_shift_poly(b->tail[i]);
            if (b->first_of_msg[i]) {
                const int m = b->msg[i];
                b->msg_init[m] = crc32c::MultModP(host_shift_poly(b->msg_len[m]), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
            }
        }
    }
    return c;
}

void set_done(SegBatch* b, const DoneWord& d) {
    b->done_ctr = d.counter;
    b->done_word = reinterpret_cast<unsigned long long*>(d.word);
    b->done_seq = d.seq;
}

// Split [0, nseg) into launch groups of <= kInlineSegments segments that
// never split a message. Returns false when one message alone is larger.
bool next_group(const int* msg_of, int nseg, int begin, int* end) {
    int e = begin;
    while (e < nseg) {
        int me = e;  // the message starting at e ends at me
        while (me < nseg && msg_of[me] == msg_of[e]) ++me;
        if (me - begin > kInlineSegments) break;
        e = me;
    }
    if (e == begin) return false;
    *end = e;
    return true;
}

}  // namespace

int LaunchCrc32c(const Segment* segs, int nseg, uint32_t* out, hipStream_t s) {
    if (nseg <= 0) return 0;
    if (ensure_tables() != 0) return -1;
    int dev = 0;
    hipGetDevice(&dev);
    uint32_t* scratch = stream_scratch(dev, s);
    if (!scratch) return -1;
    for (int i = 0; i < nseg; i += kInlineSegments) {
        const int n = nseg - i < kInlineSegments ? nseg - i : kInlineSegments;
        SegBatch b;
        const uint32_t chunks = fill_batch(&b, segs + i, n, nullptr, true);
        hipLaunchKernelGGL(crc32c_kernel, dim3(chunks), dim3(kThreads), 0, s, b, g_tables[dev].t8, scratch, out + i);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    return 0;
}

size_t Crc32cScratchBytes(int64_t nseg) { return (size_t)(nseg + 1) * sizeof(uint64_t); }

int LaunchCrc32cSegments(const uint64_t* starts_dev, const uint64_t* lens_dev, int64_t nseg, uint64_t total_bytes,
                         uint64_t max_seg_len, uint32_t* out_dev, void* scratch, hipStream_t s) {
    if (nseg <= 0) return 0;
    const uint32_t* xc = ensure_xc(max_seg_len / kMfmaChunk + 2);
    if (!xc) return -1;
    int dev = 0;
    hipGetDevice(&dev);
    uint64_t* cs = static_cast<uint64_t*>(scratch);
    if (hipMemsetAsync(out_dev, 0, sizeof(uint32_t) * nseg, s) != hipSuccess) return -1;
    hipLaunchKernelGGL(crc_chunk_count_kernel, dim3((uint32_t)((nseg + 255) / 256)), dim3(256), 0, s, lens_dev, nseg, cs);
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(1), dim3(1024), 0, s, cs, (uint64_t)nseg, cs + nseg);
    // every segment has >= 1 chunk; the total is bounded by bytes/64KiB + nseg
    const uint64_t bound = total_bytes / kMfmaChunk + (uint64_t)nseg;
    const uint64_t waves_per_wg = kThreads / 64;
    uint64_t grid = (bound + waves_per_wg - 1) / waves_per_wg;
    if (grid > 256 * 8) grid = 256 * 8;  // persistent: <= 8 workgroups per CU, waves loop over chunks
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL(crc32c_mfma_kernel, dim3((uint32_t)grid), dim3(kThreads), 0, s, starts_dev, lens_dev,
                       (const uint64_t*)cs, nseg, (const CrcMfmaConsts*)g_tables[dev].mfma, xc, out_dev);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// One fused copy + CRC launch of a filled batch: the MFMA kernel (a
// workgroup walks chunks, at most 8 workgroups per CU of the 256) or the
// byte-table kernel (one workgroup per chunk).
static void launch_copy_crc(const SegBatch& b, uint32_t chunks, int dev, uint32_t* scratch, uint32_t* out,
                            hipStream_t s, bool mfma) {
    if (mfma) {
        const uint32_t grid = chunks < 2048u ? chunks : 2048u;
        hipLaunchKernelGGL(copy_crc32c_mfma_kernel, dim3(grid), dim3(kThreads), 0, s, b,
                           (const CrcMfmaConsts*)g_tables[dev].mfma, scratch, out, chunks);
    } else {
        hipLaunchKernelGGL(copy_crc32c_kernel, dim3(chunks), dim3(kThreads), 0, s, b, g_tables[dev].t8, scratch, out);
    }
}

int LaunchBatchedCopyCrc32c(const Segment* segs, int nseg, uint32_t* out, hipStream_t s, bool mfma) {
    if (nseg <= 0) return 0;
    if (ensure_tables() != 0) return -1;
    int dev = 0;
    hipGetDevice(&dev);
    uint32_t* scratch = stream_scratch(dev, s);
    if (!scratch) return -1;
    for (int i = 0; i < nseg; i += kInlineSegments) {
        const int n = nseg - i < kInlineSegments ? nseg - i : kInlineSegments;
        SegBatch b;
        const uint32_t chunks = fill_batch(&b, segs + i, n, nullptr, true);
        launch_copy_crc(b, chunks, dev, scratch, out + i, s, mfma);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    return 0;
}

int LaunchBatchedCopyCrc32cMessages(const Segment* segs, const int* msg_of, int nseg, uint32_t* out, hipStream_t s,
                                    const DoneWord* done, bool mfma) {
    if (nseg <= 0) return 0;
    if (ensure_tables() != 0) return -1;
    int dev = 0;
    hipGetDevice(&dev);
    uint32_t* scratch = stream_scratch(dev, s);
    if (!scratch) return -1;
    for (int i = 0, e = 0; i < nseg; i = e) {
        if (!next_group(msg_of, nseg, i, &e)) return -2;
        SegBatch b;
        const uint32_t chunks = fill_batch(&b, segs + i, e - i, msg_of + i, true);
        if (done && e == nseg) set_done(&b, *done);
        launch_copy_crc(b, chunks, dev, scratch, out + msg_of[i], s, mfma);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    return 0;
}

// A kernel that just takes time: one wave sleeps until the GPU's constant
// wall clock has advanced by `ticks` (bounded: it always exits). Used to
// show that fibers waiting on a long kernel park instead of holding a
// worker pthread.
__global__ void sleep_kernel(uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

__global__ void clock_probe_kernel(unsigned long long* out) {
    if (threadIdx.x == 0) __hip_atomic_store(out, wall_clock64(), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int LaunchClockProbe(uint64_t* out_pinned, hipStream_t s) {
    hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, s, reinterpret_cast<unsigned long long*>(out_pinned));
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int LaunchSleepKernel(uint64_t us, hipStream_t s) {
    int dev = 0, khz = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
    if (us > 10000000) us = 10000000;  // never more than 10 s
    hipLaunchKernelGGL(sleep_kernel, dim3(1), dim3(64), 0, s, (uint64_t)khz * us / 1000);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int LaunchBatchedCopy(const Segment* segs, int nseg, hipStream_t s, const DoneWord* done) {
    for (int i = 0; i < nseg; i += kInlineSegments) {
        const int n = nseg - i < kInlineSegments ? nseg - i : kInlineSegments;
        SegBatch b;
        const uint32_t chunks = fill_batch(&b, segs + i, n);
        if (done && i + n == nseg) set_done(&b, *done);
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

namespace {
// ================================================================ resident copy worker
//
// A launch per batch costs the host ~6-10 us of HIP API time (kernel
// arguments of ~1.6 KB, an event record) and the batch a launch latency;
// at 150k+ batches/s that is a CPU core and a bound on the RPC legs. The
// resident worker instead stays on the GPU and takes batches from a ring in
// pinned host memory: the host writes a SegBatch into a slot and publishes
// its sequence number (one release store); workgroups of the running
// instance claim its chunks through epoch-tagged counters in HBM, copy +
// checksum them with the same code as copy_crc32c_kernel, and the workgroup
// that finishes the last chunk stores the sequence into the slot's done word
// (a system-scope release), which the completion poller reads as plain host
// memory — no launch, no event, no hipEventQuery per batch.
//
// Every instance exits on its own: after `idle_ticks` without a new batch or
// `max_ticks` of life (so other work sharing its hardware queue waits at
// most that long), or when the host sets `stop`. Exit races with a publish
// are closed Dekker-style: a workgroup announces `exiting = instance`, then
// re-reads the next slot (system-scope seq_cst both ways); the host
// publishes, then reads `exiting` and launches a new instance when it names
// the current one. Instances on the ring's stream run one after another;
// workgroups of overlapping lifetimes only ever cooperate through the
// counters. Every loop is bounded.
static_assert(sizeof(SegBatch) % 16 == 0, "SegBatch is staged into LDS in 16 B words");
constexpr int kResidentSlots = 64;

struct alignas(128) ResidentSlot {
    SegBatch batch;
    uint32_t* crc_out;  // per-message CRC32C (pinned host), null: copy only
    uint32_t chunks;
    uint32_t pad;
    uint64_t seq;       // host: published batch number (written last)
    uint64_t pad0[13];
    uint64_t done;      // device: batch number once every chunk is written
    uint64_t pad1[15];
};

struct alignas(128) ResidentCtl {
    uint64_t stop;
    uint64_t pad0[15];
    uint64_t exiting;   // instance whose workgroup is about to exit
    uint64_t pad1[15];
};

__device__ __forceinline__ uint64_t sys_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Epoch-tagged counter (epoch = low 32 bits of the batch number, count in
// the low half): adds `add` for batch k32 and returns the count before, or
// -1 when the counter has moved past k32 or the count would pass `limit`.
__device__ int64_t tagged_add(uint64_t* ctr, uint32_t k32, uint32_t limit, uint32_t add) {
    uint64_t old = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int it = 0; it < 4096; ++it) {
        const uint32_t e = (uint32_t)(old >> 32), c = (uint32_t)old;
        const int32_t d = (int32_t)(e - k32);
        if (d > 0) return -1;                // already a later batch's counter
        const uint32_t cur = d < 0 ? 0 : c;  // an older batch's counter: this batch starts at 0
        if (cur + add > limit) return -1;
        const uint64_t nv = ((uint64_t)k32 << 32) | (uint64_t)(cur + add);
        if (__hip_atomic_compare_exchange_strong(ctr, &old, nv, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
            return cur;
    }
    return -1;
}

// One 16 KiB chunk of a batch held in LDS (the body of copy_crc32c_kernel;
// a null destination checksums only; crc_out null copies only).
__device__ void resident_chunk(const SegBatch& b, uint32_t chunk, const uint32_t (*t)[256], uint32_t* wave_acc,
                               uint32_t* scratch, uint32_t* crc_out) {
    const int seg = find_segment(b, chunk);
    const uint64_t len = b.len[seg];
    const uint8_t* base = static_cast<const uint8_t*>(b.src[seg]);
    uint8_t* dbase = static_cast<uint8_t*>(b.dst[seg]);
    const uint32_t seg_chunks = b.chunk_start[seg + 1] - b.chunk_start[seg];
    const uint32_t k = chunk - b.chunk_start[seg];
    const uint32_t after = seg_chunks - 1 - k;
    const int64_t chunk_end = (int64_t)len - (int64_t)after * (int64_t)kChunkBytes;
    const int64_t lane_end = chunk_end - (int64_t)(kThreads - 1 - threadIdx.x) * kLaneBytes;
    const int64_t lane_beg = lane_end - kLaneBytes;
    const bool want_crc = crc_out != nullptr;
    uint32_t crc = 0;
    if (lane_end > 0) {
        if (lane_beg >= 0) {
            const u32x4_unaligned* p = reinterpret_cast<const u32x4_unaligned*>(base + lane_beg);
            u32x4_unaligned* q = reinterpret_cast<u32x4_unaligned*>(dbase + lane_beg);
            u32x4_unaligned v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = p[i];
            if (dbase) {
#pragma unroll
                for (int i = 0; i < 4; ++i) q[i] = v[i];
            }
            if (want_crc) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    crc = crc_word8(crc, v[i].x, v[i].y, t);
                    crc = crc_word8(crc, v[i].z, v[i].w, t);
                }
            }
        } else {
            for (int64_t i = 0; i < lane_end; ++i) {
                const uint8_t c = base[i];
                if (dbase) dbase[i] = c;
                crc = t[0][(crc ^ c) & 0xff] ^ (crc >> 8);
            }
        }
        if (want_crc) crc = mult_mod_p(c_lane_shift[kThreads - 1 - threadIdx.x], crc);
    }
    if (want_crc) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) crc ^= __shfl_xor(crc, off, 64);
        if ((threadIdx.x & 63) == 0) wave_acc[threadIdx.x >> 6] = crc;
    }
    __syncthreads();
    if (want_crc && threadIdx.x == 0) {
        const uint32_t acc = wave_acc[0] ^ wave_acc[1] ^ wave_acc[2] ^ wave_acc[3];
        fold_chunk(b, seg, after, seg_chunks, acc, scratch, crc_out);
    }
}

__global__ void __launch_bounds__(kThreads) resident_copy_kernel(ResidentSlot* ring, ResidentCtl* ctl,
                                                                 uint64_t* claim, uint64_t* fin,
                                                                 uint32_t* scratch, const uint32_t* tables,
                                                                 uint64_t start_seq, uint64_t instance,
                                                                 uint64_t idle_ticks, uint64_t max_ticks) {
    __shared__ uint32_t t[8][256];
    __shared__ uint32_t wave_acc[kThreads / 64];
    __shared__ __attribute__((aligned(16))) SegBatch sb;
    __shared__ int64_t s_chunk;
    __shared__ int s_state;  // 0 work, 1 exit
    __shared__ uint32_t* s_out;
    __shared__ uint32_t s_chunks;
    {
        const uint4* src = reinterpret_cast<const uint4*>(tables);
        uint4* dst = reinterpret_cast<uint4*>(&t[0][0]);
        dst[threadIdx.x] = src[threadIdx.x];
        dst[threadIdx.x + kThreads] = src[threadIdx.x + kThreads];
    }
    const uint64_t t_start = wall_clock64();
    uint64_t t_idle = t_start;
    uint64_t k = start_seq;
    for (;;) {
        ResidentSlot* slot = &ring[k % kResidentSlots];
        // ---- wait for batch k (thread 0 polls; the group follows)
        if (threadIdx.x == 0) {
            int state = 1;
            for (uint32_t polls = 0;; ++polls) {
                const uint64_t s = sys_load(&slot->seq);
                if (s == k) {
                    state = 0;
                    break;
                }
                if ((int64_t)(s - k) > 0) {  // the slot was reused: batch k is long done (we lagged)
                    state = 2;
                    break;
                }
                if (sys_load(&ctl->stop)) break;
                const uint64_t now = wall_clock64();
                if (now - t_idle > idle_ticks || now - t_start > max_ticks || polls >= (1u << 22)) {
                    __hip_atomic_store(&ctl->exiting, instance, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
                    if (__hip_atomic_load(&slot->seq, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM) == k) {
                        __hip_atomic_store(&ctl->exiting, 0ull, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
                        state = 0;
                    }
                    break;
                }
                __builtin_amdgcn_s_sleep(8);
            }
            s_state = state;
            if (state == 0) {
                s_out = slot->crc_out;
                s_chunks = slot->chunks;
            }
        }
        __syncthreads();
        if (s_state == 1) return;
        if (s_state == 2) {
            ++k;
            __syncthreads();
            continue;
        }
        const uint32_t k32 = (uint32_t)k;
        const uint32_t chunks = s_chunks;
        uint32_t* crc_out = s_out;
        const uint32_t si = (uint32_t)(k % kResidentSlots);
        uint32_t* slot_scratch = scratch + (size_t)si * kInlineSegments * 2;
        // claim before fetching the descriptor: in a small batch most
        // workgroups find nothing left and move on at the cost of one CAS
        if (threadIdx.x == 0) s_chunk = tagged_add(&claim[si], k32, chunks, 1);
        __syncthreads();
        int64_t c = s_chunk;
        __syncthreads();
        if (c >= 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the slot was published before its seq
            {
                const uint4* src = reinterpret_cast<const uint4*>(&slot->batch);
                uint4* dst = reinterpret_cast<uint4*>(&sb);
                constexpr int kWords = (int)(sizeof(SegBatch) / sizeof(uint4));
                for (int i = threadIdx.x; i < kWords; i += kThreads) dst[i] = src[i];
            }
            __syncthreads();
            uint32_t mine = 0;
            for (uint32_t guard = 0; c >= 0 && guard <= chunks; ++guard) {
                resident_chunk(sb, (uint32_t)c, t, wave_acc, slot_scratch, crc_out);
                ++mine;
                if (threadIdx.x == 0) s_chunk = tagged_add(&claim[si], k32, chunks, 1);
                __syncthreads();
                c = s_chunk;
                __syncthreads();
            }
            // one system-scope release for everything this workgroup wrote
            // in the batch (the barrier above ordered every lane's stores)
            if (threadIdx.x == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                const int64_t f = tagged_add(&fin[si], k32, chunks, mine);
                if (f >= 0 && f + mine == chunks)
                    __hip_atomic_store(&slot->done, k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        t_idle = wall_clock64();
        ++k;
    }
}

}  // namespace

// ---- host side of the resident worker
struct ResidentRing {
    int device = -1;
    ResidentSlot* slots = nullptr;  // pinned, coherent
    ResidentCtl* ctl = nullptr;
    uint64_t* claim = nullptr;      // HBM
    uint64_t* fin = nullptr;
    uint32_t* scratch = nullptr;
    hipStream_t stream = nullptr;
    std::mutex mu;
    uint64_t next_seq = 1;
    uint64_t instance = 0;          // last launched instance id
    hipEvent_t last_ev = nullptr;   // recorded after the last launched instance
    uint64_t idle_ticks = 0, max_ticks = 0;
    uint32_t groups = 16;           // workgroups per instance
    std::atomic<int64_t> launches{0}, batches{0}, ring_full_waits{0};
};

namespace {
std::mutex g_resident_mu;
ResidentRing* g_resident[64] = {};

// (re)launch an instance starting at the oldest batch not yet done; mu held
int resident_launch_locked(ResidentRing* r) {
    uint64_t start = r->next_seq;
    for (uint64_t s = r->next_seq > kResidentSlots ? r->next_seq - kResidentSlots : 1; s < r->next_seq; ++s) {
        const ResidentSlot& sl = r->slots[s % kResidentSlots];
        if (__atomic_load_n(&sl.done, __ATOMIC_ACQUIRE) < s) {
            start = s;
            break;
        }
    }
    const uint64_t inst = ++r->instance;
    hipLaunchKernelGGL(resident_copy_kernel, dim3(r->groups), dim3(kThreads), 0, r->stream, r->slots, r->ctl,
                       r->claim, r->fin, r->scratch, g_tables[r->device].t8, start, inst, r->idle_ticks,
                       r->max_ticks);
    if (hipGetLastError() != hipSuccess) return -1;
    if (!r->last_ev && hipEventCreateWithFlags(&r->last_ev, hipEventDisableTiming) != hipSuccess) return -1;
    if (hipEventRecord(r->last_ev, r->stream) != hipSuccess) return -1;
    r->launches.fetch_add(1, std::memory_order_relaxed);
    return 0;
}
}  // namespace

ResidentRing* ResidentRingFor(int device, uint32_t idle_us, uint32_t max_us, uint32_t groups) {
    if (device < 0 || device >= 64) return nullptr;
    std::lock_guard<std::mutex> g(g_resident_mu);
    if (g_resident[device]) return g_resident[device];
    int prev = 0;
    hipGetDevice(&prev);
    if (prev != device) hipSetDevice(device);
    ResidentRing* r = new ResidentRing;
    r->device = device;
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0) khz = 100000;
    r->idle_ticks = (uint64_t)khz * idle_us / 1000;
    r->max_ticks = (uint64_t)khz * max_us / 1000;
    r->groups = groups < 1 ? 1 : (groups > 256 ? 256 : groups);
    bool ok = ensure_tables() == 0 &&
              hipHostMalloc(reinterpret_cast<void**>(&r->slots), sizeof(ResidentSlot) * kResidentSlots,
                            hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess &&
              hipHostMalloc(reinterpret_cast<void**>(&r->ctl), sizeof(ResidentCtl),
                            hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&r->claim), sizeof(uint64_t) * kResidentSlots) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&r->fin), sizeof(uint64_t) * kResidentSlots) == hipSuccess &&
              hipMalloc(reinterpret_cast<void**>(&r->scratch),
                        sizeof(uint32_t) * 2 * kInlineSegments * kResidentSlots) == hipSuccess &&
              hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) == hipSuccess;
    if (ok) {
        memset(r->slots, 0, sizeof(ResidentSlot) * kResidentSlots);
        memset(r->ctl, 0, sizeof(ResidentCtl));
        ok = hipMemset(r->claim, 0, sizeof(uint64_t) * kResidentSlots) == hipSuccess &&
             hipMemset(r->fin, 0, sizeof(uint64_t) * kResidentSlots) == hipSuccess &&
             hipMemset(r->scratch, 0, sizeof(uint32_t) * 2 * kInlineSegments * kResidentSlots) == hipSuccess &&
             hipDeviceSynchronize() == hipSuccess;
    }
    if (prev != device) hipSetDevice(prev);
    if (!ok) return nullptr;  // leaks the partial ring; the engine falls back to launches
    g_resident[device] = r;
    return r;
}

int ResidentSubmit(ResidentRing* r, const Segment* segs, const int* msg_of, int nseg, uint32_t* crc_out,
                   uint64_t* first_seq, uint64_t* last_seq) {
    if (nseg <= 0) return -1;
    std::lock_guard<std::mutex> g(r->mu);
    *first_seq = r->next_seq;
    for (int i = 0, e = 0; i < nseg; i = e) {
        if (msg_of) {
            if (!next_group(msg_of, nseg, i, &e)) return -2;
        } else {
            e = nseg - i < kInlineSegments ? nseg : i + kInlineSegments;
        }
        const uint64_t k = r->next_seq;
        ResidentSlot& sl = r->slots[k % kResidentSlots];
        // the slot is free once its previous batch (k - slots) is done
        if (k > kResidentSlots) {
            const uint64_t need = k - kResidentSlots;
            for (int spins = 0; __atomic_load_n(&sl.done, __ATOMIC_ACQUIRE) < need; ++spins) {
                if (spins == 0) r->ring_full_waits.fetch_add(1, std::memory_order_relaxed);
                if (spins > 2000000) return -1;  // ~seconds: the device stopped consuming
                if ((spins & 1023) == 1023 && hipEventQuery(r->last_ev) == hipSuccess &&
                    resident_launch_locked(r) != 0)
                    return -1;
                __builtin_ia32_pause();
            }
        }
        SegBatch b;
        const uint32_t chunks = fill_batch(&b, segs + i, e - i, msg_of ? msg_of + i : nullptr, crc_out != nullptr);
        memcpy(&sl.batch, &b, sizeof(b));
        sl.crc_out = crc_out ? crc_out + (msg_of ? msg_of[i] : i) : nullptr;
        sl.chunks = chunks;
        __atomic_store_n(&sl.seq, k, __ATOMIC_RELEASE);
        r->next_seq = k + 1;
        r->batches.fetch_add(1, std::memory_order_relaxed);
    }
    *last_seq = r->next_seq - 1;
    // Dekker with the instances' exit path: publish (above), full fence,
    // then look whether the current instance announced its exit
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    const uint64_t exiting = __atomic_load_n(&r->ctl->exiting, __ATOMIC_SEQ_CST);
    if (r->instance == 0 || exiting == r->instance) return resident_launch_locked(r);
    return 0;
}

bool ResidentDone(ResidentRing* r, uint64_t first_seq, uint64_t last_seq) {
    for (uint64_t s = first_seq; s <= last_seq; ++s) {
        if (__atomic_load_n(&r->slots[s % kResidentSlots].done, __ATOMIC_ACQUIRE) < s) return false;
    }
    return true;
}

void ResidentKick(ResidentRing* r) {
    std::lock_guard<std::mutex> g(r->mu);
    if (r->last_ev && hipEventQuery(r->last_ev) != hipSuccess) return;  // an instance is still on the device
    // nothing running: start one if a published batch is not done
    for (uint64_t s = r->next_seq > kResidentSlots ? r->next_seq - kResidentSlots : 1; s < r->next_seq; ++s) {
        if (__atomic_load_n(&r->slots[s % kResidentSlots].done, __ATOMIC_ACQUIRE) < s) {
            resident_launch_locked(r);
            return;
        }
    }
}

void ResidentShutdown() {
    std::lock_guard<std::mutex> g(g_resident_mu);
    for (ResidentRing* r : g_resident) {
        if (!r) continue;
        __atomic_store_n(&r->ctl->stop, 1ull, __ATOMIC_SEQ_CST);
        hipStreamSynchronize(r->stream);  // every instance exits within its idle bound
    }
}

ResidentStats GetResidentStats() {
    ResidentStats s;
    std::lock_guard<std::mutex> g(g_resident_mu);
    for (ResidentRing* r : g_resident) {
        if (!r) continue;
        s.launches += r->launches.load(std::memory_order_relaxed);
        s.batches += r->batches.load(std::memory_order_relaxed);
        s.ring_full_waits += r->ring_full_waits.load(std::memory_order_relaxed);
    }
    return s;
}

}  // namespace gpu
}  // namespace mrpc
