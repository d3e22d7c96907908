// Batched snappy compression and decompression on CDNA4 (gfx950) — the
// device half of the snappy body codec (reference: policy/snappy_compress.cpp
// :28-64 over butil/third_party/snappy; SURVEY K3 "per-64 KB-block CTA
// kernel").
//
// Framing: every job is an independent raw snappy stream whose uncompressed
// size is <= kSnappyMaxBlock (64 KiB). Job tables live in device memory, so
// one launch covers any number of blocks; one wave64 workgroup owns a block.
//
// Decompression rebuilds the block in LDS (sized per launch to the largest
// block, so 32 KiB blocks run 5 waves per CU instead of 2) and streams it to
// HBM with 16-byte stores. The tag stream is serial, so the whole wave walks
// it in lockstep, but never through memory latency: a 256-byte window of
// the compressed stream sits in VGPRs (4 bytes per lane, one coalesced load
// per refill) and tag bytes are pulled out with v_readlane (uniform index),
// short literals with ds_bpermute. Each element is then materialised by all
// 64 lanes at once:
//   literal          out[pos + j] = in[src + j]                  (window or HBM)
//   copy, off >= len out[pos + j] = out[pos - off + j]
//   copy, off <  len out[pos + j] = out[pos - off + (j % off)]    (the repeating
//                    pattern already exists, so an overlapping copy is one
//                    parallel step, not a byte loop)
// LDS instructions of one wave execute in order, so consecutive elements
// need no wait between them.
//
// Compression first stages the block in LDS (coalesced 16-byte loads), so
// the lanes' serial match loops probe LDS instead of waiting on HBM for
// every position, then splits it into 64 contiguous segments, one per lane; each
// lane runs a greedy hash matcher with snappy's skip heuristic over
// incompressible runs and emits literal / copy elements into its own scratch
// slot. Candidates come from two LDS tables: a 128-entry u16 table per lane
// (the most recent position in its own segment: short offsets, copy-1 form)
// and a block-wide 4096-entry table holding the EARLIEST position of every
// hash, filled by all lanes with ds_min before matching starts — the
// earliest occurrence of a 4-byte hash precedes every later one, so it is a
// legal source for any lane, which gives matches across segments without
// ordering the lanes. Matches never cross a segment end, so the
// concatenation of the 64 slots (placed by a prefix sum behind the varint
// header, copied out coalesced) is a valid snappy stream any decoder
// accepts; its size lands within ~10% of the CPU codec's on repetitive
// data. Blocks up to 16 KiB also keep the output slots in LDS (a lane's
// output never exceeds its segment plus one literal header); 4 KiB blocks
// take 42 KiB of LDS per wave, 3 waves per CU. (A/B on the MI355X: 32-bit
// (position, fingerprint) entries that skip most verification loads ran
// slower — 48 KiB/wave drops to 3 waves per CU; a double-buffered window
// prefetch in the decompressor also lost to the single re-centred window.)
#include <hip/hip_runtime.h>

#include <algorithm>

#include "base/flags.h"
#include "gpu/device_pb.h"
#include "gpu/kernels.h"

namespace mrpc {
namespace gpu {

namespace {

// Length of a literal with nb (1..4) extra length bytes in `ext`. The
// stored value is length - 1: 0xFFFFFFFF (a 4 GiB literal) would wrap to 0
// in 32 bits and pass as an empty literal, so it saturates instead and fails
// every bound check like any other literal longer than its piece.
__device__ __forceinline__ uint32_t lit_len(uint32_t ext, uint32_t nb) {
    const uint32_t raw = ext & (0xFFFFFFFFu >> (32 - 8 * nb));
    return raw == 0xFFFFFFFFu ? raw : raw + 1;
}


constexpr int kWave = 64;
constexpr uint32_t kWindow = 256;  // bytes of compressed stream held in VGPRs

// Job pointers come from a device table, so the compiler cannot prove they
// are global; say so, or every access becomes a flat op that also ties up
// the LDS counter.
typedef const __attribute__((address_space(1))) uint8_t gbyte_c;
typedef __attribute__((address_space(1))) uint8_t gbyte;
__device__ __forceinline__ gbyte_c* as_global(const void* p) { return (gbyte_c*)p; }
__device__ __forceinline__ gbyte* as_global(void* p) { return (gbyte*)p; }
typedef uint32_t __attribute__((aligned(1))) u32_unaligned;
__device__ __forceinline__ uint32_t load32(gbyte_c* p) {
    return *reinterpret_cast<const __attribute__((address_space(1))) u32_unaligned*>(p);
}

// 4 bytes per lane of the stream starting at 4-byte-aligned `wbase` (relative
// to `in`); bytes outside [0, in_len) read as 0 and are never consumed.
typedef __attribute__((address_space(3))) uint8_t lbyte;

__device__ __forceinline__ uint32_t load_window(gbyte_c* in, uint32_t in_len, uint32_t wbase, int lane) {
    const uint32_t pos = wbase + 4u * (uint32_t)lane;
    if (pos + 4 <= in_len) return load32(in + pos);
    uint32_t v = 0;
    for (uint32_t k = 0; k < 4; ++k) {
        if (pos + k < in_len) v |= (uint32_t)in[pos + k] << (8 * k);
    }
    return v;
}

__device__ __forceinline__ uint32_t window_byte(uint32_t win, uint32_t q) {
    const uint32_t d = (uint32_t)__builtin_amdgcn_readlane((int)win, (int)(q >> 2));
    return (d >> ((q & 3) * 8)) & 0xff;
}

// Decodes the elements of in[ip, in_len) into LDS buf[0, ulen) and streams
// the result to dst; `win` holds the window at `wbase`. Returns 0 or a code.
__device__ __forceinline__ int decode_elements(gbyte_c* in, uint32_t in_len, uint32_t ip, uint32_t wbase,
                                               uint32_t win, uint32_t ulen, uint8_t* buf, void* dstp, int lane) {
    int bad = 0;
    uint32_t op = 0;
    while (!bad && ip < in_len) {
        if (ip + 5 > wbase + kWindow) {  // tag + up to 4 extra bytes must be in the window
            wbase = ip & ~3u;
            win = load_window(in, in_len, wbase, lane);
        }
        // The tag and the 4 bytes after it in one go: two dword readlanes and
        // a 64-bit shift (ip + 5 <= wbase + 256 keeps both dwords in range).
        const uint32_t q = ip - wbase;
        const uint32_t dlo = (uint32_t)__builtin_amdgcn_readlane((int)win, (int)(q >> 2));
        const uint32_t dhi = (uint32_t)__builtin_amdgcn_readlane((int)win, (int)(q >> 2) + 1);
        const uint64_t x = ((((uint64_t)dhi) << 32) | dlo) >> ((q & 3) * 8);
        const uint32_t tag = (uint32_t)x & 0xff;
        const uint32_t ext = (uint32_t)(x >> 8);  // next 4 bytes, little endian
        ++ip;
        const uint32_t kind = tag & 3;
        if (kind == 0) {
            uint32_t len = (tag >> 2) + 1;
            if (len > 60) {
                const uint32_t nb = len - 60;  // 1..4 little-endian length bytes
                if (ip + nb > in_len) {
                    bad = 3;
                    break;
                }
                len = lit_len(ext, nb);
                ip += nb;
            }
            if (len > in_len - ip || len > ulen - op) {
                bad = 4;
                break;
            }
            if (ip + len <= wbase + kWindow) {
                // short literal: lanes gather bytes from the VGPR window
                for (uint32_t j0 = 0; j0 < len; j0 += kWave) {
                    const uint32_t j = j0 + (uint32_t)lane;
                    const uint32_t qq = ip - wbase + j;
                    const uint32_t d = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((qq >> 2) & 63) << 2, (int)win);
                    if (j < len) buf[op + j] = (uint8_t)(d >> ((qq & 3) * 8));
                }
            } else {
                for (uint32_t j = lane; j < len; j += kWave) buf[op + j] = in[ip + j];
            }
            ip += len;
            op += len;
        } else {
            uint32_t len, off, need;
            if (kind == 1) {
                len = ((tag >> 2) & 7) + 4;
                off = ((tag >> 5) << 8) | (ext & 0xff);
                need = 1;
            } else if (kind == 2) {
                len = (tag >> 2) + 1;
                off = ext & 0xffff;
                need = 2;
            } else {
                len = (tag >> 2) + 1;
                off = ext;
                need = 4;
            }
            ip += need;
            // one unsigned compare covers off == 0 and off > op
            if (ip > in_len || off - 1 >= op || len > ulen - op) {
                bad = 6;
                break;
            }
            const uint32_t from = op - off;
            if (len <= (uint32_t)kWave && off >= len) {
                if ((uint32_t)lane < len) buf[op + lane] = buf[from + lane];  // the common case: one step
            } else if (off >= len) {
                for (uint32_t j = lane; j < len; j += kWave) buf[op + j] = buf[from + j];
            } else {
                for (uint32_t j = lane; j < len; j += kWave) buf[op + j] = buf[from + j % off];
            }
            op += len;
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (!bad && op != ulen) bad = 7;
    if (bad) return bad;
    __syncthreads();
    // LDS -> HBM, 16 B per lane per step (1 KiB per wave instruction)
    gbyte* dst = as_global(dstp);
    const bool aligned = ((uintptr_t)dstp & 15) == 0;
    const uint32_t vec_end = aligned ? (ulen & ~15u) : 0;
    for (uint32_t o = lane * 16; o < vec_end; o += kWave * 16) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<__attribute__((address_space(1))) u32x4*>(dst + o) = *reinterpret_cast<const u32x4*>(buf + o);
    }
    for (uint32_t o = vec_end + lane; o < ulen; o += kWave) dst[o] = buf[o];
    return 0;
}

__global__ void __launch_bounds__(kWave) snappy_decompress_kernel(const SnappyJob* __restrict__ jobs, int n,
                                                                  uint32_t lds_cap, uint32_t* __restrict__ out_len,
                                                                  int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint8_t buf[];
    const int blk = blockIdx.x;
    if (blk >= n) return;
    const int lane = threadIdx.x;
    const SnappyJob job = jobs[blk];
    gbyte_c* in = as_global(job.src);
    const uint32_t in_len = (uint32_t)job.src_len;
    uint32_t win = load_window(in, in_len, 0, lane);
    // uncompressed length (varint, <= 5 bytes; all inside the first window)
    uint32_t ulen = 0, ip = 0;
    int bad = 0;
    for (int shift = 0;; shift += 7) {
        if (ip >= in_len || shift >= 35) {
            bad = 1;
            break;
        }
        const uint32_t c = window_byte(win, ip++);
        ulen |= (c & 0x7f) << shift;
        if (!(c & 0x80)) break;
    }
    if (!bad && (ulen > lds_cap || ulen > job.dst_cap)) bad = 2;
    if (!bad) bad = decode_elements(in, in_len, ip, 0, win, ulen, buf, job.dst, lane);
    if (lane == 0) {
        err[blk] = bad;
        out_len[blk] = bad ? 0 : ulen;
    }
}

// Headerless pieces cut by snappy_split_kernel; this launch takes the ones
// with lo < ulen <= hi (hi = its LDS per wave).
__global__ void __launch_bounds__(kWave) snappy_decompress_pieces_kernel(const SnappyPiece* __restrict__ pieces,
                                                                         int n, uint32_t lo, uint32_t hi,
                                                                         int* __restrict__ err) {
    extern __shared__ __attribute__((aligned(16))) uint8_t buf[];
    const int blk = blockIdx.x;
    if (blk >= n) return;
    const int lane = threadIdx.x;
    const SnappyPiece pc = pieces[blk];
    if (pc.ulen == 0) {
        if (lo == 0 && lane == 0) err[blk] = 0;
        return;
    }
    if (pc.ulen <= lo || pc.ulen > hi) return;
    // a piece starts anywhere in its stream: walk it from the dword below,
    // so every window load is an aligned dword per lane
    const uint32_t mis = (uint32_t)((uintptr_t)pc.src & 3);
    gbyte_c* in = as_global(static_cast<const uint8_t*>(pc.src) - mis);
    const uint32_t in_len = pc.src_len + mis;
    const uint32_t win = load_window(in, in_len, 0, lane);
    const int bad = decode_elements(in, in_len, mis, 0, win, pc.ulen, buf, pc.dst, lane);
    if (lane == 0) err[blk] = bad;
}

// ------------------------------------------------- parallel piece decoder
// Pieces of up to kParMax bytes (the RPC path's 4 KiB device-encoded
// pieces) decode in three data-parallel phases instead of one element per
// wave step (the serial decoder above spends ~470 cycles per element on
// text: every element is a wave-uniform branch tree plus an LDS round trip,
// 117 us for 4 KiB pieces of log records, benchmarks/snappy_rpc_shapes.py):
//  1. parse: the compressed piece is staged in LDS with 16-byte loads; lane j
//     parses the element header at ip + j speculatively, the true element
//     starts are found by one v_readlane hop each, and a wave prefix sum
//     gives every element its output position. Each element then writes,
//     for every output byte it produces, WHERE that byte comes from: a
//     literal byte of the input (flag bit set) or an earlier output position
//     (copies) — a source map of u16 entries in LDS;
//  2. resolve: pointer jumping over the map (src[p] = src[src[p]] until every
//     entry names a literal byte) — log2(chain depth) rounds of fully
//     parallel LDS work, overlapping copies included;
//  3. gather: out[p] = input[src[p]], 8 bytes per lane per step, stored
//     straight to the destination (HBM or pinned host memory).
constexpr uint32_t kParMax = 8192;
constexpr uint16_t kLitFlag = 0x8000;

// Wave64 inclusive prefix sum / max on DPP (row_shr 1,2,4,8 inside rows of
// 16, then row_bcast:15 and row_bcast:31 across rows): VALU modifiers, no
// LDS round trip per step as with __shfl_up (ds_bpermute).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
    return v;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// OR of a 64-bit value over the wave (DPP inclusive scan of each half, lane
// 63's result)
__device__ __forceinline__ uint64_t wave_or64(uint64_t x) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
#define MRPC_OR_STEP(ctrl, rm)                                                  \
    lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, ctrl, rm, 0xf, false); \
    hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, ctrl, rm, 0xf, false);
    MRPC_OR_STEP(0x111, 0xf)
    MRPC_OR_STEP(0x112, 0xf)
    MRPC_OR_STEP(0x114, 0xf)
    MRPC_OR_STEP(0x118, 0xf)
    MRPC_OR_STEP(0x142, 0xa)
    MRPC_OR_STEP(0x143, 0xc)
#undef MRPC_OR_STEP
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, 63) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 63) << 32);
}

// Phase stamps (shader clock) of block 0, for benchmarks/snappy_rpc_shapes.py
__device__ __forceinline__ void stamp(uint64_t* stamps, int blk, int lane, int i) {
    if (stamps && blk == 0 && lane == 0) stamps[i] = __builtin_amdgcn_s_memtime();
}

// One piece per wave; the body of snappy_decompress_pieces_par_kernel and of
// the decode role of codec_waves_kernel (every exit is wave-uniform).
__device__ __forceinline__ void decode_piece_wave(const SnappyPiece* __restrict__ pieces, int blk, uint32_t lo,
                                                  uint32_t hi, uint32_t cin_cap, int* __restrict__ err,
                                                  uint64_t* __restrict__ stamps) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x;
    const SnappyPiece pc = pieces[blk];
    if (pc.ulen == 0) {
        if (lo == 0 && lane == 0) err[blk] = 0;
        return;
    }
    if (pc.ulen <= lo || pc.ulen > hi) return;
    const uint32_t ulen = pc.ulen;
    stamp(stamps, blk, lane, 0);
    // Incompressible pieces (one long literal, 1.14:1 or worse) and very
    // compressible ones (a few long copies, 8:1 or better) decode faster one
    // element per wave step: the source map costs one pass per 64 output
    // bytes and the resolve one round per doubling of the copy-chain depth,
    // whatever the element count (MI355X, 4 KiB pieces: random 18 vs 3.5 us,
    // one repeated byte 41 vs 22 us per launch of 112; text stays here).
    if ((uint64_t)pc.src_len * 8 >= (uint64_t)ulen * 7 || (uint64_t)pc.src_len * 8 <= ulen) {
        const uint32_t mis4 = (uint32_t)((uintptr_t)pc.src & 3);
        gbyte_c* in4 = as_global(static_cast<const uint8_t*>(pc.src) - mis4);
        const uint32_t in_len = pc.src_len + mis4;
        const uint32_t win = load_window(in4, in_len, 0, lane);
        const int bad = decode_elements(in4, in_len, mis4, 0, win, ulen, lds, pc.dst, lane);
        if (lane == 0) err[blk] = bad;
        return;
    }
    // stage: the piece from the 16-byte boundary below it (a 16-byte
    // aligned chunk never crosses a page, so reading its unused head and
    // tail stays inside mapped memory)
    const uint32_t mis = (uint32_t)((uintptr_t)pc.src & 15);
    const uint32_t end = mis + pc.src_len;  // input is cin[mis, end)
    if (end + 8 > cin_cap) {
        if (lane == 0) err[blk] = 9;  // more compressed bytes than a valid piece can have: host codec
        return;
    }
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    lbyte* const cin = (lbyte*)lds;
    __attribute__((address_space(3))) uint16_t* const smap =
        (__attribute__((address_space(3))) uint16_t*)(lds + cin_cap);
    // a bit per output position: an element starts there (256 words, up
    // to kParMax positions), after the map
    __attribute__((address_space(3))) uint32_t* const starts =
        (__attribute__((address_space(3))) uint32_t*)(lds + cin_cap + 2 * ((hi + 7) & ~7u));
    {
        gbyte_c* g = as_global(static_cast<const uint8_t*>(pc.src) - mis);
        for (uint32_t o = lane * 16; o < end; o += kWave * 16)
            *reinterpret_cast<__attribute__((address_space(3))) u32x4*>(cin + o) =
                *reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(g + o);
        for (uint32_t i = lane; i < (ulen + 31) / 32; i += kWave) starts[i] = 0;
    }
    __syncthreads();
    stamp(stamps, blk, lane, 1);
    const __attribute__((address_space(3))) uint32_t* cin32 = (const __attribute__((address_space(3))) uint32_t*)cin;
    // ---- 1. parse + source map
    uint32_t ip = mis, upos = 0;
    int bad = 0;
    uint64_t t_dec = 0, t_chain = 0, t_iter = 0;  // phase stamps only
    while (ip < end) {
        const uint64_t ta = stamps ? __builtin_amdgcn_s_memtime() : 0;
        const uint32_t q = ip + (uint32_t)lane;
        const uint32_t w = q >> 2;
        const uint64_t x = ((((uint64_t)cin32[w + 1]) << 32) | cin32[w]) >> ((q & 3) * 8);
        const uint32_t tag = (uint32_t)x & 0xff;
        const uint32_t ext = (uint32_t)(x >> 8);
        const uint32_t kind = tag & 3;
        uint32_t len, off = 0, hdr;
        if (kind == 0) {
            len = (tag >> 2) + 1;
            hdr = 1;
            if (len > 60) {
                const uint32_t nb = len - 60;
                len = lit_len(ext, nb);
                hdr += nb;
            }
        } else if (kind == 1) {
            len = ((tag >> 2) & 7) + 4;
            off = ((tag >> 5) << 8) | (ext & 0xff);
            hdr = 2;
        } else {
            len = (tag >> 2) + 1;
            off = kind == 2 ? (ext & 0xffff) : ext;
            hdr = kind == 2 ? 3 : 5;
        }
        const uint64_t csize = (uint64_t)hdr + (kind == 0 ? len : 0);
        const uint32_t step = (uint32_t)min(csize, (uint64_t)0x7FFFFFFF);
        const uint64_t tb = stamps ? __builtin_amdgcn_s_memtime() : 0;
        // the element chain in hops of four elements: n1..n4 = the start 1..4
        // elements after a lane's position (sticky at the first start past
        // the window), two bpermute rounds, then one readlane per four
        // elements; the hop points' next three starts are OR-reduced into the
        // mask. (One dependent readlane per element was ~60 cycles each: a
        // third of a 2 KiB text piece's parse.)
        const uint32_t lim = min((uint32_t)kWave, end - ip);
        const uint32_t n1 = (uint32_t)lane + step;
        auto pull = [&](uint32_t via, uint32_t val) -> uint32_t {
            const uint32_t got = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((via < lim ? via : 0u) << 2), (int)val);
            return via < lim ? got : via;
        };
        const uint32_t n2 = pull(n1, n1);
        const uint32_t n3 = pull(n2, n1);
        const uint32_t n4 = pull(n2, n2);
        uint64_t hops = 0;
        uint32_t p = 0;
        while (p < lim) {
            hops |= 1ull << p;
            p = (uint32_t)__builtin_amdgcn_readlane((int)n4, (int)p);
        }
        uint64_t bits = 0;
        if ((hops >> lane) & 1) {
            bits = (1ull << lane) | (n1 < lim ? 1ull << n1 : 0ull) | (n2 < lim ? 1ull << n2 : 0ull) |
                   (n3 < lim ? 1ull << n3 : 0ull);
        }
        const uint64_t mask = wave_or64(bits);
        const uint64_t tc = stamps ? __builtin_amdgcn_s_memtime() : 0;
        const bool marked = (mask >> lane) & 1;
        const uint32_t u0 = upos + wave_incl_sum(marked ? len : 0) - (marked ? len : 0);
        int e = 0;
        if (marked) {
            if ((uint64_t)q + csize > end) e = 3;                 // truncated
            else if ((uint64_t)u0 + len > ulen) e = 4;            // past the piece
            else if (kind != 0 && (off == 0 || off > u0)) e = 6;  // before the piece
        }
        const uint64_t eb = __ballot(e != 0);
        if (eb) {
            bad = __builtin_amdgcn_readlane(e, (int)__builtin_ctzll(eb));
            break;
        }
        // the element's source at its first output byte, and its start bit;
        // the source map is filled in one pass after the parse
        const uint32_t base = kind == 0 ? (kLitFlag | (q + hdr)) : (u0 - off);
        if (marked) {
            smap[u0] = (uint16_t)base;
            atomicOr((unsigned int*)(starts + (u0 >> 5)), 1u << (u0 & 31));
        }
        const uint32_t span_end =
            (uint32_t)__builtin_amdgcn_readlane((int)(u0 + len), (int)(63 - __builtin_clzll(mask)));
        upos = span_end;
        ip += p;
        if (stamps) {
            t_dec += tb - ta;
            t_chain += tc - tb;
            t_iter += 1;
        }
    }
    if (stamps && blk == 0 && lane == 0) {
        stamps[5] = t_dec;
        stamps[6] = t_chain;
        stamps[9] = t_iter;
    }
    if (!bad && (ip != end || upos != ulen)) bad = 7;
    if (bad) {
        if (lane == 0) err[blk] = bad;
        return;
    }
    __syncthreads();
    // source map, four consecutive positions per lane, 256 per pass: a
    // position's element is the latest start at or before it (the lane's own
    // start bits, then a DPP max-scan over the lanes before it and the carry
    // from the previous pass), its source the element's first-byte source
    // plus the distance (start entries keep their value, so the pass reads
    // and rewrites the map in place). One pass per 256 output bytes over the
    // whole piece; it was one per parse iteration (~150 bytes each) with a
    // scatter, a barrier and two bpermute round trips.
    {
        const uint64_t tf = stamps ? __builtin_amdgcn_s_memtime() : 0;
        uint32_t carry = 0;
        for (uint32_t P = 0; P < ulen; P += 4 * kWave) {
            const uint32_t pos = P + 4u * (uint32_t)lane;
            const uint32_t bits = pos < ulen ? (starts[pos >> 5] >> (pos & 31)) & 0xFu : 0u;
            uint32_t l[4];
            l[0] = (bits & 1) ? pos + 1 : 0u;
            l[1] = (bits & 2) ? pos + 2 : l[0];
            l[2] = (bits & 4) ? pos + 3 : l[1];
            l[3] = (bits & 8) ? pos + 4 : l[2];
            const uint32_t incl = wave_incl_max(l[3]);
            const uint32_t before =
                max(carry, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x138, 0xf, 0xf, false));
            uint32_t u[4], b[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) u[k] = max(before, l[k]) - 1;  // position 0 always starts an element
#pragma unroll
            for (int k = 0; k < 4; ++k) b[k] = smap[u[k]];
#pragma unroll
            for (int k = 0; k < 4; ++k) b[k] = (b[k] + (pos + (uint32_t)k - u[k])) & 0xffff;
            if (pos + 4 <= ulen) {
                typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                u32x2 v;
                v[0] = b[0] | (b[1] << 16);
                v[1] = b[2] | (b[3] << 16);
                *reinterpret_cast<__attribute__((address_space(3))) u32x2*>(smap + pos) = v;
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (pos + (uint32_t)k < ulen) smap[pos + k] = (uint16_t)b[k];
            }
            carry = max(carry, (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1));
        }
        if (stamps && blk == 0 && lane == 0) stamps[7] = __builtin_amdgcn_s_memtime() - tf;
    }
    __syncthreads();
    stamp(stamps, blk, lane, 2);
    // ---- 2. resolve: pointer jumping until every entry is a literal byte;
    // 8 entries per lane per step: one 16-byte read, up to 8 independent
    // reads of their sources, one 16-byte write
    for (int round = 0;; ++round) {
        bool more = false;
        for (uint32_t o = lane * 8; o < ulen; o += kWave * 8) {
            u32x4 m = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(smap + o);
            // branch-free: every lane issues its 8 reads back to back (a
            // resolved entry re-reads entry 0, and keeps its value)
            uint32_t e[8], r[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) e[k] = (m[k >> 1] >> (16 * (k & 1))) & 0xffff;
#pragma unroll
            for (int k = 0; k < 8; ++k) r[k] = smap[(e[k] & kLitFlag) ? 0u : e[k]];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const bool copy = !(e[k] & kLitFlag) && o + k < ulen;
                r[k] = copy ? r[k] : e[k];
                more |= copy && !(r[k] & kLitFlag);
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) m[k] = r[2 * k] | (r[2 * k + 1] << 16);
            *reinterpret_cast<__attribute__((address_space(3))) u32x4*>(smap + o) = m;
        }
        if (!__ballot(more)) break;
        if (round > 16) {  // cannot happen for a valid piece (depth <= ulen)
            if (lane == 0) err[blk] = 10;
            return;
        }
    }
    __syncthreads();
    stamp(stamps, blk, lane, 3);
    // ---- 3. gather + store, 8 bytes per lane per step
    gbyte* dst = as_global(pc.dst);
    const bool aligned8 = ((uintptr_t)pc.dst & 7) == 0;
    const uint32_t vec_end = aligned8 ? (ulen & ~7u) : 0;
    for (uint32_t o = lane * 8; o < vec_end; o += kWave * 8) {
        const u32x4 m = *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(smap + o);
        uint32_t lo32 = 0, hi32 = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t pair = m[k];
            const uint32_t b0 = cin[pair & 0x7fff], b1 = cin[(pair >> 16) & 0x7fff];
            if (k < 2) lo32 |= (b0 | (b1 << 8)) << (16 * k);
            else hi32 |= (b0 | (b1 << 8)) << (16 * (k - 2));
        }
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        u32x2 val;
        val[0] = lo32;
        val[1] = hi32;
        *reinterpret_cast<__attribute__((address_space(1))) u32x2*>(dst + o) = val;
    }
    for (uint32_t o = vec_end + lane; o < ulen; o += kWave) dst[o] = cin[smap[o] & 0x7fff];
    stamp(stamps, blk, lane, 4);
    if (lane == 0) err[blk] = 0;
}

__global__ void __launch_bounds__(kWave) snappy_decompress_pieces_par_kernel(const SnappyPiece* __restrict__ pieces,
                                                                             int n, uint32_t lo, uint32_t hi,
                                                                             uint32_t cin_cap,
                                                                             int* __restrict__ err,
                                                                             uint64_t* __restrict__ stamps) {
    if ((int)blockIdx.x >= n) return;
    decode_piece_wave(pieces, (int)blockIdx.x, lo, hi, cin_cap, err, stamps);
}

// One wave per whole stream, cut at exact multiples of the piece limit: a
// fragmenting encoder (ours at -gpu_snappy_block_kb, CPU encoders at 64 KiB)
// never lets an element span such a multiple or a copy reach back across
// one, so every multiple is an element start and the pieces between them
// decode independently. Both limits (piece_limit and 64 KiB) are checked in
// the same walk.
//
// The walk is parallel where it can be: with `ip` at an element start, lane
// j speculatively parses the element header at ip + j (bytes from a 256 B
// VGPR window via ds_bpermute). Only the chain ip -> ip + size(ip) -> ... is
// serial, and each step is one v_readlane of the precomputed sizes. Marked
// lanes (the true element starts) then get their output position from a
// wave prefix sum and run every check at once: truncation, offsets before
// the stream, lengths past the declared size, elements spanning a cut,
// copies reaching before their piece. Piece starts go to LDS; the slots are
// written at the end.
constexpr int kSplitMaxSmall = 4096;  // pieces at piece_limit (16 MiB at 4 KiB)
constexpr int kSplitMaxBig = 1024;    // 64 KiB pieces (64 MiB)
__global__ void __launch_bounds__(kWave) snappy_split_kernel(const SnappyStream* __restrict__ streams, int n,
                                                             uint32_t piece_limit, SnappyPiece* __restrict__ pieces,
                                                             int* __restrict__ stream_err) {
    __shared__ uint32_t starts_small[kSplitMaxSmall];
    __shared__ uint32_t starts_big[kSplitMaxBig];
    const int sid = blockIdx.x;
    if (sid >= n) return;
    const int lane = threadIdx.x;
    const SnappyStream st = streams[sid];
    gbyte_c* in = as_global(st.src);
    const uint32_t in_len = st.src_len;
    SnappyPiece* const slots = pieces + st.first;
    const uint32_t L0 = min(max(piece_limit, 1u), kSnappyMaxBlock), L1 = kSnappyMaxBlock;
    uint32_t wbase = 0;
    uint32_t win = load_window(in, in_len, 0, lane);
    uint32_t total = 0, ip = 0;
    int bad = 0;
    for (int shift = 0;; shift += 7) {
        if (ip >= in_len || shift >= 35) {
            bad = 1;
            break;
        }
        const uint32_t c = window_byte(win, ip++);
        total |= (c & 0x7f) << shift;
        if (!(c & 0x80)) break;
    }
    if (!bad && total > st.dst_cap) bad = 2;
    const uint32_t np0 = (total + L0 - 1) / L0, np1 = (total + L1 - 1) / L1;
    int cut0 = np0 > (uint32_t)kSplitMaxSmall || np0 > st.max_pieces;  // this limit cannot be used
    int cut1 = np1 > (uint32_t)kSplitMaxBig || np1 > st.max_pieces;
    uint64_t upos = 0;  // output position of the element at ip
    while (!bad && ip < in_len) {
        if (ip + 69 > wbase + kWindow) {  // headers at ip .. ip+63 (+5 bytes each) inside the window
            wbase = ip & ~3u;
            win = load_window(in, in_len, wbase, lane);
        }
        // speculative header parse at q = ip + lane
        const uint32_t q = ip + (uint32_t)lane;
        const uint32_t r = q - wbase;
        const uint32_t d0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((r >> 2) & 63) << 2), (int)win);
        const uint32_t d1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((((r >> 2) + 1) & 63) << 2), (int)win);
        const uint64_t x = ((((uint64_t)d1) << 32) | d0) >> ((r & 3) * 8);
        const uint32_t tag = (uint32_t)x & 0xff;
        const uint32_t ext = (uint32_t)(x >> 8);
        const uint32_t kind = tag & 3;
        uint32_t len, off = 0;
        uint64_t csize;
        if (kind == 0) {
            len = (tag >> 2) + 1;
            uint32_t nb = 0;
            if (len > 60) {
                nb = len - 60;
                len = lit_len(ext, nb);
            }
            csize = 1ull + nb + len;
        } else if (kind == 1) {
            len = ((tag >> 2) & 7) + 4;
            off = ((tag >> 5) << 8) | (ext & 0xff);
            csize = 2;
        } else {
            len = (tag >> 2) + 1;
            off = kind == 2 ? (ext & 0xffff) : ext;
            csize = kind == 2 ? 3 : 5;
        }
        // the chain: serial, one readlane per element
        const uint32_t step = (uint32_t)min(csize, (uint64_t)0x7FFFFFFF);
        uint64_t mask = 0;
        uint32_t p = 0;
        while (p < (uint32_t)kWave && ip + p < in_len) {
            mask |= 1ull << p;
            p += (uint32_t)__builtin_amdgcn_readlane((int)step, (int)p);
        }
        const bool marked = (mask >> lane) & 1;
        // output positions of the marked elements: exclusive wave scan
        uint64_t v = marked ? (uint64_t)len : 0;
        for (int o = 1; o < kWave; o <<= 1) {
            const uint64_t t = __shfl_up(v, (unsigned)o, kWave);
            if (lane >= o) v += t;
        }
        const uint64_t u0 = upos + v - (marked ? len : 0);  // this element's output start
        const uint64_t u1 = u0 + len;
        int e = 0, c0 = 0, c1 = 0;
        if (marked) {
            if ((uint64_t)q + csize > in_len) e = 3;               // truncated
            else if (u1 > total) e = 4;                            // past the declared length
            else if (kind != 0 && (off == 0 || off > u0)) e = 6;   // before the stream
            if (!e) {
                const uint32_t a = (uint32_t)u0, z = (uint32_t)u1 - 1;
                c0 = a / L0 != z / L0 || (kind != 0 && off > a % L0);
                c1 = a / L1 != z / L1 || (kind != 0 && off > a % L1);
                if (a % L0 == 0 && a / L0 < (uint32_t)kSplitMaxSmall) starts_small[a / L0] = q;
                if (a % L1 == 0 && a / L1 < (uint32_t)kSplitMaxBig) starts_big[a / L1] = q;
            }
        }
        // wave-uniform verdicts
        const uint64_t eb = __ballot(e != 0);
        if (eb) {
            bad = __builtin_amdgcn_readlane(e, (int)__builtin_ctzll(eb));
            break;
        }
        cut0 |= __ballot(c0) != 0;
        cut1 |= __ballot(c1) != 0;
        upos = __shfl(u1, (int)(63 - __builtin_clzll(mask)), kWave);  // after the last marked element
        ip += p;
    }
    if (!bad && ip != in_len) bad = 3;
    if (!bad && upos != total) bad = 7;
    if (!bad && cut0 && cut1) bad = 8;  // not cuttable: the host decodes it
    __syncthreads();
    uint32_t np = 0;
    if (!bad) {
        const bool small = !cut0;
        const uint32_t L = small ? L0 : L1;
        const uint32_t* starts = small ? starts_small : starts_big;
        np = small ? np0 : np1;
        for (uint32_t k = lane; k < np; k += kWave) {
            const uint32_t s0 = starts[k], s1 = k + 1 < np ? starts[k + 1] : in_len;
            slots[k] = SnappyPiece{(const uint8_t*)st.src + s0, (uint8_t*)st.dst + (size_t)k * L, s1 - s0,
                                   min(L, total - k * L)};
        }
    }
    for (uint32_t k = np + lane; k < st.max_pieces; k += kWave) slots[k] = SnappyPiece{nullptr, nullptr, 0, 0};
    if (lane == 0) stream_err[sid] = bad;
}

// ------------------------------------------------------------- compression

constexpr int kHashBits = 7;  // per-lane table
constexpr int kHashEntries = 1 << kHashBits;
constexpr int kFirstBits = 12;  // block-wide earliest-position table
constexpr int kFirstEntries = 1 << kFirstBits;
constexpr uint16_t kNoPos = 0xFFFF;
__device__ __forceinline__ uint64_t load64(gbyte_c* p) {
    typedef uint64_t __attribute__((aligned(1))) u64_unaligned;
    return *reinterpret_cast<const __attribute__((address_space(1))) u64_unaligned*>(p);
}

// Unaligned 4/8-byte LDS reads as aligned dword reads + v_alignbyte: an
// (aligned(1)) dereference compiles to one ds_read_u8 per byte, and the
// compressor's serial probe loop waits on every one of them. The reads may
// touch up to 7 bytes past the staged block (the LDS layout leaves them
// readable; callers never use those bytes).
typedef const __attribute__((address_space(3))) uint32_t lword_c;
__device__ __forceinline__ uint32_t lload32(const lbyte* p) {
    const uintptr_t a = (uintptr_t)p;
    lword_c* w = (lword_c*)(a & ~(uintptr_t)3);
    return __builtin_amdgcn_alignbyte(w[1], w[0], (uint32_t)(a & 3));
}
__device__ __forceinline__ uint64_t lload64(const lbyte* p) {
    const uintptr_t a = (uintptr_t)p;
    lword_c* w = (lword_c*)(a & ~(uintptr_t)3);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], sh = (uint32_t)(a & 3);
    return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
}

// A literal element's tag (1-3 bytes) for `len` bytes; the bytes follow.
template <typename O>
__device__ __forceinline__ O emit_literal_tag(O o, uint32_t len) {
    const uint32_t n = len - 1;
    if (n < 60) {
        *o++ = (uint8_t)(n << 2);
    } else if (n < 256) {
        *o++ = (uint8_t)(60 << 2);
        *o++ = (uint8_t)n;
    } else {
        *o++ = (uint8_t)(61 << 2);
        *o++ = (uint8_t)n;
        *o++ = (uint8_t)(n >> 8);
    }
    return o;
}
constexpr int kLitSpans = 8;  // deferred literal copies per lane (more are copied in place)

template <typename O, typename S>
__device__ __forceinline__ O emit_literal(O o, S src, uint32_t len) {
    const uint32_t n = len - 1;
    if (n < 60) {
        *o++ = (uint8_t)(n << 2);
    } else if (n < 256) {
        *o++ = (uint8_t)(60 << 2);
        *o++ = (uint8_t)n;
    } else {
        *o++ = (uint8_t)(61 << 2);
        *o++ = (uint8_t)n;
        *o++ = (uint8_t)(n >> 8);
    }
    // 16 source bytes per LDS round trip (two lload64 issued together), then
    // 4 (lload32), written byte by byte (the output slot has any alignment;
    // stores need no wait)
    uint32_t k = 0;
    for (; k + 16 <= len; k += 16) {
        const uint64_t a = lload64(src + k), b = lload64(src + k + 8);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[k + i] = (uint8_t)(a >> (8 * i));
#pragma unroll
        for (int i = 0; i < 8; ++i) o[k + 8 + i] = (uint8_t)(b >> (8 * i));
    }
    for (; k + 4 <= len; k += 4) {
        const uint32_t v = lload32(src + k);
        o[k] = (uint8_t)v;
        o[k + 1] = (uint8_t)(v >> 8);
        o[k + 2] = (uint8_t)(v >> 16);
        o[k + 3] = (uint8_t)(v >> 24);
    }
    for (; k < len; ++k) o[k] = src[k];
    return o + len;
}

template <typename O>
__device__ __forceinline__ O emit_copy2(O o, uint32_t off, uint32_t len) {
    o[0] = (uint8_t)(((len - 1) << 2) | 2);
    o[1] = (uint8_t)off;
    o[2] = (uint8_t)(off >> 8);
    return o + 3;
}

// Same split as snappy's encoder: 64-byte pieces, a 60 so the tail stays
// >= 4, and the 2-byte copy-1 form for short, near matches.
template <typename O>
__device__ __forceinline__ O emit_copy(O o, uint32_t off, uint32_t len) {
    while (len >= 68) {
        o = emit_copy2(o, off, 64);
        len -= 64;
    }
    if (len > 64) {
        o = emit_copy2(o, off, 60);
        len -= 60;
    }
    if (len < 12 && off < 2048) {
        o[0] = (uint8_t)(((off >> 8) << 5) | ((len - 4) << 2) | 1);
        o[1] = (uint8_t)off;
        return o + 2;
    }
    return emit_copy2(o, off, len);
}


// Dynamic LDS: the block's input (in_cap bytes), then — kOutLds — the 64
// lanes' output slots of `slot` bytes each; otherwise the slots live in the
// global scratch (blocks above 32 KiB, whose slots would not fit).
// kCand (blocks up to kCandMax, the RPC path's 4 KiB blocks): no per-lane
// recent table; after the earliest-position table is built, a candidate pass
// gives every position its match candidate (the earliest earlier position
// with the same 4 bytes, verified) in a u16 array after the slots, four
// positions per three LDS round trips with no chain between positions. The
// lane's walk then reads four candidates per round trip, so a run of misses
// costs ALU only; the wave pays round trips where some lane extends a match.
constexpr uint32_t kCandMax = 8192;
static_assert(kCandMax / kWave <= 128, "match records hold a slice offset and length in 7 bits each");
// (Padding the staged input and the candidates so that lanes 64 bytes apart
// hit distinct LDS banks was measured slower on MI355X: 56 vs 51 us per
// 112-block launch of text; the layouts stay dense.)
__host__ __device__ constexpr uint32_t CompressInBytes(uint32_t in_cap, bool) { return in_cap; }
__host__ __device__ constexpr uint32_t CompressCandBytes(uint32_t in_cap) { return 2 * in_cap + 16; }
// One block per wave; the body of snappy_compress_kernel and of the
// compress role of codec_waves_kernel.
template <bool kOutLds, bool kCand>
__device__ __forceinline__ void compress_wave(const SnappyJob* __restrict__ jobs, int blk,
                                              uint8_t* __restrict__ scratch, uint32_t* __restrict__ out_len,
                                              int* __restrict__ err, uint32_t in_cap, uint32_t slot_bytes,
                                              uint64_t* __restrict__ stamps) {
    __shared__ uint16_t table[kCand ? 1 : kWave * kHashEntries];
    // kCand: an 11-bit earliest-position table (8 KiB): with the candidate
    // array replacing the per-lane tables, a 4 KiB block's workgroup fits in
    // 30 KiB of LDS, five per CU instead of three
    constexpr int kFB = kCand ? 11 : kFirstBits;
    __shared__ __attribute__((aligned(16))) uint32_t first_pos[1 << kFB];
    __shared__ uint32_t sizes[kWave];
    __shared__ uint64_t spans[kWave * kLitSpans];  // deferred literal copies per lane
    extern __shared__ __attribute__((aligned(16))) uint8_t dyn_lds[];
    const int lane = threadIdx.x;
    const SnappyJob job = jobs[blk];
    const uint32_t ulen = (uint32_t)job.src_len;
    if (job.src_len > in_cap) {
        if (lane == 0) {
            err[blk] = 1;
            out_len[blk] = 0;
        }
        return;
    }
    lbyte* const in = (lbyte*)dyn_lds;
    const uint32_t in_bytes = CompressInBytes(in_cap, kCand);
    // input accessors over the (kCand: padded) staging
    auto dw = [&](uint32_t d) -> uint32_t { return ((lword_c*)in)[d]; };
    auto rd8 = [&](uint32_t x) -> uint8_t { return in[x]; };
    auto rd32 = [&](uint32_t x) -> uint32_t {
        const uint32_t d = x >> 2;
        return __builtin_amdgcn_alignbyte(dw(d + 1), dw(d), x & 3);
    };
    auto rd64 = [&](uint32_t x) -> uint64_t {
        const uint32_t d = x >> 2, w0 = dw(d), w1 = dw(d + 1), w2 = dw(d + 2), sh = x & 3;
        return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
    };
    stamp(stamps, blk, lane, 0);
    // stage the block in LDS: every match probe below is an LDS read, not an
    // HBM round trip on the lane's serial path
    {
        gbyte_c* src = as_global(job.src);
        uint32_t done = 0;
        if ((reinterpret_cast<uintptr_t>(job.src) & 15) == 0) {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            done = ulen & ~15u;
            for (uint32_t o = lane * 16; o < done; o += kWave * 16) {
                *reinterpret_cast<__attribute__((address_space(3))) u32x4*>(in + o) =
                    *reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(src + o);
            }
        }
        for (uint32_t o = done + lane; o < ulen; o += kWave) in[o] = src[o];
        uint32_t* t = reinterpret_cast<uint32_t*>(table);
        if (!kCand)
            for (int i = lane; i < kWave * kHashEntries / 2; i += kWave) t[i] = 0xFFFFFFFFu;
        for (int i = lane; i < (1 << kFB); i += kWave) first_pos[i] = 0xFFFFFFFFu;
    }
    __syncthreads();
    stamp(stamps, blk, lane, 1);
    const uint32_t seg = (ulen + kWave - 1) / kWave;
    const uint32_t s = min(ulen, seg * (uint32_t)lane);
    const uint32_t e = min(ulen, s + seg);
    if (kCand) {
        // 32 positions per LDS round trip: the chunk's 9 words are read
        // together, then its atomics issue back to back (an LDS read between
        // them would wait for every atomic issued before it: a round trip per
        // 4 positions). Reads may run 35 bytes past the block (the slots
        // follow it in LDS; those positions are masked).
        for (uint32_t qb = s & ~3u; qb < e; qb += 32) {
            uint32_t w[9];
#pragma unroll
            for (int i = 0; i < 9; ++i) w[i] = dw((qb >> 2) + (uint32_t)i);
#pragma unroll
            for (int i = 0; i < 32; ++i) {
                const uint32_t q = qb + (uint32_t)i;
                const uint32_t v = __builtin_amdgcn_alignbyte(w[(i >> 2) + 1], w[i >> 2], (uint32_t)(i & 3));
                if (q >= s && q < e && q + 4 <= ulen) atomicMin(&first_pos[(v * 0x1e35a7bdu) >> (32 - kFB)], q);
            }
        }
    } else {
        // an 8-byte window of the segment in registers, refilled every 4
        // positions: the atomics issue back to back instead of each waiting
        // on its own LDS read
        uint32_t wb = 0xFFFFFFFFu, w0 = 0, w1 = 0;
        for (uint32_t q = s; q < e && q + 4 <= ulen; ++q) {
            const uint32_t qb = q & ~3u;
            if (qb != wb) {
                w0 = dw(qb >> 2);
                w1 = dw((qb >> 2) + 1);
                wb = qb;
            }
            const uint32_t v = __builtin_amdgcn_alignbyte(w1, w0, q & 3);
            atomicMin(&first_pos[(v * 0x1e35a7bdu) >> (32 - kFB)], q);
        }
    }
    __syncthreads();
    if (stamps && blk == 0 && lane == 0) stamps[8] = __builtin_amdgcn_s_memtime();  // atomics done
    // candidates (kCand): u16 per position after the output slots; a lane
    // writes and reads only its own segment's entries (no barrier needed)
    __attribute__((address_space(3))) uint16_t* const mc =
        (__attribute__((address_space(3))) uint16_t*)(in + in_bytes + (kOutLds ? kWave * slot_bytes : 0));
    if (kCand) {
        // three round trips per 16 positions (words; table entries;
        // candidate bytes), not three per 4 (16, not 32: register arrays of
        // 32 took the kernel from 84 to 206 VGPRs)
        for (uint32_t qb = s & ~3u; qb < e; qb += 16) {
            uint32_t w[5], c[16], x[16];
#pragma unroll
            for (int i = 0; i < 5; ++i) w[i] = dw((qb >> 2) + (uint32_t)i);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint32_t v = __builtin_amdgcn_alignbyte(w[(i >> 2) + 1], w[i >> 2], (uint32_t)(i & 3));
                c[i] = first_pos[(v * 0x1e35a7bdu) >> (32 - kFB)];
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint32_t q = qb + (uint32_t)i;
                x[i] = rd32(c[i] < q ? c[i] : 0u);
            }
            uint32_t mv[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const uint32_t q = qb + (uint32_t)i;
                const uint32_t v = __builtin_amdgcn_alignbyte(w[(i >> 2) + 1], w[i >> 2], (uint32_t)(i & 3));
                const bool ok = c[i] < q && q + 4 <= ulen && x[i] == v;
                mv[i] = ok ? c[i] : kNoPos;
            }
            if (qb >= s && qb + 16 <= e) {
                // the whole chunk is the lane's: four 8-byte stores (qb is a
                // multiple of 4), not 16 guarded 2-byte ones
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    *(__attribute__((address_space(3))) uint64_t*)(mc + qb + 4 * j) =
                        (uint64_t)mv[4 * j] | ((uint64_t)mv[4 * j + 1] << 16) | ((uint64_t)mv[4 * j + 2] << 32) |
                        ((uint64_t)mv[4 * j + 3] << 48);
            } else {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    const uint32_t q = qb + (uint32_t)i;
                    if (q >= s && q < e) mc[q] = (uint16_t)mv[i];
                }
            }
        }
    }
    stamp(stamps, blk, lane, 2);
    uint16_t* ht = table + (kCand ? 0 : lane * kHashEntries);
    uint32_t walk_iters = 0, walk_hits = 0;  // phase stamps only
    auto match = [&](auto o0) {
        auto o = o0;
        // Literal bytes are not copied inside the walk: their tags are
        // written and their bytes filled after it, so a lane that found a
        // long literal does not hold the wave's other lanes (a divergent wave
        // pays for every path any lane takes).
        uint64_t* const sp = spans + lane * kLitSpans;
        int nsp = 0;
        auto literal = [&](auto out, uint32_t from, uint32_t n) {
            if (nsp < kLitSpans) {
                out = emit_literal_tag(out, n);
                sp[nsp++] = (uint64_t)from | ((uint64_t)n << 24) | ((uint64_t)(uint32_t)(out - o0) << 44);
                return out + n;
            }
            out = emit_literal_tag(out, n);
            for (uint32_t k = 0; k < n; ++k) out[k] = rd8(from + k);
            return out + n;
        };
        uint32_t p = s, lit = s;
        if (kCand) {
            // The walk only decides: each match is recorded as two u16 in the
            // lane's own candidate entries it has already passed (record k at
            // s + 2k, s + 2k + 1 < p: a match covers >= 4 positions), and a
            // second loop emits the records. A wave runs every path any lane
            // takes, so with the emission inside the walk each of the ~29
            // iterations (the lane over unique bytes misses at every position)
            // that some lane matched in paid the literal and copy emission
            // too (~1.2k cycles per iteration, profiles/r6_codec_late.txt).
            uint32_t cb = 0xFFFFFFFFu, nm = 0;
            uint64_t cw = 0;
            while (p + 4 <= e) {
                ++walk_iters;
                if ((p >> 2) != cb) {  // four candidates per LDS read
                    cb = p >> 2;
                    cw = *(const __attribute__((address_space(3))) uint64_t*)(mc + (cb << 2));
                }
                const uint32_t cand = (uint32_t)(cw >> (16 * (p & 3))) & 0xFFFF;
                if (cand != kNoPos) {
                    uint32_t len = 4;
                    for (;;) {
                        if (p + len >= e) break;
                        const uint64_t x = rd64(cand + len) ^ rd64(p + len);
                        if (x) {
                            len += (uint32_t)__builtin_ctzll(x) >> 3;
                            break;
                        }
                        len += 8;
                    }
                    len = min(len, e - p);
                    ++walk_hits;
                    // p - s < seg <= 128 and len - 4 < 128: 7 bits each
                    mc[s + 2 * nm] = (uint16_t)((p - s) | ((len - 4) << 7));
                    mc[s + 2 * nm + 1] = (uint16_t)(p - cand);
                    ++nm;
                    p += len;
                    lit = p;
                } else if ((p | 3) - lit < 32) {
                    // steps are 1 up to lit + 32: jump to the next position of
                    // this candidate group that has one, or to the group's end
                    // (the fields shifted in from the top read as candidates,
                    // and the first of them is the group's end). A lane over
                    // unique bytes takes 8 iterations per 32 positions, not 29.
                    const uint64_t t = (p & 3) == 3 ? ~0ull : ~(cw >> (16 * ((p & 3) + 1)));
                    const uint64_t nz = (((t & 0x7FFF7FFF7FFF7FFFull) + 0x7FFF7FFF7FFF7FFFull) | t) & 0x8000800080008000ull;
                    p += 1 + ((uint32_t)__builtin_ctzll(nz) >> 4);
                } else {
                    p += 1 + ((p - lit) >> 5);
                }
            }
            lit = s;
            for (uint32_t k = 0; k < nm; ++k) {
                const uint32_t a = mc[s + 2 * k], off = mc[s + 2 * k + 1];
                const uint32_t mp = s + (a & 127), mlen = (a >> 7) + 4;
                if (mp > lit) o = literal(o, lit, mp - lit);
                o = emit_copy(o, off, mlen);
                lit = mp + mlen;
            }
        } else {
        // the probe's serial chain is LDS round trips; per position: the
        // 4 bytes at p come from a register window (refilled every 4 bytes),
        // both candidates (the lane's recent table, the block's earliest
        // table) are read in one round trip, and both are verified in one more
        uint32_t wb = 0xFFFFFFFFu, w0 = 0, w1 = 0;
        while (p + 4 <= e) {
            const uint32_t pb = p & ~3u;
            if (pb != wb) {
                lword_c* w = (lword_c*)(in + pb);
                w0 = w[0];
                w1 = w[1];
                wb = pb;
            }
            const uint32_t v = __builtin_amdgcn_alignbyte(w1, w0, p & 3);
            const uint32_t hm = v * 0x1e35a7bdu;
            const uint32_t h = hm >> (32 - kHashBits);
            const uint32_t c1 = ht[h];
            const uint32_t c2 = first_pos[hm >> (32 - kFB)];
            ht[h] = (uint16_t)p;
            const bool ok1 = c1 != kNoPos, ok2 = c2 < p;
            const uint32_t v1 = lload32(in + (ok1 ? c1 : 0u));
            const uint32_t v2 = lload32(in + (ok2 ? c2 : 0u));
            const bool hit1 = ok1 && v1 == v;
            const bool hit = hit1 || (ok2 && v2 == v);
            const uint32_t cand = hit1 ? c1 : c2;
            if (hit) {
                // 8 bytes per LDS round trip; the first differing byte comes
                // from the XOR (reads may run up to 7 bytes past e: clamped)
                uint32_t len = 4;
                for (;;) {
                    if (p + len >= e) break;
                    const uint64_t x = lload64(in + cand + len) ^ lload64(in + p + len);
                    if (x) {
                        len += (uint32_t)__builtin_ctzll(x) >> 3;
                        break;
                    }
                    len += 8;
                }
                len = min(len, e - p);
                if (p > lit) o = literal(o, lit, p - lit);
                o = emit_copy(o, p - cand, len);
                p += len;
                lit = p;
            } else {
                p += 1 + ((p - lit) >> 5);
            }
        }
        }
        if (e > lit) o = literal(o, lit, e - lit);
        // the deferred literal bytes: 16 per LDS round trip
        for (int i = 0; i < nsp; ++i) {
            const uint64_t d = sp[i];
            const uint32_t from = (uint32_t)(d & 0xFFFFFF), n = (uint32_t)((d >> 24) & 0xFFFFF);
            auto out = o0 + (uint32_t)(d >> 44);
            uint32_t k = 0;
            for (; k + 16 <= n; k += 16) {
                const uint64_t x0 = rd64(from + k), x1 = rd64(from + k + 8);
#pragma unroll
                for (int j = 0; j < 8; ++j) out[k + j] = (uint8_t)(x0 >> (8 * j));
#pragma unroll
                for (int j = 0; j < 8; ++j) out[k + 8 + j] = (uint8_t)(x1 >> (8 * j));
            }
            for (; k + 4 <= n; k += 4) {
                const uint32_t x = rd32(from + k);
                out[k] = (uint8_t)x;
                out[k + 1] = (uint8_t)(x >> 8);
                out[k + 2] = (uint8_t)(x >> 16);
                out[k + 3] = (uint8_t)(x >> 24);
            }
            for (; k < n; ++k) out[k] = rd8(from + k);
        }
        return (uint32_t)(o - o0);
    };
    lbyte* const lds_slots = in + in_bytes;
    uint8_t* const gscratch = scratch + (size_t)blk * SnappyCompressScratchPerBlock();
    if (kOutLds) {
        sizes[lane] = match(lds_slots + (size_t)lane * slot_bytes);
    } else {
        sizes[lane] = match(as_global(gscratch + (size_t)lane * SnappyCompressSlot()));
    }
    __syncthreads();
    stamp(stamps, blk, lane, 3);
    if (stamps && blk == 0) {
        // walk iterations: the wave's (its slowest lane's) and the lanes'
        // sum; matches: the lanes' sum
        const uint32_t it_max = wave_max(walk_iters), it_sum = wave_incl_sum(walk_iters);
        const uint32_t hit_sum = wave_incl_sum(walk_hits);
        if (lane == kWave - 1) {
            stamps[5] = it_max;
            stamps[6] = it_sum;
            stamps[7] = hit_sum;
        }
    }
    // varint header + prefix sum of the 64 slot sizes (DPP scan: lane k
    // holds slot k's size)
    uint32_t hdr = 1;
    for (uint32_t u = ulen; u >= 0x80; u >>= 7) ++hdr;
    const uint32_t my_size = sizes[lane];
    const uint32_t incl = wave_incl_sum(my_size);
    const uint32_t total = hdr + (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
    const uint32_t my_off = hdr + incl - my_size;
    gbyte* dst = as_global(job.dst);
    if (total > job.dst_cap) {
        if (lane == 0) {
            err[blk] = 2;
            out_len[blk] = 0;
        }
        return;
    }
    if (kOutLds && total <= (uint32_t)sizeof(first_pos) && ((uintptr_t)job.dst & 15) == 0) {
        // assemble the stream in LDS (the earliest-position table is free
        // now): every lane moves its own slot, 16 bytes per read, then the
        // wave streams the whole block out with coalesced 16-byte stores
        // instead of one wave step per slot
        __syncthreads();
        lbyte* const stage = (lbyte*)first_pos;
        if (lane < (int)hdr) {
            const uint32_t u = ulen >> (7 * lane);
            stage[lane] = (uint8_t)((u & 0x7f) | (lane + 1 < (int)hdr ? 0x80 : 0));
        }
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        // (read as 4-byte-aligned vectors: any slot stride works)
        typedef unsigned int u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
        const lbyte* src = lds_slots + (size_t)lane * slot_bytes;
        for (uint32_t j = 0; j < my_size; j += 16) {
            const u32x4a4 v = *reinterpret_cast<const __attribute__((address_space(3))) u32x4a4*>(src + j);
            const uint32_t n = min(16u, my_size - j);
#pragma unroll
            for (uint32_t b = 0; b < 16; ++b) {
                if (b < n) stage[my_off + j + b] = (uint8_t)(v[b >> 2] >> (8 * (b & 3)));
            }
        }
        __syncthreads();
        const uint32_t vec_end = total & ~15u;
        for (uint32_t o = (uint32_t)lane * 16; o < vec_end; o += kWave * 16)
            *reinterpret_cast<__attribute__((address_space(1))) u32x4*>(dst + o) =
                *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(stage + o);
        for (uint32_t o = vec_end + lane; o < total; o += kWave) dst[o] = stage[o];
    } else {
        if (lane < (int)hdr) {
            uint32_t u = ulen >> (7 * lane);
            dst[lane] = (uint8_t)((u & 0x7f) | (lane + 1 < (int)hdr ? 0x80 : 0));
        }
        // coalesced copy-out: the wave moves one slot at a time
        uint32_t at = hdr;
        for (int k = 0; k < kWave; ++k) {
            const uint32_t sz = (uint32_t)__builtin_amdgcn_readlane((int)my_size, k);
            if (kOutLds) {
                const lbyte* src = lds_slots + (size_t)k * slot_bytes;
                for (uint32_t j = lane; j < sz; j += kWave) dst[at + j] = src[j];
            } else {
                gbyte_c* src = as_global(gscratch + (size_t)k * SnappyCompressSlot());
                for (uint32_t j = lane; j < sz; j += kWave) dst[at + j] = src[j];
            }
            at += sz;
        }
    }
    if (lane == 0) {
        out_len[blk] = total;
        err[blk] = 0;
    }
    stamp(stamps, blk, lane, 4);
}

template <bool kOutLds, bool kCand>
__global__ void __launch_bounds__(kWave) snappy_compress_kernel(const SnappyJob* __restrict__ jobs, int n,
                                                                uint8_t* __restrict__ scratch,
                                                                uint32_t* __restrict__ out_len,
                                                                int* __restrict__ err, uint32_t in_cap,
                                                                uint32_t slot_bytes,
                                                                uint64_t* __restrict__ stamps) {
    if ((int)blockIdx.x >= n) return;
    compress_wave<kOutLds, kCand>(jobs, (int)blockIdx.x, scratch, out_len, err, in_cap, slot_bytes, stamps);
}

// One launch per device-body codec batch, one wave per unit of work:
// workgroups [0, ncomp) compress a block each, the rest decode a headerless
// piece each, and the wave that finishes the last piece of a message scans
// its protobuf fields (the group counter is reset for the batch's next
// launch). The per-stage sequence it replaces ran compress, decompress and
// pb-scan launches back to back on the batch's stream: ~31 + 33 + 5 us of
// latency-bound kernels per batch, each wave far from filling its CU, so
// sharing one dispatch halves the batch's device time while keeping the
// small-footprint waves that pack 5 per CU (many batches in flight share
// the chip). Two alternatives were measured and removed in round 6
// (profiles/r5_device_codec_ab.txt): a 1024-thread workgroup per block with
// a block-wide parse (faster alone, 26 vs 29 us, but it holds a CU per
// block: 139k vs 158-161k QPS on the device text leg with batches
// overlapping) and a data-parallel compressor whose matches cross the lane
// slices (ratio 2.14 vs 1.96, but 47 vs 28 us per launch: 116k QPS).
// Instantiated per role set: a batch of only decode pieces gets a kernel
// without the compressor's registers and static LDS (the per-wave footprint
// decides how many waves of concurrent batches share a CU).
template <bool kComp, bool kDec>
__global__ void __launch_bounds__(kWave) codec_waves_kernel(FusedCodecArgs a, uint32_t in_cap, uint32_t slot,
                                                            uint32_t cin_cap, uint32_t phi) {
    const int b = blockIdx.x;
    if (kComp && b < a.ncomp) {
        compress_wave<true, true>(a.comp, b, nullptr, a.comp_len, a.comp_err, in_cap, slot, nullptr);
        return;
    }
    if (!kDec) return;
    const int j = b - a.ncomp;
    if (j >= a.npieces) return;
    decode_piece_wave(a.pieces, j, 0, phi, cin_cap, a.piece_err, nullptr);
    const uint32_t g = a.piece_group ? a.piece_group[j] : kFusedNoGroup;
    if (g == kFusedNoGroup) return;
    __shared__ int last;
    __threadfence();  // this piece's bytes before the count
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(&a.group_done[g], 1u) + 1 == a.group_pieces[g];
    __syncthreads();
    if (!last) return;
    __threadfence();  // every other piece's bytes after the count
    if (threadIdx.x == 0) {
        a.group_done[g] = 0;
        const PbScanJob sj = a.scans[g];
        a.scan_n[g] = devpb::scan_message((devpb::gbyte_c*)sj.buf, 0, sj.len,
                                          a.scan_fields + (uint64_t)g * a.max_fields * 2, a.max_fields);
    }
}

}  // namespace

int LaunchCodecWaves(const FusedCodecArgs& a, hipStream_t s) {
    const int n = a.ncomp + a.npieces;
    if (n <= 0) return 0;
    const uint32_t mu = a.max_ulen ? a.max_ulen : 1;
    if (mu > kCandMax || mu > kParMax) return -1;
    const uint32_t in_cap = (mu + 15) & ~15u;
    const uint32_t seg = (mu + kWave - 1) / kWave;
    const uint32_t slot = (seg + 16 + 15) & ~15u;
    const uint32_t comp_lds = CompressInBytes(in_cap, true) + kWave * slot + CompressCandBytes(in_cap);
    const uint32_t cin_cap = (uint32_t)((SnappyMaxCompressedLength(mu) + 16 + 15) & ~15ull);
    const uint32_t dec_lds = cin_cap + 2 * ((mu + 7) & ~7u) + 16 * kWave;
    const uint32_t lds = std::max(a.ncomp ? comp_lds : 0u, a.npieces ? dec_lds : 0u);
    if (a.ncomp && a.npieces) {
        hipLaunchKernelGGL((codec_waves_kernel<true, true>), dim3((unsigned)n), dim3(kWave), lds, s, a, in_cap, slot,
                           cin_cap, mu);
    } else if (a.ncomp) {
        hipLaunchKernelGGL((codec_waves_kernel<true, false>), dim3((unsigned)n), dim3(kWave), lds, s, a, in_cap, slot,
                           cin_cap, mu);
    } else {
        hipLaunchKernelGGL((codec_waves_kernel<false, true>), dim3((unsigned)n), dim3(kWave), lds, s, a, in_cap, slot,
                           cin_cap, mu);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int LaunchSnappyDecompress(const SnappyJob* jobs_dev, int n, uint32_t max_ulen, uint32_t* out_len_dev, int* err_dev,
                           hipStream_t s) {
    if (n <= 0) return 0;
    if (max_ulen == 0) max_ulen = 1;
    if (max_ulen > kSnappyMaxBlock) return -1;
    const uint32_t lds = (max_ulen + 4095) & ~4095u;  // LDS per wave; blocks larger than this fail with code 2
    hipLaunchKernelGGL(snappy_decompress_kernel, dim3(n), dim3(kWave), lds, s, jobs_dev, n, lds, out_len_dev, err_dev);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int LaunchSnappySplit(const SnappyStream* streams_dev, int n, uint32_t piece_limit, SnappyPiece* pieces_dev,
                      int* stream_err_dev, hipStream_t s) {
    if (n <= 0) return 0;
    if (piece_limit == 0) return -1;
    hipLaunchKernelGGL(snappy_split_kernel, dim3(n), dim3(kWave), 0, s, streams_dev, n, piece_limit, pieces_dev,
                       stream_err_dev);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int LaunchSnappyDecompressPiecesSerial(const SnappyPiece* pieces_dev, int n, uint32_t lo, uint32_t hi, int* err_dev,
                                       hipStream_t s) {
    if (n <= 0) return 0;
    if (hi == 0 || hi > kSnappyMaxBlock || lo >= hi) return -1;
    const uint32_t lds = (hi + 4095) & ~4095u;
    hipLaunchKernelGGL(snappy_decompress_pieces_kernel, dim3(n), dim3(kWave), lds, s, pieces_dev, n, lo, hi, err_dev);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int LaunchSnappyDecompressPiecesStamped(const SnappyPiece* pieces_dev, int n, uint32_t lo, uint32_t hi, int* err_dev,
                                        uint64_t* stamps, hipStream_t s) {
    if (n <= 0) return 0;
    if (hi == 0 || hi > kSnappyMaxBlock || lo >= hi) return -1;
    // pieces up to kParMax: the parallel decoder; larger ones: the serial one
    if (lo < kParMax) {
        const uint32_t phi = std::min(hi, kParMax);
        const uint32_t cin_cap = (uint32_t)((SnappyMaxCompressedLength(phi) + 16 + 15) & ~15ull);
        const uint32_t lds = cin_cap + 2 * ((phi + 7) & ~7u) + 16 * kWave;
        hipLaunchKernelGGL(snappy_decompress_pieces_par_kernel, dim3(n), dim3(kWave), lds, s, pieces_dev, n, lo, phi,
                           cin_cap, err_dev, stamps);
        if (hipGetLastError() != hipSuccess) return -1;
        if (hi <= kParMax) return 0;
        lo = kParMax;
    }
    return LaunchSnappyDecompressPiecesSerial(pieces_dev, n, lo, hi, err_dev, s);
}

int LaunchSnappyDecompressPieces(const SnappyPiece* pieces_dev, int n, uint32_t lo, uint32_t hi, int* err_dev,
                                 hipStream_t s) {
    return LaunchSnappyDecompressPiecesStamped(pieces_dev, n, lo, hi, err_dev, nullptr, s);
}

int LaunchSnappyCompressStamped(const SnappyJob* jobs_dev, int n, uint32_t max_ulen, void* scratch, uint32_t* out_len_dev,
                                int* err_dev, uint64_t* stamps, hipStream_t s) {
    if (n <= 0) return 0;
    if (max_ulen == 0) max_ulen = 1;
    if (max_ulen > kSnappyMaxBlock) return -1;
    const uint32_t in_cap = (max_ulen + 15) & ~15u;  // larger jobs fail with code 1
    // a lane's output never exceeds its segment plus one literal header
    const uint32_t seg = (max_ulen + kWave - 1) / kWave;
    const uint32_t slot = (seg + 16 + 15) & ~15u;
    // slots in LDS too while that keeps >= 2 waves per CU (blocks up to
    // 16 KiB: <= 67 KiB); a 32 KiB block with LDS slots would run alone on its CU
    static_assert(16384 + kWave * ((16384 / kWave + 16 + 15) & ~15u) + kWave * kHashEntries * 2 + kFirstEntries * 4 +
                          kWave * 4 + kWave * kLitSpans * 8 <= 80 * 1024,
                  "16 KiB blocks keep their slots in LDS");
    if (max_ulen <= kCandMax) {
        // input, slots and the candidate array in LDS: <= 8 + 9 + 16 KiB
        const uint32_t cslot = slot;
        hipLaunchKernelGGL((snappy_compress_kernel<true, true>), dim3(n), dim3(kWave),
                           CompressInBytes(in_cap, true) + kWave * cslot + CompressCandBytes(in_cap), s, jobs_dev, n,
                           static_cast<uint8_t*>(scratch), out_len_dev, err_dev, in_cap, cslot, stamps);
    } else if (!SnappyCompressUsesScratch(max_ulen)) {
        hipLaunchKernelGGL((snappy_compress_kernel<true, false>), dim3(n), dim3(kWave), in_cap + kWave * slot, s,
                           jobs_dev, n, static_cast<uint8_t*>(scratch), out_len_dev, err_dev, in_cap, slot, stamps);
    } else {
        hipLaunchKernelGGL((snappy_compress_kernel<false, false>), dim3(n), dim3(kWave), in_cap, s, jobs_dev, n,
                           static_cast<uint8_t*>(scratch), out_len_dev, err_dev, in_cap, slot, stamps);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int LaunchSnappyCompress(const SnappyJob* jobs_dev, int n, uint32_t max_ulen, void* scratch, uint32_t* out_len_dev,
                         int* err_dev, hipStream_t s) {
    return LaunchSnappyCompressStamped(jobs_dev, n, max_ulen, scratch, out_len_dev, err_dev, nullptr, s);
}

}  // namespace gpu
}  // namespace mrpc
