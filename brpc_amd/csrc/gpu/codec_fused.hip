// Fused, workgroup-parallel snappy codec for device-resident bodies on CDNA4
// (gfx950): the device half of the body codec (reference:
// src/brpc/policy/snappy_compress.cpp:28-64 over
// src/butil/third_party/snappy/snappy.cc:875, which the reference runs on
// the CPU per message).
//
// Why not one wave per block (snappy_kernels.hip): at RPC batch sizes a
// launch carries a few hundred blocks, under one wave per SIMD, and a
// wave that walks a block's element chain is pure latency — the kernel took
// ~31 us whatever its grid. Here a block gets 256 threads (4
// waves that hide each other's LDS latency) and no phase walks the whole
// block serially:
//
// Compress (block of n <= 8 KiB bytes, staged in LDS):
//   1. every position p hashes its 4 bytes into a 4096-entry table with
//      ds_min: the table keeps the EARLIEST position of each hash, a legal
//      source for every later position;
//   2. every position reads its candidate, verifies it, and measures the
//      match length L[p] (8 bytes per LDS round trip, capped at 64 = one
//      snappy copy element); NC[p] = the first position >= p with a match
//      (a block-wide suffix-min over the threads' first matches);
//   3. the greedy parse is the orbit of 0 under next(p) = p + L[p] (copy)
//      or NC[p + 1] (a literal run up to the next match). Each thread walks
//      its 16-32 byte segment from a speculative entry (its segment start);
//      rounds then hand every segment its predecessor's exit and re-walk
//      the segments whose entry changed, until no exit moves. Segment 0 is
//      exact from the start and segment s is exact once s-1 is, so this is
//      the sequential parse; walks from different entries merge within a
//      few elements, so it settles in a few rounds;
//   4. element sizes -> block prefix sum -> tags written in LDS; literal
//      bytes are placed by every thread for its own positions (the run in
//      force comes from a block max-scan of run starts); the stream leaves
//      with 16-byte stores.
//   Matches span the whole block (no per-lane segment caps), so the ratio
//   is that of a greedy matcher over the block.
//
// Decode (headerless piece, n <= 8 KiB out):
//   1. the element chain over the compressed bytes, found with the same
//      speculative segment walks (a walk from inside an element reads
//      garbage sizes, but only until it lands on a true boundary, and the
//      rounds keep only the walk from the true entry);
//   2. element output sizes -> prefix sum -> each element's descriptor at
//      its output position; a block max-scan of element starts gives every
//      output byte its element, hence its source: a literal byte of the
//      piece, or an earlier output byte (copy);
//   3. the source map resolved by pointer jumping (log2 of the copy-chain
//      depth rounds), then gathered and stored 16 bytes per store.
//
// A message whose pieces all decoded is pb-scanned by the workgroup that
// finishes its last piece (a per-group HBM counter, release/acquire
// fences), so a codec batch is ONE launch: compress, decode and index run
// concurrently instead of as serial kernels on one stream.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gpu/device_pb.h"
#include "gpu/kernels.h"

namespace mrpc {
namespace gpu {

namespace {

constexpr int kT = 1024;  // threads per workgroup: 16 waves, 4 per SIMD to hide LDS latency
constexpr int kWaves = kT / 64;
constexpr int kTableBits = 12;
constexpr uint32_t kNone = 0xFFFFFFFFu;


typedef const __attribute__((address_space(1))) uint8_t gbyte_c;
typedef __attribute__((address_space(1))) uint8_t gbyte;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- scans
struct OpSum {
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; }
};
struct OpMax {
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; }
};
struct OpMin {
    __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a < b ? a : b; }
};

// Inclusive wave64 scan on DPP (row shifts, then row broadcasts 15 and 31):
// VALU cross-lane moves, no LDS round trip. `identity` fills lanes with no
// source.
template <typename Op>
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, Op op, uint32_t identity = 0) {
    const int id = (int)identity;
    v = op((uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x111, 0xf, 0xf, false), v);
    v = op((uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x112, 0xf, 0xf, false), v);
    v = op((uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x114, 0xf, 0xf, false), v);
    v = op((uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x118, 0xf, 0xf, false), v);
    v = op((uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x142, 0xa, 0xf, false), v);
    v = op((uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x143, 0xc, 0xf, false), v);
    return v;
}

// Block-wide exclusive scan (identity for thread 0); *total = the reduction.
// wtot: kWaves words of LDS. Ends with a barrier, so wtot may be reused.
template <typename Op>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t identity, Op op, uint32_t* wtot,
                                                    uint32_t* total) {
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const uint32_t incl = wave_incl_scan(v, op, identity);
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    uint32_t pre = identity, tot = identity;
#pragma unroll
    for (int k = 0; k < kWaves; ++k) {
        const uint32_t x = wtot[k];
        if (k < w) pre = op(pre, x);
        tot = op(tot, x);
    }
    const uint32_t prev = (uint32_t)__shfl_up((int)incl, 1u, 64);
    __syncthreads();
    *total = tot;
    return lane ? op(pre, prev) : pre;
}

// Exclusive SUFFIX scan: op over the values of threads t' > t.
template <typename Op>
__device__ __forceinline__ uint32_t block_excl_suffix(uint32_t v, uint32_t identity, Op op, uint32_t* wtot,
                                                      uint32_t* xch) {
    const int t = threadIdx.x;
    xch[kT - 1 - t] = v;
    __syncthreads();
    uint32_t tot;
    const uint32_t r = block_excl_scan(xch[t], identity, op, wtot, &tot);
    xch[kT - 1 - t] = r;
    __syncthreads();
    const uint32_t out = xch[t];
    __syncthreads();
    return out;
}

// ---------------------------------------------------------------- LDS bytes
__device__ __forceinline__ uint32_t rd32(const uint8_t* in, uint32_t x) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(in);
    const uint32_t d = x >> 2;
    return __builtin_amdgcn_alignbyte(w[d + 1], w[d], x & 3);
}
__device__ __forceinline__ uint64_t rd64(const uint8_t* in, uint32_t x) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(in);
    const uint32_t d = x >> 2, sh = x & 3, w0 = w[d], w1 = w[d + 1], w2 = w[d + 2];
    return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
}

// Stage src[0, n) at lds (16-byte aligned) and zero `pad` bytes after it.
// A source that is not 16-byte aligned is read as the aligned 16-byte
// chunks that cover it (a chunk never crosses a page, so it is mapped) and
// the bytes land at lds + (src & 15): returns that misalignment, the
// caller's byte view starts there (word reads take lds and mis + offset).
__device__ __forceinline__ uint32_t stage_in(const void* src, uint32_t n, uint8_t* lds, uint32_t pad) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(src);
    const uint32_t mis = (uint32_t)(a & 15);
    const __attribute__((address_space(1))) u32x4* g = (const __attribute__((address_space(1))) u32x4*)(a - mis);
    const uint32_t chunks = (mis + n + 15) >> 4;
    u32x4* l = reinterpret_cast<u32x4*>(lds);
    for (uint32_t c = threadIdx.x; c < chunks; c += kT) l[c] = g[c];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < pad; i += kT) lds[mis + n + i] = 0;
    return mis;
}

__device__ __forceinline__ uint32_t varint_len(uint32_t v) {
    uint32_t k = 1;
    while (v >= 0x80) {
        v >>= 7;
        ++k;
    }
    return k;
}

__device__ __forceinline__ uint32_t lit_tag_bytes(uint32_t ll) { return ll <= 60 ? 1 : (ll <= 256 ? 2 : 3); }

__device__ __forceinline__ uint32_t hash4(uint32_t v) { return (v * 0x1e35a7bdu) >> (32 - kTableBits); }

// Store total bytes of `stage` to dst: 16-byte stores when dst is aligned.
__device__ __forceinline__ void store_out(void* dst, const uint8_t* stage, uint32_t total) {
    gbyte* d = (gbyte*)dst;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        const uint32_t vec = total & ~15u;
        for (uint32_t o = threadIdx.x * 16; o < vec; o += kT * 16)
            *reinterpret_cast<__attribute__((address_space(1))) u32x4*>(d + o) =
                *reinterpret_cast<const u32x4*>(stage + o);
        for (uint32_t o = vec + threadIdx.x; o < total; o += kT) d[o] = stage[o];
    } else {
        for (uint32_t o = threadIdx.x; o < total; o += kT) d[o] = stage[o];
    }
}

// Phase stamps (shader clock, cumulative since the workgroup started) of
// the first compress block and the first decode piece, into stats[4..] and
// stats[16..] (benchmarks/fused_codec_ab.py prints them per phase).
struct Stamper {
    uint32_t* st = nullptr;
    uint64_t t0 = 0;
    __device__ Stamper(uint32_t* stats, bool first, int base) {
        if (stats && first && threadIdx.x == 0) {
            st = stats + base;
            t0 = __builtin_amdgcn_s_memtime();
        }
    }
    __device__ void operator()(int k) const {
        if (st) st[k] = (uint32_t)(__builtin_amdgcn_s_memtime() - t0);
    }
};

// ---------------------------------------------------------------- chains
constexpr int kChainPer = 10;  // positions per thread: covers a compressed 8 KiB piece (<= 9589 bytes)
static_assert(SnappyMaxCompressedLength(kFusedMaxBlock) <= (uint64_t)kChainPer * kT, "chain positions per thread");
// The element chain of a block (compress: the greedy parse's element
// starts; decode: the element boundaries of the compressed bytes) is the
// orbit of 0 under nx[] (nx[i] > i). It is found by pointer jumping over
// every position at once: J_0 = nx, J_{k+1} = J_k o J_k (double-buffered),
// and in round k every position already on the chain marks J_k of itself,
// so after round k every chain element within 2^(k+1) steps of 0 is marked.
// The rounds end once J_{k+1}(0) has left the block (the chain is shorter
// than 2^(k+1)): ceil(log2(elements)) + 1 rounds of a few independent LDS
// ops per position, with no serial walk and no data-dependent worst case
// (a speculative per-segment walk needed 15 rounds on periodic input).
// on: npos + 64 bytes; j0, j1: npos u16 each. marks: one u64 per 64
// positions (the ballot of on[]). Returns where the chain ends (>= npos).
__device__ __forceinline__ uint32_t chain_marks(const uint16_t* nx, uint32_t npos, uint64_t* marks, uint8_t* on,
                                                uint16_t* j0, uint16_t* j1, uint32_t* rounds_out) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t W = (npos + 63) / 64;
    for (uint32_t i = t; i < W * 64; i += kT) {
        if (i < npos) j0[i] = nx[i];
        on[i] = i == 0;
    }
    __syncthreads();
    uint32_t rounds = 0, end;
    for (int k = 0;; ++k) {
        const uint16_t* src = (k & 1) ? j1 : j0;
        uint16_t* dst = (k & 1) ? j0 : j1;
        // up to kChainPer positions per thread: every load is issued before
        // any result is used
        uint32_t j[kChainPer];
#pragma unroll
        for (int u = 0; u < kChainPer; ++u) {
            const uint32_t i = (uint32_t)t + (uint32_t)u * kT;
            j[u] = i < npos ? src[i] : npos;
        }
#pragma unroll
        for (int u = 0; u < kChainPer; ++u) {
            const uint32_t i = (uint32_t)t + (uint32_t)u * kT;
            if (i >= npos) break;
            const uint32_t jj = j[u] < npos ? src[j[u]] : j[u];
            if (j[u] < npos && on[i]) on[j[u]] = 1;
            dst[i] = (uint16_t)jj;
        }
        ++rounds;
        __syncthreads();
        // (dst is the next round's source, never written by it: no second
        // barrier before the next round)
        end = dst[0];
        if (end >= npos) break;  // block-uniform: read after the barrier
    }
    for (uint32_t w = (uint32_t)wv; w < W; w += kWaves) {
        const uint64_t m = __ballot(on[w * 64 + lane] != 0);
        if (lane == 0) marks[w] = m;
    }
    __syncthreads();
    if (rounds_out) *rounds_out = rounds;
    return end;
}

// ---------------------------------------------------------------- compress
constexpr uint32_t kCompWins = kFusedMaxBlock / 64;  // 128
// LDS: in (C + 96: 16 B of alignment slack, 80 B of zero pad) | L (C) |
// cand (2C) | NX (2C + 16) | table (16 KiB, later the output stage) |
// mb, wm (u64 x kCompWins) | nz, wsz, wbase, carry (u32 x (kCompWins + 1)) |
// wtot | xch | ex
__host__ __device__ constexpr uint32_t CompressLds(uint32_t C) {
    return (C + 96) + C + 2 * C + (2 * C + 16) + (4u << kTableBits) + 16 * kCompWins + 16 * (kCompWins + 1) +
           4 * (kWaves + kT + 4 * kWaves) + (C + 64) + 6 * C + 64;
}

__device__ void compress_block(const FusedCodecArgs& a, int job, uint8_t* lds) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const SnappyJob jb = a.comp[job];
    const uint32_t n = (uint32_t)jb.src_len;
    const uint32_t C = (a.max_ulen + 15) & ~15u;
    if (jb.src_len > a.max_ulen || n == 0) {
        if (t == 0) {
            a.comp_err[job] = n == 0 ? 0 : 1;
            a.comp_len[job] = 0;
        }
        return;
    }
    uint8_t* raw = lds;
    uint8_t* L = raw + C + 96;
    uint16_t* cand = reinterpret_cast<uint16_t*>(L + C);
    uint16_t* NX = cand + C;
    uint32_t* table = reinterpret_cast<uint32_t*>(NX + C + 8);
    uint8_t* stage = reinterpret_cast<uint8_t*>(table);
    uint64_t* mb = reinterpret_cast<uint64_t*>(table + (1u << kTableBits));  // match-position bits per window
    uint64_t* wm = mb + kCompWins;                                            // element starts per window
    uint32_t* nz = reinterpret_cast<uint32_t*>(wm + kCompWins);               // next window with a match
    uint32_t* wsz = nz + kCompWins + 1;
    uint32_t* wbase = wsz + kCompWins + 1;
    uint32_t* carry = wbase + kCompWins + 1;
    uint32_t* wtot = carry + kCompWins + 1;
    uint32_t* xch = wtot + kWaves;
    uint32_t* ex = xch + kT;
    uint8_t* on = reinterpret_cast<uint8_t*>(ex + 4 * kWaves);  // chain: C + 64 bytes, then two u16 jump arrays
    uint16_t* j0 = reinterpret_cast<uint16_t*>(on + C + 64);
    uint16_t* j1 = j0 + C;
    uint16_t* ES = j1 + C;  // output bytes of the element starting at p, if one does
    const uint32_t W = (n + 63) / 64;

    const Stamper stamp(a.stats, job == 0, 4);
    for (uint32_t i = t; i < (1u << kTableBits); i += kT) table[i] = kNone;
    const uint32_t mis = stage_in(jb.src, n, raw, 80);
    const uint8_t* in = raw + mis;
    __syncthreads();
    stamp(0);
    // 1. earliest position of every hash (interleaved positions; a hash
    //    already holding an earlier position skips its atomic, so a long run
    //    of one repeated key costs one round of contended atomics, not n)
    for (uint32_t p = t; p + 4 <= n; p += kT) {
        uint32_t* e = &table[hash4(rd32(raw, mis + p))];
        if (*e > p) atomicMin(e, p);
    }
    __syncthreads();
    stamp(1);
    // 2. candidate and match length (<= 64: one copy element) per position;
    //    the wave's ballot is the window's match mask
    for (uint32_t base = 0; base < W * 64; base += kT) {
        const uint32_t p = base + (uint32_t)t;
        uint32_t l = 0, c = 0;
        if (p + 4 <= n) {
            const uint32_t key = rd32(raw, mis + p);
            const uint32_t cp = table[hash4(key)];
            if (cp < p && rd32(raw, mis + cp) == key) {
                const uint32_t cap = min(64u, n - p);
                l = 4;
                while (l < cap) {
                    const uint64_t x = rd64(raw, mis + cp + l) ^ rd64(raw, mis + p + l);
                    if (x) {
                        l += (uint32_t)__builtin_ctzll(x) >> 3;
                        break;
                    }
                    l += 8;
                }
                l = min(l, cap);
                c = cp;
            }
        }
        if (p < n) {
            L[p] = (uint8_t)l;
            cand[p] = (uint16_t)c;
        }
        const uint64_t m = __ballot(l >= 4);
        const uint32_t w = (base >> 6) + (uint32_t)wv;
        if (lane == 0 && w < W) mb[w] = m;
    }
    __syncthreads();
    stamp(2);
    // nz[w]: the first window >= w with a match (W: none)
    {
        const uint32_t v = (uint32_t)t < W ? (mb[t] ? (uint32_t)t : W) : W;
        const uint32_t r = min(v, block_excl_suffix(v, W, OpMin(), wtot, xch));
        if ((uint32_t)t <= W) nz[t] = (uint32_t)t < W ? r : W;
    }
    __syncthreads();
    // the parse's successor: a copy jumps over its match, a literal runs to
    // the next match position (NC)
    auto next_match = [&](uint32_t q) -> uint32_t {
        if (q >= n) return n;
        const uint32_t w = q >> 6;
        const uint64_t m = mb[w] >> (q & 63);
        if (m) return q + (uint32_t)__builtin_ctzll(m);
        const uint32_t w2 = nz[w + 1];
        return w2 < W ? w2 * 64 + (uint32_t)__builtin_ctzll(mb[w2]) : n;
    };
    for (uint32_t p = t; p < n; p += kT) {
        const uint32_t l = L[p];
        const uint32_t nx = l >= 4 ? p + l : next_match(p + 1);
        NX[p] = (uint16_t)nx;
        ES[p] = (uint16_t)(l >= 4 ? ((l < 12 && p - cand[p] < 2048) ? 2 : 3) : lit_tag_bytes(nx - p) + (nx - p));
    }
    __syncthreads();
    stamp(3);
    // 3. the greedy parse
    uint32_t rounds = 0;
    chain_marks(NX, n, wm, on, j0, j1, &rounds);
    stamp(4);
    if (a.stats && t == 0) {
        atomicAdd(&a.stats[0], rounds);
        atomicMax(&a.stats[1], rounds);
    }
    // 4. element sizes per window (lane = position), window offsets
    auto elem_size = [&](uint32_t p, bool st) -> uint32_t { return st ? ES[p] : 0u; };
    for (uint32_t k = (uint32_t)wv; k < W; k += kWaves) {
        const uint32_t p = k * 64 + (uint32_t)lane;
        const bool st = p < n && ((wm[k] >> lane) & 1);
        const uint32_t incl = wave_incl_scan(elem_size(p, st), OpSum());
        if (lane == 63) wsz[k] = incl;
    }
    __syncthreads();
    uint32_t body;
    const uint32_t hdr = varint_len(n);
    const uint32_t wb = block_excl_scan((uint32_t)t < W ? wsz[t] : 0u, 0u, OpSum(), wtot, &body);
    if ((uint32_t)t < W) wbase[t] = hdr + wb;
    const uint32_t total = hdr + body;
    stamp(5);
    if (total > jb.dst_cap || total > (4u << kTableBits)) {  // block-uniform
        if (t == 0) {
            a.comp_err[job] = 2;
            a.comp_len[job] = 0;
        }
        return;
    }
    // (the table is free: its last reads were before the barriers above)
    {
        // latest literal-run start + 1 before each window (0: none)
        const uint64_t rb = (uint32_t)t < W ? wm[t] & ~mb[t] : 0;
        const uint32_t v = rb ? (uint32_t)t * 64 + 64 - (uint32_t)__builtin_clzll(rb) : 0u;
        uint32_t tot;
        const uint32_t c = block_excl_scan(v, 0u, OpMax(), wtot, &tot);
        if ((uint32_t)t < W) carry[t] = c;
    }
    // 5. tags: every element start's lane writes its tag at its offset
    for (uint32_t k = (uint32_t)wv; k < W; k += kWaves) {
        const uint32_t p = k * 64 + (uint32_t)lane;
        const bool st = p < n && ((wm[k] >> lane) & 1);
        const uint32_t sz = elem_size(p, st);
        const uint32_t o = wbase[k] + wave_incl_scan(sz, OpSum()) - sz;
        if (!st) continue;
        const uint32_t l = L[p];
        if (l >= 4) {
            const uint32_t off = p - cand[p];
            if (l < 12 && off < 2048) {
                stage[o] = (uint8_t)(((off >> 8) << 5) | ((l - 4) << 2) | 1);
                stage[o + 1] = (uint8_t)off;
            } else {
                stage[o] = (uint8_t)(((l - 1) << 2) | 2);
                stage[o + 1] = (uint8_t)off;
                stage[o + 2] = (uint8_t)(off >> 8);
            }
        } else {
            const uint32_t ll = NX[p] - p, v = ll - 1;
            uint32_t h = 1;
            if (ll <= 60) {
                stage[o] = (uint8_t)(v << 2);
            } else if (ll <= 256) {
                stage[o] = 60 << 2;
                stage[o + 1] = (uint8_t)v;
                h = 2;
            } else {
                stage[o] = 61 << 2;
                stage[o + 1] = (uint8_t)v;
                stage[o + 2] = (uint8_t)(v >> 8);
                h = 3;
            }
            cand[p] = (uint16_t)(o + h);  // where the run's bytes go (cand is unused at literals)
        }
    }
    if (t < (int)hdr) stage[t] = (uint8_t)(((n >> (7 * t)) & 0x7f) | (t + 1 < (int)hdr ? 0x80 : 0));
    __syncthreads();
    stamp(6);
    // 6. literal bytes, one position per lane: the run in force at p is the
    //    latest literal-run start <= p
    for (uint32_t p = t; p < n; p += kT) {
        const uint32_t w = p >> 6, b = p & 63;
        const uint64_t rb = wm[w] & ~mb[w] & (b == 63 ? ~0ull : ((2ull << b) - 1));
        const uint32_t r1 = rb ? w * 64 + 64 - (uint32_t)__builtin_clzll(rb) : carry[w];
        if (r1 == 0) continue;
        const uint32_t r = r1 - 1;
        if (p < NX[r]) stage[cand[r] + (p - r)] = in[p];
    }
    __syncthreads();
    stamp(7);
    store_out(jb.dst, stage, total);
    stamp(8);
    if (t == 0) {
        a.comp_len[job] = total;
        a.comp_err[job] = 0;
    }
}

// ---------------------------------------------------------------- decode
constexpr uint32_t kDecWins = (uint32_t)((SnappyMaxCompressedLength(kFusedMaxBlock) + 63) / 64);  // 150
__host__ __device__ constexpr uint32_t DecodeCinCap(uint32_t C) {
    return (uint32_t)((SnappyMaxCompressedLength(C) + 15) & ~15ull);
}
// LDS: cin (cap + 128) | NX (2 x (cap + 16)) | desc (2C) | src (2C) |
// cm (u64 x kDecWins) | sb (u64 x kCompWins) | wsz, wbase (u32 x kDecWins) |
// ocarry (u32 x kCompWins) | wtot | xch | ex
__host__ __device__ constexpr uint32_t DecodeLds(uint32_t C) {
    return DecodeCinCap(C) + 128 + 2 * (DecodeCinCap(C) + 16) + 2 * C + 2 * C + 8 * kDecWins + 8 * kCompWins +
           8 * kDecWins + 4 * kCompWins + 4 * (kWaves + kT + 4 * kWaves) + (DecodeCinCap(C) + 64) +
           4 * DecodeCinCap(C) + 64;
}

__device__ void decode_piece(const FusedCodecArgs& a, int job, uint8_t* lds) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const SnappyPiece pc = a.pieces[job];
    const uint32_t C = (a.max_ulen + 15) & ~15u;
    const uint32_t cap = DecodeCinCap(C);
    const uint32_t m = pc.src_len, n = pc.ulen;
    uint8_t* raw = lds;
    uint16_t* NX = reinterpret_cast<uint16_t*>(raw + cap + 128);
    uint16_t* desc = NX + cap + 16;
    uint16_t* src = desc + C;
    uint64_t* cm = reinterpret_cast<uint64_t*>(src + C);  // element starts per compressed window
    uint64_t* sb = cm + kDecWins;                          // element starts per output window
    uint32_t* wsz = reinterpret_cast<uint32_t*>(sb + kCompWins);
    uint32_t* wbase = wsz + kDecWins;
    uint32_t* ocarry = wbase + kDecWins;
    uint32_t* wtot = ocarry + kCompWins;
    uint32_t* xch = wtot + kWaves;
    uint32_t* ex = xch + kT;
    uint8_t* on = reinterpret_cast<uint8_t*>(ex + 4 * kWaves);  // chain: cap + 64 bytes, then two u16 jump arrays
    uint16_t* j0 = reinterpret_cast<uint16_t*>(on + cap + 64);
    uint16_t* j1 = j0 + cap;
    __shared__ int bad;
    if (t == 0) bad = 0;
    const bool fits = n <= a.max_ulen && m <= cap && n > 0 && m > 0;
    if (fits) {
        const uint32_t Wc = (m + 63) / 64, Wo = (n + 63) / 64;
        for (uint32_t i = t; i < Wo; i += kT) sb[i] = 0;
        const Stamper stamp(a.stats, job == 0, 16);
        const uint32_t mis = stage_in(pc.src, m, raw, 16);
        const uint8_t* cin = raw + mis;
        __syncthreads();
        stamp(0);
        // 1. every compressed position's element size as if an element
        //    started there; the chain from position 0 keeps the true ones
        //    (a size running past the piece saturates at m + 1)
        auto elem = [&](uint32_t i, uint32_t* len, uint32_t* off, uint32_t* lsrc) -> uint32_t {
            const uint32_t tag = cin[i];
            const uint32_t kind = tag & 3;
            *off = 0;
            *lsrc = 0;
            if (kind == 0) {
                uint32_t l = (tag >> 2) + 1, h = 1;
                if (l > 60) {
                    const uint32_t nb = l - 60;
                    const uint32_t r = rd32(raw, mis + i + 1) & (0xFFFFFFFFu >> (32 - 8 * nb));
                    l = r >= 0x7FFF0000u ? 0x7FFF0000u : r + 1;
                    h += nb;
                }
                *len = l;
                *lsrc = i + h;
                return h + l;
            }
            if (kind == 1) {
                *len = ((tag >> 2) & 7) + 4;
                *off = ((tag >> 5) << 8) | cin[i + 1];
                return 2;
            }
            *len = (tag >> 2) + 1;
            if (kind == 2) {
                *off = cin[i + 1] | ((uint32_t)cin[i + 2] << 8);
                return 3;
            }
            *off = rd32(raw, mis + i + 1);
            return 5;
        };
        for (uint32_t i = t; i < m; i += kT) {
            uint32_t len, off, ls;
            const uint32_t cs = elem(i, &len, &off, &ls);
            NX[i] = (uint16_t)min(i + cs, m + 1);
        }
        __syncthreads();
        stamp(1);
        uint32_t rounds = 0;
        const uint32_t end = chain_marks(NX, m, cm, on, j0, j1, &rounds);
        stamp(2);
        if (a.stats && t == 0) {
            atomicAdd(&a.stats[2], rounds);
            atomicMax(&a.stats[3], rounds);
        }
        if (end != m) {
            if (t == 0) bad = 3;  // the chain does not end at the piece's end
        } else {
            // 2. output lengths per compressed window (lane = position)
            for (uint32_t k = (uint32_t)wv; k < Wc; k += kWaves) {
                const uint32_t i = k * 64 + (uint32_t)lane;
                uint32_t len = 0, off, ls;
                if (i < m && ((cm[k] >> lane) & 1)) elem(i, &len, &off, &ls);
                const uint32_t incl = wave_incl_scan(len, OpSum());  // a sound chain's lengths fit
                if (lane == 63) wsz[k] = incl;
            }
        }
        __syncthreads();  // (publishes `bad`)
        stamp(3);
        if (!bad) {
            uint32_t total;
            const uint32_t wb = block_excl_scan((uint32_t)t < Wc ? wsz[t] : 0u, 0u, OpSum(), wtot, &total);
            if ((uint32_t)t < Wc) wbase[t] = wb;
            if (total != n) {
                if (t == 0) bad = 4;
            } else {
                __syncthreads();
                // descriptors at element starts: a literal's source in the
                // piece, or a copy's offset
                for (uint32_t k = (uint32_t)wv; k < Wc; k += kWaves) {
                    const uint32_t i = k * 64 + (uint32_t)lane;
                    uint32_t len = 0, off = 0, ls = 0;
                    const bool st = i < m && ((cm[k] >> lane) & 1);
                    if (st) elem(i, &len, &off, &ls);
                    const uint32_t o = wbase[k] + wave_incl_scan(len, OpSum()) - len;
                    if (!st) continue;
                    if ((cin[i] & 3) == 0) {
                        desc[o] = (uint16_t)(0x8000u | ls);
                    } else if (off == 0 || off > o) {
                        atomicOr(&bad, 6);  // a copy from before the piece
                        desc[o] = 0x8000u;
                    } else {
                        desc[o] = (uint16_t)off;
                    }
                    atomicOr(reinterpret_cast<uint32_t*>(sb) + (o >> 5), 1u << (o & 31));
                }
            }
        }
        __syncthreads();
        if (!bad) {
            {
                // latest element start + 1 before each output window
                const uint64_t bits = (uint32_t)t < Wo ? sb[t] : 0;
                const uint32_t v = bits ? (uint32_t)t * 64 + 64 - (uint32_t)__builtin_clzll(bits) : 0u;
                uint32_t tot;
                const uint32_t c = block_excl_scan(v, 0u, OpMax(), wtot, &tot);
                if ((uint32_t)t < Wo) ocarry[t] = c;
            }
            __syncthreads();
            stamp(5);
            // 3. source map: every output byte's literal byte, or an earlier
            //    output byte (4 consecutive bytes per thread, interleaved)
            for (uint32_t q0 = (uint32_t)t * 4; q0 < n; q0 += kT * 4) {
                for (uint32_t q = q0; q < q0 + 4 && q < n; ++q) {
                    const uint32_t w = q >> 6, b = q & 63;
                    const uint64_t mine = sb[w] & (b == 63 ? ~0ull : ((2ull << b) - 1));
                    const uint32_t s = (mine ? w * 64 + 64 - (uint32_t)__builtin_clzll(mine) : ocarry[w]) - 1;
                    const uint32_t d = desc[s];
                    src[q] = (uint16_t)((d & 0x8000u) ? (0x8000u | ((d & 0x7FFFu) + (q - s))) : (q - d));
                }
            }
            __syncthreads();
            stamp(6);
            // pointer jumping: every copy byte ends at a literal byte
            for (;;) {
                bool more = false;
                for (uint32_t q0 = (uint32_t)t * 4; q0 < n; q0 += kT * 4) {
                    for (uint32_t q = q0; q < q0 + 4 && q < n; ++q) {
                        const uint32_t v = src[q];
                        if (!(v & 0x8000u)) {
                            const uint32_t w = src[v];
                            src[q] = (uint16_t)w;
                            more |= !(w & 0x8000u);
                        }
                    }
                }
                if (!__syncthreads_or(more)) break;
            }
            stamp(7);
            // gather + store, 4 bytes per thread and store
            gbyte* d = (gbyte*)pc.dst;
            const bool al = (reinterpret_cast<uintptr_t>(pc.dst) & 3) == 0;
            for (uint32_t q0 = (uint32_t)t * 4; q0 < n; q0 += kT * 4) {
                if (al && q0 + 4 <= n) {
                    uint32_t x = 0;
#pragma unroll
                    for (int j = 0; j < 4; ++j) x |= (uint32_t)cin[src[q0 + j] & 0x7FFFu] << (8 * j);
                    *reinterpret_cast<__attribute__((address_space(1))) uint32_t*>(d + q0) = x;
                } else {
                    for (uint32_t q = q0; q < q0 + 4 && q < n; ++q) d[q] = cin[src[q] & 0x7FFFu];
                }
            }
            stamp(8);
        }
    }
    __syncthreads();
    if (t == 0) a.piece_err[job] = !fits ? (n == 0 ? 0 : 1) : bad;
    // the message is complete when its last piece is: that workgroup scans it
    const uint32_t g = a.piece_group ? a.piece_group[job] : kFusedNoGroup;
    if (g == kFusedNoGroup) return;
    __shared__ int last;
    __threadfence();  // this piece's bytes before the count
    __syncthreads();
    if (t == 0) {
        const uint32_t prev = atomicAdd(&a.group_done[g], 1u);
        last = prev + 1 == a.group_pieces[g];
    }
    __syncthreads();
    if (!last) return;
    __threadfence();  // every other piece's bytes after the count
    if (t == 0) {
        a.group_done[g] = 0;  // reusable by the next launch of this batch
        const PbScanJob sj = a.scans[g];
        a.scan_n[g] = devpb::scan_message((devpb::gbyte_c*)sj.buf, 0, sj.len,
                                          a.scan_fields + (uint64_t)g * a.max_fields * 2, a.max_fields);
    }
}

__global__ void __launch_bounds__(kT) codec_fused_kernel(FusedCodecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int b = blockIdx.x;
    if (b < a.ncomp) {
        compress_block(a, b, lds);
    } else {
        decode_piece(a, b - a.ncomp, lds);
    }
}

}  // namespace

int LaunchFusedCodec(const FusedCodecArgs& a, hipStream_t s) {
    const int n = a.ncomp + a.npieces;
    if (n <= 0) return 0;
    if (a.max_ulen == 0 || a.max_ulen > kFusedMaxBlock) return -1;
    const uint32_t C = (a.max_ulen + 15) & ~15u;
    const uint32_t lds = std::max(a.ncomp ? CompressLds(C) : 0u, a.npieces ? DecodeLds(C) : 0u);
    hipLaunchKernelGGL(codec_fused_kernel, dim3((unsigned)n), dim3(kT), lds, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace gpu
}  // namespace mrpc
