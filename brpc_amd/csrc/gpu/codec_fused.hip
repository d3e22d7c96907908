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

constexpr int kT = 256;  // threads per workgroup
constexpr int kWaves = kT / 64;
constexpr int kTableBits = 12;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kWalkSeg = 64;                            // positions (or compressed bytes) per walk segment
constexpr uint32_t kCompSegs = kFusedMaxBlock / kWalkSeg;    // 128
static_assert(kCompSegs <= (uint32_t)kT, "one walker thread per segment");

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

template <typename Op>
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, Op op) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)v, (unsigned)o, 64);
        if (lane >= o) v = op(y, v);
    }
    return v;
}

// Block-wide exclusive scan (identity for thread 0); *total = the reduction.
// wtot: kWaves words of LDS. Ends with a barrier, so wtot may be reused.
template <typename Op>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t identity, Op op, uint32_t* wtot,
                                                    uint32_t* total) {
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const uint32_t incl = wave_incl_scan(v, op);
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

// ---------------------------------------------------------------- compress
// LDS: in (C + 96, 16 B of alignment slack + 80 B of zero pad) | L (C) |
// cand (2C) | NC (2C + 16) | table (16 KiB, later the output stage) |
// wtot (kWaves) | xch (kT) | ex (kT) | segruns (u64 x kCompSegs) | segcarry
__host__ __device__ constexpr uint32_t CompressLds(uint32_t C) {
    return (C + 96) + C + 2 * C + (2 * C + 16) + (4u << kTableBits) + 4 * (kWaves + 2 * kT) + 8 + 12 * kCompSegs +
           64;
}

__device__ void compress_block(const FusedCodecArgs& a, int job, uint8_t* lds) {
    const int t = threadIdx.x;
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
    uint16_t* NC = cand + C;
    uint32_t* table = reinterpret_cast<uint32_t*>(NC + C + 8);
    uint8_t* stage = reinterpret_cast<uint8_t*>(table);
    uint32_t* wtot = table + (1u << kTableBits);
    uint32_t* xch = wtot + kWaves;
    uint32_t* ex = xch + kT;
    uint64_t* segruns = reinterpret_cast<uint64_t*>(ex + kT + 2);  // 8-byte aligned: 6C + 112 + 16 KiB + 4 * (516 + 2)
    uint32_t* segcarry = reinterpret_cast<uint32_t*>(segruns + kCompSegs);

    for (uint32_t i = t; i < (1u << kTableBits); i += kT) table[i] = kNone;
    const uint32_t mis = stage_in(jb.src, n, raw, 80);
    const uint8_t* in = raw + mis;
    const uint32_t G = (n + kT - 1) / kT;  // segment = the thread's positions, <= 32
    const uint32_t lo = min(n, G * (uint32_t)t), hi = min(n, lo + G);
    __syncthreads();
    // 1. earliest position of every hash
    for (uint32_t p = lo; p < hi && p + 4 <= n; ++p) atomicMin(&table[hash4(rd32(raw, mis + p))], p);
    __syncthreads();
    // 2. candidates and match lengths (<= 64, one copy element)
    uint32_t first = n;
    for (uint32_t p = lo; p < hi; ++p) {
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
        L[p] = (uint8_t)l;
        cand[p] = (uint16_t)c;
        if (l >= 4 && first == n) first = p;
    }
    // NC[p]: the first match position >= p (n: none)
    {
        uint32_t carry = block_excl_suffix(first, n, OpMin(), wtot, xch);
        for (uint32_t p = hi; p-- > lo;) {
            if (L[p] >= 4) carry = p;
            NC[p] = (uint16_t)carry;
        }
        if (t == 0) NC[n] = (uint16_t)n;
    }
    __syncthreads();
    // 3. the greedy parse: speculative walks over 64-position segments (one
    //    thread each), re-walked until every segment's entry is its
    //    predecessor's exit. A segment this long holds several elements, so
    //    walks from different entries meet inside it and the corrections
    //    stop after a few rounds instead of crawling one segment per round.
    const uint32_t S = (n + kWalkSeg - 1) / kWalkSeg;
    const bool walker = (uint32_t)t < S;
    const uint32_t wlo = walker ? (uint32_t)t * kWalkSeg : n, whi = walker ? min(n, wlo + kWalkSeg) : n;
    uint32_t entry = wlo;
    uint64_t mask = 0;
    auto walk = [&](uint32_t e) -> uint32_t {
        mask = 0;
        while (e < whi) {
            mask |= 1ull << (e - wlo);
            const uint32_t l = L[e];
            e = l >= 4 ? e + l : NC[e + 1];
        }
        return e;
    };
    uint32_t exitp = walker ? walk(entry) : n;
    if (walker) ex[t] = exitp;
    uint32_t rounds = 0;
    for (;;) {
        __syncthreads();
        const uint32_t want = walker ? (t ? ex[t - 1] : 0u) : entry;
        __syncthreads();
        bool moved = false;
        if (want != entry) {
            entry = want;
            const uint32_t e = walk(entry);
            moved = e != exitp;
            exitp = e;
            ex[t] = e;
        }
        ++rounds;
        if (!__syncthreads_or(moved)) break;
    }
    if (a.stats && t == 0) {
        atomicAdd(&a.stats[0], rounds);
        atomicMax(&a.stats[1], rounds);
    }
    // 4. sizes, offsets, tags (the walkers); literal bytes (everyone)
    uint32_t out = 0;
    for (uint64_t m = mask; m; m &= m - 1) {
        const uint32_t p = wlo + (uint32_t)__builtin_ctzll(m);
        const uint32_t l = L[p];
        if (l >= 4) {
            out += (l < 12 && p - cand[p] < 2048) ? 2 : 3;
        } else {
            const uint32_t ll = NC[p + 1] - p;
            out += lit_tag_bytes(ll) + ll;
        }
    }
    uint32_t body;
    const uint32_t base = block_excl_scan(out, 0u, OpSum(), wtot, &body);
    const uint32_t hdr = varint_len(n);
    const uint32_t total = hdr + body;
    if (total > jb.dst_cap || total > (4u << kTableBits)) {  // block-uniform
        if (t == 0) {
            a.comp_err[job] = 2;
            a.comp_len[job] = 0;
        }
        return;
    }
    // (the table is free: the last reads of it were before the barriers above)
    uint32_t o = hdr + base;
    uint64_t runs = 0;
    for (uint64_t m = mask; m; m &= m - 1) {
        const uint32_t b = (uint32_t)__builtin_ctzll(m);
        const uint32_t p = wlo + b;
        const uint32_t l = L[p];
        if (l >= 4) {
            const uint32_t off = p - cand[p];
            if (l < 12 && off < 2048) {
                stage[o] = (uint8_t)(((off >> 8) << 5) | ((l - 4) << 2) | 1);
                stage[o + 1] = (uint8_t)off;
                o += 2;
            } else {
                stage[o] = (uint8_t)(((l - 1) << 2) | 2);
                stage[o + 1] = (uint8_t)off;
                stage[o + 2] = (uint8_t)(off >> 8);
                o += 3;
            }
        } else {
            const uint32_t ll = NC[p + 1] - p, v = ll - 1;
            if (ll <= 60) {
                stage[o++] = (uint8_t)(v << 2);
            } else if (ll <= 256) {
                stage[o] = 60 << 2;
                stage[o + 1] = (uint8_t)v;
                o += 2;
            } else {
                stage[o] = 61 << 2;
                stage[o + 1] = (uint8_t)v;
                stage[o + 2] = (uint8_t)(v >> 8);
                o += 3;
            }
            cand[p] = (uint16_t)o;  // where the run's bytes go (cand is unused at literals)
            o += ll;
            runs |= 1ull << b;
        }
    }
    if (t < (int)hdr) stage[t] = (uint8_t)(((n >> (7 * t)) & 0x7f) | (t + 1 < (int)hdr ? 0x80 : 0));
    // the run in force at p: the latest run start <= p (segment masks, and
    // a block max-scan of each segment's last run start + 1 for the carry)
    uint32_t tot;
    const uint32_t carry =
        block_excl_scan(runs ? wlo + 64 - (uint32_t)__builtin_clzll(runs) : 0u, 0u, OpMax(), wtot, &tot);
    if (walker) {
        segruns[t] = runs;
        segcarry[t] = carry;
    }
    __syncthreads();
    for (uint32_t p = lo; p < hi; ++p) {
        const uint32_t w = p / kWalkSeg, b = p % kWalkSeg;
        const uint64_t mine = segruns[w] & (b == 63 ? ~0ull : ((2ull << b) - 1));
        const uint32_t r1 = mine ? w * kWalkSeg + 64 - (uint32_t)__builtin_clzll(mine) : segcarry[w];
        if (r1 == 0) continue;
        const uint32_t r = r1 - 1;
        if (p < NC[r + 1]) stage[cand[r] + (p - r)] = in[p];
    }
    __syncthreads();
    store_out(jb.dst, stage, total);
    if (t == 0) {
        a.comp_len[job] = total;
        a.comp_err[job] = 0;
    }
}

// ---------------------------------------------------------------- decode
// LDS: cin (cap + 32 + 96) | desc (2C) | src (2C) | sbits (C/8 + 16) |
// wtot | xch | ex (u32 x kT, exits as u32) | flag
__host__ __device__ constexpr uint32_t DecodeCinCap(uint32_t C) {
    return (uint32_t)((SnappyMaxCompressedLength(C) + 15) & ~15ull);
}
__host__ __device__ constexpr uint32_t DecodeLds(uint32_t C) {
    return DecodeCinCap(C) + 128 + 2 * C + 2 * C + (C / 8 + 16) + 4 * (kWaves + 2 * kT) + 64;
}

__device__ void decode_piece(const FusedCodecArgs& a, int job, uint8_t* lds) {
    const int t = threadIdx.x;
    const SnappyPiece pc = a.pieces[job];
    const uint32_t C = (a.max_ulen + 15) & ~15u;
    const uint32_t m = pc.src_len, n = pc.ulen;
    uint8_t* raw = lds;
    uint16_t* desc = reinterpret_cast<uint16_t*>(raw + DecodeCinCap(C) + 128);
    uint16_t* src = desc + C;
    uint32_t* sbits = reinterpret_cast<uint32_t*>(src + C);
    uint32_t* wtot = sbits + C / 32 + 4;
    uint32_t* xch = wtot + kWaves;
    uint32_t* ex = xch + kT;
    __shared__ int bad;
    if (t == 0) bad = 0;
    const bool fits = n <= a.max_ulen && m <= DecodeCinCap(C) && n > 0 && m > 0;
    if (fits) {
        for (uint32_t i = t; i < C / 32 + 1; i += kT) sbits[i] = 0;
        const uint32_t mis = stage_in(pc.src, m, raw, 16);
        const uint8_t* cin = raw + mis;
        __syncthreads();
        // 1. the element chain over the compressed bytes: speculative walks
        //    over 64-byte segments, re-walked until the entries agree
        const uint32_t S = (m + kWalkSeg - 1) / kWalkSeg;  // <= 150 for 8 KiB pieces
        const bool walker = (uint32_t)t < S;
        const uint32_t lo = walker ? (uint32_t)t * kWalkSeg : m, hi = walker ? min(m, lo + kWalkSeg) : m;
        auto csize = [&](uint32_t i) -> uint32_t {
            const uint32_t tag = cin[i];
            const uint32_t kind = tag & 3;
            if (kind == 1) return 2;
            if (kind == 2) return 3;
            if (kind == 3) return 5;
            uint32_t len = (tag >> 2) + 1, h = 1;
            if (len > 60) {
                const uint32_t nb = len - 60;
                const uint32_t raw_len = rd32(raw, mis + i + 1) & (0xFFFFFFFFu >> (32 - 8 * nb));
                if (raw_len >= 0x7FFF0000u) return 0x7FFF0000u;  // far past any piece
                len = raw_len + 1;
                h += nb;
            }
            return h + len;
        };
        uint64_t mask = 0;
        uint32_t entry = lo;
        auto walk = [&](uint32_t e) -> uint32_t {
            mask = 0;
            while (e < hi) {
                mask |= 1ull << (e - lo);
                e = min(e + csize(e), 0x7FFF0000u);
            }
            return e;
        };
        uint32_t exitp = walker ? walk(entry) : m;
        if (walker) ex[t] = exitp;
        uint32_t rounds = 0;
        for (;;) {
            __syncthreads();
            const uint32_t want = walker ? (t ? ex[t - 1] : 0u) : entry;
            __syncthreads();
            bool moved = false;
            if (want != entry) {
                entry = want;
                const uint32_t e = walk(entry);
                moved = e != exitp;
                exitp = e;
                ex[t] = e;
            }
            ++rounds;
            if (!__syncthreads_or(moved)) break;
        }
        if (a.stats && t == 0) {
            atomicAdd(&a.stats[2], rounds);
            atomicMax(&a.stats[3], rounds);
        }
        if ((uint32_t)t == S - 1 && exitp != m) bad = 3;  // the chain must end exactly at the piece's end
        // 2. output sizes -> positions; descriptors at element starts
        auto elem = [&](uint32_t i, uint32_t* len, uint32_t* off, uint32_t* lsrc) {
            const uint32_t tag = cin[i];
            const uint32_t kind = tag & 3;
            if (kind == 0) {
                uint32_t l = (tag >> 2) + 1, h = 1;
                if (l > 60) {
                    const uint32_t nb = l - 60;
                    l = (rd32(raw, mis + i + 1) & (0xFFFFFFFFu >> (32 - 8 * nb))) + 1;
                    h += nb;
                }
                *len = l;
                *off = 0;
                *lsrc = i + h;
            } else if (kind == 1) {
                *len = ((tag >> 2) & 7) + 4;
                *off = ((tag >> 5) << 8) | cin[i + 1];
            } else if (kind == 2) {
                *len = (tag >> 2) + 1;
                *off = cin[i + 1] | ((uint32_t)cin[i + 2] << 8);
            } else {
                *len = (tag >> 2) + 1;
                *off = rd32(raw, mis + i + 1);
            }
        };
        uint32_t outb = 0;
        for (uint64_t k = mask; k; k &= k - 1) {
            uint32_t len, off, ls = 0;
            elem(lo + (uint32_t)__builtin_ctzll(k), &len, &off, &ls);
            outb = min(outb + len, 0x7FFF0000u);
        }
        uint32_t total;
        uint32_t o = block_excl_scan(outb, 0u, OpSum(), wtot, &total);
        // (the scan's barriers publish `bad`: a broken chain's sizes are
        // garbage, so nothing below is written unless the chain is sound)
        if (bad || total != n) {
            if (t == 0 && !bad) bad = 4;
        } else {
            for (uint64_t k = mask; k; k &= k - 1) {
                uint32_t len, off, ls = 0;
                const uint32_t i = lo + (uint32_t)__builtin_ctzll(k);
                elem(i, &len, &off, &ls);
                if (off == 0 && (cin[i] & 3) == 0) {
                    desc[o] = (uint16_t)(0x8000u | ls);
                } else if (off == 0 || off > o) {
                    atomicOr(&bad, 6);  // a copy from before the piece
                    desc[o] = 0x8000u;
                } else {
                    desc[o] = (uint16_t)off;
                }
                atomicOr(&sbits[o >> 5], 1u << (o & 31));
                o += len;
            }
        }
        __syncthreads();
        if (bad == 0) {
            // every output byte's element: the latest start <= it (thread t
            // owns output word t: bytes [32t, 32t + 32))
            const uint32_t ob = 32u * (uint32_t)t, oe = min(n, ob + 32);
            const uint32_t bits = ob < n ? sbits[t] : 0u;
            uint32_t tot;
            const uint32_t carry =
                block_excl_scan(bits ? ob + 32 - (uint32_t)__builtin_clz(bits) : 0u, 0u, OpMax(), wtot, &tot);
            for (uint32_t q = ob; q < oe; ++q) {
                const uint32_t b = q - ob;
                const uint32_t mine = bits & (b == 31 ? 0xFFFFFFFFu : ((2u << b) - 1));
                const uint32_t s = (mine ? ob + 32 - (uint32_t)__builtin_clz(mine) : carry) - 1;
                const uint32_t d = desc[s];
                src[q] = (uint16_t)((d & 0x8000u) ? (0x8000u | ((d & 0x7FFFu) + (q - s))) : (q - d));
            }
            __syncthreads();
            // 3. pointer jumping: every copy byte ends at a literal byte
            for (;;) {
                bool more = false;
                for (uint32_t q = ob; q < oe; ++q) {
                    const uint32_t v = src[q];
                    if (!(v & 0x8000u)) {
                        const uint32_t w = src[v];
                        src[q] = (uint16_t)w;
                        more |= !(w & 0x8000u);
                    }
                }
                if (!__syncthreads_or(more)) break;
            }
            // gather: one 32-byte run of the output per thread
            if (ob < n) {
                gbyte* d = (gbyte*)pc.dst + ob;
                const uint32_t cnt = oe - ob;
                if (cnt == 32 && (reinterpret_cast<uintptr_t>(pc.dst) & 15) == 0) {
                    uint32_t w[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        uint32_t x = 0;
#pragma unroll
                        for (int j = 0; j < 4; ++j) x |= (uint32_t)cin[src[ob + 4 * k + j] & 0x7FFFu] << (8 * j);
                        w[k] = x;
                    }
                    auto* dv = reinterpret_cast<__attribute__((address_space(1))) u32x4*>(d);
                    dv[0] = u32x4{w[0], w[1], w[2], w[3]};
                    dv[1] = u32x4{w[4], w[5], w[6], w[7]};
                } else {
                    for (uint32_t q = 0; q < cnt; ++q) d[q] = cin[src[ob + q] & 0x7FFFu];
                }
            }
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
