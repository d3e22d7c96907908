// Batched snappy decompression on CDNA4 (gfx950) — the device half of the
// snappy body codec (reference: policy/snappy_compress.cpp:28-64 over
// butil/third_party/snappy; SURVEY K3 "per-64 KB-block CTA kernel").
//
// Layout: every input is an independent raw snappy stream whose
// uncompressed size is <= kSnappyMaxBlock (64 KiB) — the sender splits
// device payloads into such blocks, the same unit snappy's own compressor
// matches within. The job table (src, dst, lengths) lives in device memory,
// so one launch covers any number of blocks. One wave64 workgroup owns one
// block and rebuilds it in LDS (64 KiB of the CU's 160 KiB: 2 blocks per CU
// resident), then streams it to HBM with 16-byte coalesced stores.
//
// The tag stream is inherently serial, so the whole wave walks it in
// lockstep: the tag bytes are wave-uniform (every lane loads the same
// address, one cache line), and each element is materialised by all 64
// lanes at once:
//   literal          out[pos + j] = in[src + j]                  (j = lane, lane+64, ...)
//   copy, off >= len out[pos + j] = out[pos - off + j]
//   copy, off <  len out[pos + j] = out[pos - off + (j % off)]    (the repeating
//                    pattern is read from bytes that already exist, so even an
//                    overlapping copy is one parallel step, not a byte loop)
// LDS accesses of one wave execute in order; a wave-scope fence between
// elements keeps the compiler from reordering them.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "gpu/kernels.h"

namespace mrpc {
namespace gpu {

namespace {

constexpr int kWave = 64;

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ void __launch_bounds__(kWave) snappy_decompress_kernel(const SnappyJob* __restrict__ jobs, int n,
                                                                  uint32_t* __restrict__ out_len,
                                                                  int* __restrict__ err) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[kSnappyMaxBlock];
    const int blk = blockIdx.x;
    if (blk >= n) return;
    const int lane = threadIdx.x;
    const SnappyJob job = jobs[blk];
    const uint8_t* in = static_cast<const uint8_t*>(job.src);
    const uint32_t in_len = (uint32_t)job.src_len;
    // uncompressed length (varint, <= 5 bytes)
    uint32_t ulen = 0, ip = 0;
    int bad = 0;
    for (int shift = 0;; shift += 7) {
        if (ip >= in_len || shift >= 35) {
            bad = 1;
            break;
        }
        const uint32_t c = in[ip++];
        ulen |= (c & 0x7f) << shift;
        if (!(c & 0x80)) break;
    }
    if (!bad && (ulen > kSnappyMaxBlock || ulen > job.dst_cap)) bad = 2;
    uint32_t op = 0;
    while (!bad && ip < in_len) {
        const uint32_t tag = in[ip++];
        const uint32_t kind = tag & 3;
        if (kind == 0) {
            uint32_t len = (tag >> 2) + 1;
            if (len > 60) {
                const uint32_t nb = len - 60;  // 1..4 little-endian length bytes
                if (ip + nb > in_len) {
                    bad = 3;
                    break;
                }
                uint32_t l = 0;
                for (uint32_t k = 0; k < nb; ++k) l |= (uint32_t)in[ip + k] << (8 * k);
                ip += nb;
                len = l + 1;
            }
            if (len > in_len - ip || len > ulen - op) {
                bad = 4;
                break;
            }
            for (uint32_t j = lane; j < len; j += kWave) buf[op + j] = in[ip + j];
            ip += len;
            op += len;
        } else {
            uint32_t len, off;
            const uint32_t need = kind == 1 ? 1 : (kind == 2 ? 2 : 4);
            if (ip + need > in_len) {
                bad = 5;
                break;
            }
            if (kind == 1) {
                len = ((tag >> 2) & 7) + 4;
                off = ((tag >> 5) << 8) | in[ip];
            } else if (kind == 2) {
                len = (tag >> 2) + 1;
                off = (uint32_t)in[ip] | ((uint32_t)in[ip + 1] << 8);
            } else {
                len = (tag >> 2) + 1;
                off = (uint32_t)in[ip] | ((uint32_t)in[ip + 1] << 8) | ((uint32_t)in[ip + 2] << 16) |
                      ((uint32_t)in[ip + 3] << 24);
            }
            ip += need;
            if (off == 0 || off > op || len > ulen - op) {
                bad = 6;
                break;
            }
            const uint32_t from = op - off;
            if (off >= len) {
                for (uint32_t j = lane; j < len; j += kWave) buf[op + j] = buf[from + j];
            } else {
                for (uint32_t j = lane; j < len; j += kWave) buf[op + j] = buf[from + j % off];
            }
            op += len;
        }
        wave_sync();
    }
    if (!bad && op != ulen) bad = 7;
    if (bad) {
        if (lane == 0) {
            err[blk] = bad;
            out_len[blk] = 0;
        }
        return;
    }
    wave_sync();
    // LDS -> HBM, 16 B per lane per step (1 KiB per wave instruction)
    uint8_t* dst = static_cast<uint8_t*>(job.dst);
    const bool aligned = ((uintptr_t)dst & 15) == 0;
    const uint32_t vec_end = aligned ? (ulen & ~15u) : 0;
    for (uint32_t o = lane * 16; o < vec_end; o += kWave * 16) {
        *reinterpret_cast<uint4*>(dst + o) = *reinterpret_cast<const uint4*>(buf + o);
    }
    for (uint32_t o = vec_end + lane; o < ulen; o += kWave) dst[o] = buf[o];
    if (lane == 0) {
        out_len[blk] = ulen;
        err[blk] = 0;
    }
}

}  // namespace

int LaunchSnappyDecompress(const SnappyJob* jobs_dev, int n, uint32_t* out_len_dev, int* err_dev, hipStream_t s) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(snappy_decompress_kernel, dim3(n), dim3(kWave), 0, s, jobs_dev, n, out_len_dev, err_dev);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace gpu
}  // namespace mrpc
