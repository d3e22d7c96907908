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

namespace mrpc {
namespace gpu {

namespace {

typedef const __attribute__((address_space(1))) uint8_t gbyte_c;

__device__ __forceinline__ bool read_varint(gbyte_c* b, uint64_t& p, uint64_t end, uint64_t& v) {
    v = 0;
    for (int shift = 0; shift < 70; shift += 7) {
        if (p >= end) return false;
        const uint64_t c = b[p++];
        v |= (c & 0x7f) << shift;
        if (!(c & 0x80)) return shift < 63 || c <= 1;  // 10th byte may only carry bit 63
    }
    return false;
}

// Walks one message b[start, end) into row (max_fields {tag, value} pairs);
// returns the field count or a negative code.
__device__ __forceinline__ int32_t scan_message(gbyte_c* b, uint64_t start, uint64_t end, uint64_t* row,
                                                uint32_t max_fields) {
    uint64_t p = start;
    int32_t k = 0;
    int32_t status = 0;
    while (p < end) {
        uint64_t tag;
        if (!read_varint(b, p, end, tag) || tag > 0xFFFFFFFFull) {
            status = -1;
            break;
        }
        const uint32_t field = (uint32_t)(tag >> 3), wire = (uint32_t)(tag & 7);
        if (field == 0) {
            status = -3;
            break;
        }
        uint64_t value = 0;
        if (wire == 0) {
            if (!read_varint(b, p, end, value)) {
                status = -1;
                break;
            }
        } else if (wire == 1 || wire == 5) {
            const uint64_t nb = wire == 1 ? 8 : 4;
            if (end - p < nb) {
                status = -1;
                break;
            }
            for (uint64_t j = 0; j < nb; ++j) value |= (uint64_t)b[p + j] << (8 * j);
            p += nb;
        } else if (wire == 2) {
            uint64_t len;
            if (!read_varint(b, p, end, len) || len > end - p || len > 0xFFFFFFFFull) {
                status = -1;
                break;
            }
            value = ((p - start) << 32) | len;
            p += len;
        } else {
            status = -4;
            break;
        }
        if ((uint32_t)k >= max_fields) {
            status = -2;
            break;
        }
        typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
        u64x2 v;
        v.x = tag;
        v.y = value;
        *reinterpret_cast<u64x2*>(row + 2 * k) = v;
        ++k;
    }
    return status ? status : k;
}

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
    nfields[i] = scan_message(b, start, end, fields + (uint64_t)i * max_fields * 2, max_fields);
}

// Messages in separate buffers (one per job): the batched codec path, where
// every request decoded its body into its own HBM block.
__global__ void __launch_bounds__(256) pb_scan_ptrs_kernel(const PbScanJob* __restrict__ jobs, int64_t n,
                                                           uint32_t max_fields, uint64_t* __restrict__ fields,
                                                           int32_t* __restrict__ nfields) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const PbScanJob job = jobs[i];
    nfields[i] = scan_message((gbyte_c*)job.buf, 0, job.len, fields + (uint64_t)i * max_fields * 2, max_fields);
}

}  // namespace

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
