// Device-side protobuf wire walk shared by the gfx950 kernels that index
// messages (pb_kernels.hip: the batched scans; snappy_kernels.hip: the scan
// a fused codec launch runs once the last piece of a message is decoded).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mrpc {
namespace gpu {
namespace devpb {

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

}  // namespace devpb
}  // namespace gpu
}  // namespace mrpc
