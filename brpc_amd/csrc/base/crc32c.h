// CRC32C (Castagnoli). Role of butil/crc32c.h (reference
// src/butil/crc32c.cc:17,25-349). Host path uses SSE4.2 crc32q when the CPU
// has it (runtime-detected) or slicing-by-8 tables. Combine() joins CRCs of
// adjacent pieces in O(log n) via GF(2) polynomial arithmetic, which is what
// lets the HIP kernel (ops/crc32c_mfma.hip) checksum chunks independently and
// fold them on device.
#pragma once

#include <cstddef>
#include <cstdint>

namespace mrpc {
namespace crc32c {

// Extend a finalized crc with more data (Value(a+b) == Extend(Value(a), b)).
uint32_t Extend(uint32_t init_crc, const void* data, size_t n);
inline uint32_t Value(const void* data, size_t n) { return Extend(0, data, n); }
// crc(A || B) from crc(A), crc(B), len(B)
uint32_t Combine(uint32_t crc_a, uint32_t crc_b, size_t len_b);
// Raw (non-inverted) register update used by GPU kernels / tests.
uint32_t ExtendRaw(uint32_t reg, const void* data, size_t n);
// x^(8*n) mod P as a reflected polynomial; multiplies the register for a
// shift of n zero bytes.
uint32_t ShiftBytesPoly(size_t n);
uint32_t MultModP(uint32_t a, uint32_t b);
bool HasHardwareSupport();

}  // namespace crc32c
}  // namespace mrpc
