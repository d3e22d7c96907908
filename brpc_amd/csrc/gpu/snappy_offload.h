// GPU snappy offload for RPC bodies (see snappy_offload.cc): installs the
// device codec behind rpc/compress.h's snappy handler for bodies of at
// least min_bytes. Standard raw snappy on the wire; anything the device
// path cannot take (a stream it cannot cut, HBM blocks of another GPU)
// falls back to the CPU codec.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

namespace mrpc {
namespace gpu {

int EnableGpuSnappy(int device, size_t min_bytes, std::string* error = nullptr);
void DisableGpuSnappy();

struct GpuSnappyStats {
    int64_t compress_calls = 0, decompress_calls = 0, fallbacks = 0;
    int64_t indexed_parses = 0, index_fallbacks = 0;  // decompress + pb_scan parses
    int64_t packs = 0;  // bodies serialized straight into pinned memory and compressed there
    int64_t pack_runs = 0, pack_run_chunks = 0;  // packed fields those bodies left to pb_run_encode_kernel
    int64_t unpack_runs = 0, unpack_fallbacks = 0;  // packed fields of decoded bodies parsed on the device
    int64_t plain_routed = 0;  // -gpu_snappy_packed_only: plain bodies left to the CPU codec
};
GpuSnappyStats GetGpuSnappyStats();

// One numeric run through pb_run_encode_kernel (gpu/kernels.h PbRunKind /
// PbRunFormat) via the codec batch: `values` in the field's vector layout,
// `out` the varint payload or the JSON number list. 0 on success.
int EncodeRunOnDevice(const void* values, size_t n, uint32_t kind, uint32_t format, std::string* out, int device);
// A packed varint payload -> elements in the kind's vector layout
// (pb_run_count/decode kernels). -1 when malformed or on a device error.
int DecodeRunOnDevice(const void* bytes, size_t len, uint32_t kind, std::string* out, int device);

}  // namespace gpu
}  // namespace mrpc
