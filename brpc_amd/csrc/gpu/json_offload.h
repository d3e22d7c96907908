// GPU structural index for large JSON bodies (see json_offload.cc):
// installs gpu::JsonIndex behind json2pb's SetJsonIndexOffload for bodies of
// at least min_bytes, so http+json and json2pb parses cut strings at
// device-found quotes instead of scanning them.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace mrpc {
namespace gpu {

int EnableGpuJsonIndex(int device, size_t min_bytes, std::string* error = nullptr);
void DisableGpuJsonIndex();

// Synchronous structural index of host bytes on `device` (fiber-friendly
// wait): ascending offsets of unescaped quotes and of {}[]:, outside
// strings. -1 on a device error or an unterminated string.
int JsonIndex(const char* data, size_t n, std::vector<uint32_t>* out, int device);

struct GpuJsonStats {
    int64_t indexed_bodies = 0, indexed_bytes = 0, failures = 0;
    int64_t pb2json_arrays = 0, pb2json_elems = 0, pb2json_failures = 0;  // number arrays printed on the device
    int64_t int_arrays = 0, int_array_fallbacks = 0;  // json2pb integer arrays parsed on the device
    int64_t sparse_skips = 0;  // bodies left to the host parser by the density check
};
GpuJsonStats GetGpuJsonStats();

}  // namespace gpu
}  // namespace mrpc
