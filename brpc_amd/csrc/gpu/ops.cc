// Synchronous (fiber-friendly) wrappers over the kernels in kernels.hip.
#include <hip/hip_runtime_api.h>

#include <vector>

#include "base/crc32c.h"
#include "gpu/hbm_pool.h"
#include "gpu/kernels.h"

namespace mrpc {
namespace gpu {

int Crc32cDevice(const void* const* ptrs, const uint64_t* lens, int n, uint32_t* out_host, int device) {
    if (n <= 0) return 0;
    if (Init(device) != 0) return -1;
    if (device < 0) device = CurrentDevice();
    int prev = 0;
    hipGetDevice(&prev);
    if (prev != device) hipSetDevice(device);
    // one device allocation: [starts n][lens n][scratch n+1][out n (u32)]
    std::vector<uint64_t> desc(2 * (size_t)n);
    uint64_t total = 0, maxlen = 0;
    for (int i = 0; i < n; ++i) {
        desc[i] = reinterpret_cast<uint64_t>(ptrs[i]);
        desc[n + i] = lens[i];
        total += lens[i];
        if (lens[i] > maxlen) maxlen = lens[i];
    }
    const size_t desc_bytes = desc.size() * sizeof(uint64_t);
    const size_t bytes = desc_bytes + Crc32cScratchBytes(n) + sizeof(uint32_t) * n;
    int rc = -1;
    // pooled scratch: a hipFree here would synchronise the whole device
    char* mem = static_cast<char*>(HbmAlloc(bytes, device));
    hipStream_t s = PoolStream(device);
    if (mem && s) {
        uint64_t* d_starts = reinterpret_cast<uint64_t*>(mem);
        uint64_t* d_lens = d_starts + n;
        void* scratch = mem + desc_bytes;
        uint32_t* out_dev = reinterpret_cast<uint32_t*>(mem + desc_bytes + Crc32cScratchBytes(n));
        if (hipMemcpyAsync(d_starts, desc.data(), desc_bytes, hipMemcpyHostToDevice, s) == hipSuccess &&
            LaunchCrc32cSegments(d_starts, d_lens, n, total, maxlen, out_dev, scratch, s) == 0 &&
            hipMemcpyAsync(out_host, out_dev, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, s) == hipSuccess) {
            rc = SyncStream(s);
        }
    }
    if (mem && rc != 0 && s) SyncStream(s);  // never recycle scratch a launch may still use
    HbmFree(mem, bytes, device);
    if (prev != device) hipSetDevice(prev);
    return rc;
}

int Crc32cOfBuf(const Buf& b, uint32_t* out, int device) {
    // host blocks are folded on the CPU (SSE4.2), device blocks on the GPU;
    // the pieces are joined with crc32c::Combine in order.
    uint32_t crc = 0;
    size_t i = 0;
    const size_t nb = b.backing_block_num();
    while (i < nb) {
        const BlockRef& r = b.ref_at(i);
        if (IsHostAccessible(r.block->kind)) {
            crc = crc32c::Extend(crc, r.block->data + r.offset, r.length);
            ++i;
            continue;
        }
        // a run of device blocks: one launch
        std::vector<const void*> ptrs;
        std::vector<uint64_t> lens;
        int dev = r.block->device;
        while (i < nb && !IsHostAccessible(b.ref_at(i).block->kind) && b.ref_at(i).block->device == dev) {
            ptrs.push_back(b.ref_at(i).block->data + b.ref_at(i).offset);
            lens.push_back(b.ref_at(i).length);
            ++i;
        }
        std::vector<uint32_t> crcs(ptrs.size());
        if (Crc32cDevice(ptrs.data(), lens.data(), (int)ptrs.size(), crcs.data(), dev) != 0) return -1;
        for (size_t k = 0; k < crcs.size(); ++k) crc = crc32c::Combine(crc, crcs[k], lens[k]);
    }
    *out = crc;
    return 0;
}

}  // namespace gpu
}  // namespace mrpc
