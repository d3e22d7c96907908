#include "gpu/device_handler.h"

#include <cstring>
#include <memory>
#include <vector>

#include "base/crc32c.h"
#include "gpu/copy_engine.h"
#include "gpu/gpu.h"
#include "gpu/hbm_pool.h"
#include "fiber/fiber.h"

namespace mrpc {
namespace gpu {

namespace {
void pinned_deleter(void* p, void* arg) { PinnedFree(p, (size_t)reinterpret_cast<uintptr_t>(arg)); }
}  // namespace

namespace {

// One copy+CRC32C pass of `in` into the contiguous destination `d` (null:
// checksum only).
int copy_with_crc(const Buf& in, char* d, uint32_t* crc, int device);

}  // namespace

int GatherToDeviceWithCrc(const Buf& in, Buf* out, uint32_t* crc, int device) {
    if (device < 0) device = CurrentDevice();
    const size_t n = in.size();
    *crc = 0;
    if (n == 0) return 0;
    Buf dev;
    char* d = static_cast<char*>(AppendNewDeviceBlock(&dev, n, device));
    if (!d) return kNoHbm;
    const int rc = copy_with_crc(in, d, crc, device);
    if (rc != 0) return rc;
    out->append(std::move(dev));
    return 0;
}

int ProcessToPinnedWithCrc(const Buf& in, Buf* out, uint32_t* crc, int device) {
    if (device < 0) device = CurrentDevice();
    const size_t n = in.size();
    *crc = 0;
    if (n == 0) return 0;
    char* h = static_cast<char*>(PinnedAlloc(n));
    if (!h) return kNoPinnedBounce;
    const int rc = copy_with_crc(in, h, crc, device);
    if (rc != 0) {
        PinnedFree(h, n);
        return rc;
    }
    out->append_user_data(h, n, pinned_deleter, reinterpret_cast<void*>((uintptr_t)n), MemKind::PINNED);
    return 0;
}

int CrcOnDevice(const Buf& in, uint32_t* crc, int device) {
    if (device < 0) device = CurrentDevice();
    *crc = 0;
    if (in.empty()) return 0;
    return copy_with_crc(in, nullptr, crc, device);
}

namespace {

struct AsyncJob {
    Buf in;
    bool to_device = false;
    int device = -1;
    std::function<void(int, Buf, uint32_t)> done;
};

void* run_async_job(void* arg) {
    std::unique_ptr<AsyncJob> j(static_cast<AsyncJob*>(arg));
    Buf out;
    uint32_t crc = 0;
    int rc;
    if (j->to_device) {
        rc = GatherToDeviceWithCrc(j->in, &out, &crc, j->device);
    } else {
        // the response goes back over TCP: the kernel reads the request's
        // pinned socket blocks once for the checksum and the bytes are sent
        // from where they already are (no pinned copy, no PCIe write back)
        rc = CrcOnDevice(j->in, &crc, j->device);
        if (rc == 0) out = j->in;
    }
    j->in.clear();
    j->done(rc, std::move(out), crc);
    return nullptr;
}

}  // namespace

void ProcessWithCrcAsync(Buf in, bool to_device, int device, std::function<void(int, Buf, uint32_t)> done) {
    AsyncJob* j = new AsyncJob;
    j->in = std::move(in);
    j->to_device = to_device;
    j->device = device;
    j->done = std::move(done);
    fiber::fiber_t tid;
    if (fiber::start_background(&tid, &fiber::ATTR_NORMAL, run_async_job, j) != 0) run_async_job(j);
}

namespace {

int copy_with_crc(const Buf& in, char* d, uint32_t* crc, int device) {
    const size_t n = in.size();
    std::vector<Segment> segs;
    std::vector<uint32_t> lens;
    segs.reserve(in.backing_block_num());
    // pageable host blocks are bounced through one pinned buffer first (the
    // kernel can only read pinned host memory)
    size_t pageable = 0;
    for (size_t i = 0; i < in.backing_block_num(); ++i) {
        if (in.ref_at(i).block->kind == MemKind::HOST) pageable += in.ref_at(i).length;
    }
    char* bounce = pageable ? static_cast<char*>(PinnedAlloc(pageable)) : nullptr;
    if (pageable && !bounce) return kNoPinnedBounce;
    size_t off = 0, boff = 0;
    for (size_t i = 0; i < in.backing_block_num(); ++i) {
        const BlockRef& r = in.ref_at(i);
        const char* src = r.block->data + r.offset;
        if (r.block->kind == MemKind::HOST) {
            memcpy(bounce + boff, src, r.length);
            src = bounce + boff;
            boff += r.length;
        } else if (!IsHostAccessible(r.block->kind) && r.block->device != device &&
                   ArenaOffset(src, r.block->device) < 0) {
            // another device's non-arena block: not mapped here
            if (bounce) PinnedFree(bounce, pageable);
            return kForeignBlock;
        }
        segs.push_back(Segment{src, d ? d + off : nullptr, r.length});
        lens.push_back(r.length);
        off += r.length;
    }
    // one message: the device folds the segment CRCs into the request's
    std::vector<uint32_t> crcs(segs.size());
    const int rc = BatchedCopy(segs.data(), (int)segs.size(), device, crcs.data(), /*fold_crc=*/true);
    if (bounce) PinnedFree(bounce, pageable);
    if (rc != 0) return kDeviceBatchFailed;
    *crc = crcs[0];
    (void)n;
    return 0;
}

}  // namespace

const char* DeviceHandlerErrorText(int rc) {
    switch (rc) {
    case 0: return "ok";
    case kNoHbm: return "no HBM block for the gathered bytes";
    case kNoPinnedBounce: return "no pinned memory for the bounce/output buffer";
    case kForeignBlock: return "a block of another device is not mapped here";
    case kDeviceBatchFailed: return "the copy+crc32c batch failed on the device";
    default: return "unknown device handler error";
    }
}

int StageToPinnedHost(const Buf& in, Buf* out) {
    // one pinned region for all device bytes, filled by one batched launch
    size_t dbytes = 0;
    int device = -1;
    for (size_t i = 0; i < in.backing_block_num(); ++i) {
        const BlockRef& r = in.ref_at(i);
        if (!IsHostAccessible(r.block->kind)) {
            dbytes += r.length;
            if (device < 0) device = r.block->device;
            if (r.block->device != device) return -1;  // mixed devices: caller stages per block
        }
    }
    if (dbytes == 0) {
        out->append(in);
        return 0;
    }
    char* h = static_cast<char*>(PinnedAlloc(dbytes));
    if (!h) return -1;
    std::vector<Segment> segs;
    size_t off = 0;
    for (size_t i = 0; i < in.backing_block_num(); ++i) {
        const BlockRef& r = in.ref_at(i);
        if (!IsHostAccessible(r.block->kind)) {
            segs.push_back(Segment{r.block->data + r.offset, h + off, r.length});
            off += r.length;
        }
    }
    if (BatchedCopy(segs.data(), (int)segs.size(), device) != 0) {
        PinnedFree(h, dbytes);
        return -1;
    }
    Buf staged;
    staged.append_user_data(h, dbytes, pinned_deleter, reinterpret_cast<void*>((uintptr_t)dbytes), MemKind::PINNED);
    off = 0;
    for (size_t i = 0; i < in.backing_block_num(); ++i) {
        const BlockRef& r = in.ref_at(i);
        if (IsHostAccessible(r.block->kind)) {
            out->append_block(r.block, r.offset, r.length);
        } else {
            staged.cutn(out, r.length);
        }
    }
    return 0;
}

}  // namespace gpu
}  // namespace mrpc
