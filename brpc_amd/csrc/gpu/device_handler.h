// GPU-touching service handlers (the minimum MI355X slice):
// a request attachment is moved into HBM, a kernel runs over it and the
// response attachment is served from HBM — with the fiber parked on the
// batch's hipEvent, never blocking a worker pthread.
//
// Host-to-device and device-to-host moves go through the batched copy
// engine (gpu/copy_engine.h): the kernel reads pinned socket blocks directly
// (or peer/local HBM) and concurrent requests share one launch.
#pragma once

#include <cstdint>
#include <functional>

#include "base/buf.h"

namespace mrpc {
namespace gpu {

// Failure codes of the handler steps below (0 = success), so the RPC's
// error text says which step failed (DeviceHandlerErrorText).
enum DeviceHandlerError {
    kNoHbm = -1,
    kNoPinnedBounce = -2,
    kForeignBlock = -3,
    kDeviceBatchFailed = -4,
};
const char* DeviceHandlerErrorText(int rc);

// Gather `in` (any mix of pinned/pageable host, local or peer HBM blocks)
// into ONE new arena block on `device` appended to *out; *crc receives the
// standard CRC32C of the bytes, folded by the same kernel that moves them.
// 0 on success.
int GatherToDeviceWithCrc(const Buf& in, Buf* out, uint32_t* crc, int device);

// Same kernel, but the destination is ONE new pinned host block: the GPU
// reads the bytes (from pinned socket blocks or HBM), folds their CRC32C and
// writes them where the socket can send them from. The handler uses it when
// its response goes back over TCP, where an HBM copy would only have to be
// staged out again (a second device round trip per request).
int ProcessToPinnedWithCrc(const Buf& in, Buf* out, uint32_t* crc, int device);

// CRC32C of `in` computed on the device (the kernel reads pinned/HBM blocks
// in place; pageable blocks are bounced through pinned memory). 0 on success.
int CrcOnDevice(const Buf& in, uint32_t* crc, int device);

// Asynchronous handler step: to_device gathers `in` into HBM with its CRC
// (GatherToDeviceWithCrc, the response is lent over xGMI); otherwise the
// device only checksums `in` and `out` shares its bytes (the response goes
// back over TCP from the socket blocks it arrived in). Returns at once and
// runs done(rc, out, crc) in a fiber when the kernel finished. A handler that uses it never parks the fiber that called it —
// usually the connection's reader, which the input messenger runs the last
// request of a read in (reference: input_messenger.cpp:169-190) — so the
// next requests of the connection are read and submitted while the device
// works (the GPU round trips of pipelined requests overlap instead of
// queueing behind each other).
void ProcessWithCrcAsync(Buf in, bool to_device, int device,
                         std::function<void(int rc, Buf out, uint32_t crc)> done);

// Copy every device block of `in` into pinned host memory (one batched
// launch); host blocks are shared. Installed as the staging hook of
// policy/device_payload.h once a device is enabled.
int StageToPinnedHost(const Buf& in, Buf* out);

}  // namespace gpu
}  // namespace mrpc
