// Batched device copy engine: the data mover under the xGMI transport.
//
// Every fiber that needs device bytes moved (an xGMI pull of a received
// payload, a gather into HBM, ...) submits its (src, dst, len) segments here
// and parks. Submissions that arrive while a launch is being issued are
// combined: the first submitter becomes the leader, closes the open batch,
// launches ONE batched-copy kernel for all of its segments on a pool stream,
// records one event and hands it to the completion poller, which wakes every
// fiber of that batch at once. Under load this turns N payload transfers per
// tick into one kernel launch + one event, instead of N hipMemcpyAsync + N
// event round trips (which is what capped the round-1 HBM path below the
// host TCP path).
//
// Sources may be local HBM, peer HBM mapped through hipIpcOpenMemHandle
// (the kernel then reads across xGMI) or pinned host memory.
#pragma once

#include <cstddef>
#include <cstdint>

#include "gpu/kernels.h"

namespace mrpc {
namespace gpu {

// Copy all segments on `device`; returns when the copies completed (fiber
// parks, pthread blocks). 0 on success. With `crcs`, the batch runs the
// fused copy+CRC32C kernel and crcs[i] receives the standard CRC32C of
// segment i (computed from the bytes while they are moved).
// With fold_crc, crcs[0] instead receives the CRC32C of all n segments
// concatenated (one message), folded on the device. With crcs, a segment
// whose dst is null is only checksummed (nothing is written).
int BatchedCopy(const Segment* segs, int n, int device, uint32_t* crcs = nullptr, bool fold_crc = false);

struct CopyEngineStats {
    int64_t submits = 0, launches = 0, segments = 0, bytes = 0;
    // summed over submissions (us): until the batch's launch began, the
    // launch API calls, launch-to-completion-seen, completion-to-resumed
    int64_t queue_us = 0, api_us = 0, gpu_us = 0, wake_us = 0;
    // launches with a completion word: summed kernel duration (GPU wall-clock
    // ticks, workgroup 0 start -> last workgroup end) and how many
    int64_t kernel_ticks = 0, kernel_timed = 0;
    // over the same launches (GPU clock correlated to the host's): launch
    // API return -> kernel start, kernel end -> completion seen (us, summed)
    int64_t start_delay_us = 0, notice_us = 0;
};
CopyEngineStats GetCopyEngineStats();

}  // namespace gpu
}  // namespace mrpc
