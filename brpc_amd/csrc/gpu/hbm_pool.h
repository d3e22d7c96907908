// Pooled device and pinned-host memory for the RPC data plane.
//
// HBM: one large IPC-exportable arena per device (hipMalloc + one
// hipIpcGetMemHandle) carved into power-of-two size classes with per-class
// free lists and per-thread caches. Every HBM block the framework hands out
// (received payloads, device attachments allocated through
// AppendNewDeviceBlock, staging for handlers) comes from here, so that
//   * no hipMalloc/hipFree is ever on the request path (hipFree synchronises
//     the whole device);
//   * any such block can be LENT to a peer process zero-copy: the peer has
//     the arena mapped (one hipIpcOpenMemHandle per peer process, done in
//     the xGMI hello), so a block is named by its arena offset alone.
// This is the MI355X analog of the reference's registered RDMA block pool
// (src/brpc/rdma/block_pool.cpp:48-50,189,362,389) whose blocks are what
// IOBuf hands to ibv_post_send without copying.
//
// Pinned host: hipHostMalloc'ed regions carved into the same kind of size
// classes. Installed as the Buf block allocator (UsePinnedBlocks) it plays
// the role of the reference's blockmem_allocate swap
// (src/brpc/rdma/rdma_helper.cpp:169-188): every socket read lands in
// DMA-able memory, so H2D staging of request bodies needs no bounce buffer.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

#include "base/buf.h"

namespace mrpc {
namespace gpu {

// ---- HBM arena
struct ArenaDesc {
    char* base = nullptr;
    size_t size = 0;
    int device = -1;
    std::string ipc_handle;  // raw hipIpcMemHandle_t bytes
};

// Create the arena of `device` (idempotent; -1 = current device).
int InitHbmPool(int device, std::string* error = nullptr);
bool HbmPoolReady(int device);
ArenaDesc GetArena(int device);
// Allocate at least n bytes of HBM on `device` from the arena. Falls back to
// a plain hipMalloc (not exportable) when the arena is exhausted; nullptr on
// failure. HbmFree must get the same n.
void* HbmAlloc(size_t n, int device);
void HbmFree(void* p, size_t n, int device);
// Offset of p inside the arena of `device`, or -1 when p is not arena memory.
int64_t ArenaOffset(const void* p, int device);

// Allocate n bytes of arena HBM and append them to *b as one DEVICE block
// owned by the Buf (returned to the pool when the last reference dies).
void* AppendNewDeviceBlock(Buf* b, size_t n, int device);

// Called (from the allocating thread) when the arena has no block of the
// requested class left: frees what can be freed (the xGMI lender reaps
// lends its peers released) before the pool falls back to hipMalloc.
void SetHbmReclaimHook(void (*fn)());

struct HbmPoolStats {
    int64_t arena_bytes = 0, carved_bytes = 0, live_blocks = 0, live_bytes = 0, fallback_allocs = 0;
    int64_t splits = 0;  // free blocks of a larger class cut up once the arena was fully carved
};
HbmPoolStats GetHbmPoolStats(int device);

// ---- pinned host slabs
void* PinnedAlloc(size_t n);
void PinnedFree(void* p, size_t n);
int64_t PinnedBytes();

}  // namespace gpu
}  // namespace mrpc
