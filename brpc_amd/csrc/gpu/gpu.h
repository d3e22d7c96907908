// MI355X device runtime for the RPC engine.
//
// The reference has no GPU code; this module is what makes the framework
// MI355X-native (SURVEY.md §2 "GPU" rows, BASELINE.json north star):
//  * HBM-resident Buf blocks (MemKind::DEVICE) with refcounted ownership so
//    attachments can stay on the GPU end to end;
//  * pinned (hipHostMalloc) block allocator so every socket buffer is
//    DMA-able by the SDMA engines without a bounce;
//  * a fiber-aware completion poller: a fiber that waits for a hipEvent
//    parks on a butex and a single poller thread wakes it — GPU work and RPC
//    handling interleave without ever blocking a worker pthread (the role
//    bthread's butex plays for sockets, applied to HIP streams);
//  * small per-device stream pools (GPU_MAX_HW_QUEUES=4 on the box, so we
//    never create more than 4 streams per device and per process).
// Everything degrades cleanly on a machine without a GPU: DeviceCount()
// returns 0 and allocation calls fail with an error string.
#pragma once

#include <cstddef>
#include <atomic>
#include <cstdint>
#include <string>

#include "base/buf.h"

typedef struct ihipStream_t* hipStream_t;
typedef struct ihipEvent_t* hipEvent_t;

namespace mrpc {
namespace gpu {

// Number of visible devices; 0 when no GPU / runtime unavailable. Does not
// create a context.
int DeviceCount();
bool Available();
// Initialise the runtime on `device` (-1 = current), install the Buf device
// copy hook and start the event poller. Idempotent. 0 on success.
int Init(int device = -1, std::string* error = nullptr);
int CurrentDevice();
std::string DeviceName(int device);
// gfx arch string of the device ("gfx950" on MI355X).
std::string DeviceArch(int device);
// PCI address of the device ("0000:75:00.0"), for placing the rank's CPU
// threads on the GPU's NUMA node (/sys/bus/pci/devices/<bdf>/local_cpulist).
std::string PciBusId(int device);

// ---- memory
void* Malloc(size_t n, int device, std::string* error = nullptr);
void Free(void* p);
void* HostMallocPinned(size_t n);
void HostFreePinned(void* p);
// Make default Buf blocks pinned host memory from the pinned slab pool
// (gpu/hbm_pool.h). Idempotent; called when a Server or Channel enables a
// GPU device, before traffic starts.
int UsePinnedBlocks();
bool PinnedBlocksInUse();

// Copies; stream-ordered on a pool stream, the calling fiber parks until
// completion (a pthread blocks).
int CopyHostToDevice(void* dst, const void* src, size_t n, int device);
int CopyDeviceToHost(void* dst, const void* src, size_t n, int device);
int CopyDeviceToDevice(void* dst, const void* src, size_t n, int device);
int Memset(void* dst, int value, size_t n, int device);

// ---- Buf helpers
// Append [dev, dev+n) as one DEVICE block. deleter(dev, arg) runs when the
// last reference dies (nullptr = caller keeps ownership).
int AppendDevice(Buf* b, void* dev, size_t n, int device, void (*deleter)(void*, void*) = nullptr,
                 void* arg = nullptr);
// Allocate HBM, upload `data` and append it as a DEVICE block owned by `b`.
int AppendHostAsDevice(Buf* b, const void* data, size_t n, int device, std::string* error = nullptr);
// Move every non-host block of `in` to one contiguous HBM allocation
// appended to *out (host blocks are uploaded). Used by device handlers.
int GatherToDevice(const Buf& in, Buf* out, int device, std::string* error = nullptr);
// Copy all of `in` (any kinds) into *out.
int CopyBufToHost(const Buf& in, std::string* out);
bool HasDeviceBlocks(const Buf& b);

// ---- streams / events
hipStream_t PoolStream(int device);  // round-robin over <=4 non-blocking streams
// Park the calling fiber until `ev` completes (pthread: hipEventSynchronize).
int WaitEvent(hipEvent_t ev);
// Record an event on `s` and wait for it fiber-friendly.
int SyncStream(hipStream_t s);
// Hand `ev` to the completion poller: when it completes the poller stores 1
// (or -1 on failure) into *butex and wakes every waiter parked on it. One
// event can release a whole batch of fibers.
// `done_us` (optional) receives the monotonic time the poller saw it done.
// `cls` groups events of similar duration (EventClass): the poller keeps a
// completion-time average per class and sleeps until the earliest event
// can be due, so a short copy handed over behind long codec batches is
// polled on the copy's time scale, not the batches'.
enum EventClass { kEventOther = 0, kEventCopy = 1, kEventCodec = 2, kEventClasses = 3 };
void WatchEvent(hipEvent_t ev, std::atomic<int>* butex, int64_t* done_us = nullptr, int cls = kEventOther);
// Same for batches [first, last] of a resident copy worker ring (the
// poller reads their pinned done words instead of querying an event).
struct ResidentRing;
struct DoneWord;  // kernels.h
void WatchResident(ResidentRing* ring, uint64_t first_seq, uint64_t last_seq, std::atomic<int>* butex,
                   int64_t* done_us = nullptr);
// Same for a launch with a completion word (kernels.h DoneWord): done when
// *word == seq (one read of pinned memory per poll). `ev`, recorded after the
// launch, is the fallback: it is queried only once the word is overdue
// (-gpu_done_word_fallback_ms), so a launch that never stores its word
// (failed) still completes with the event's verdict; *fell_back is set then.
void WatchWord(const uint64_t* word, uint64_t seq, hipEvent_t ev, std::atomic<int>* butex, int64_t* done_us,
               int cls, bool* fell_back);
// Completion-word slots of a device: a device counter and a pinned host word
// each. false: none free (the caller completes through its event alone).
bool AcquireDoneWord(int device, DoneWord* out, uint32_t* slot);
void ReleaseDoneWord(int device, uint32_t slot);
// Pooled events (hipEventDisableTiming).
hipEvent_t AcquireEvent();
void ReleaseEvent(hipEvent_t e);
// Poller statistics
int64_t PolledEvents();

}  // namespace gpu
}  // namespace mrpc
