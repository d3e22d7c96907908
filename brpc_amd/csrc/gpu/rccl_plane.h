// RCCL data plane: large HBM payloads of RPCs between ranks of one job move
// by ncclSend/ncclRecv over xGMI while the RPC meta (a per-pair sequence
// number and the length) travels on the TCP connection. The xGMI lending
// transport (gpu/xgmi.h) stays the default for payloads below
// -rccl_min_bytes; above it, RCCL's pipelined p2p kernels move the bytes
// (the analog of the reference's RDMA zero-copy SGEs,
// src/brpc/rdma/rdma_endpoint.cpp:771-895, with RCCL as the fabric).
//
// One communicator for the whole job, created collectively (every rank calls
// Init with the unique id rank 0 generated). All RCCL calls of the process
// are made by ONE poster thread, which issues whatever is ready as one
// ncclGroupStart/End group on a dedicated stream and completes waiters from
// the group's event.
//
// Matching without tags. RCCL pairs a rank's sends to a peer with that
// peer's receives in issue order, so:
//  * the sender numbers its payloads per destination and queues the send
//    BEFORE the meta that announces it is written to the socket;
//  * the receiver issues receives per source strictly in sequence order (a
//    reorder buffer holds payloads whose metas overtook earlier ones on
//    other connections), and a payload the receiver will not consume is
//    still received, into scratch, and dropped.
// Because every receive is issued after its matching send was queued, the
// stream-order wait-for graph is acyclic and the plane cannot deadlock.
// A send whose meta is never written (connection died in between) would
// stall the pair: a watchdog aborts the communicator after
// -rccl_timeout_ms without progress, fails every waiter, and traffic falls
// back to xGMI lending. Self-sends (a one-rank job, client and server in
// one process) are paired with their receive in the same group.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

#include "base/buf.h"

namespace mrpc {
namespace gpu {
namespace rccl {

// Generate a unique id (rank 0). Empty string when RCCL is unavailable.
std::string UniqueId(std::string* error = nullptr);
// Collective: create the communicator of `world` ranks on `device` and
// connect every pair (one warm-up exchange). 0 on success.
int Init(int rank, int world, const std::string& unique_id, int device, std::string* error = nullptr);
bool Active();
int Rank();
int World();
// Identity of the job's plane (hash of the unique id), carried in the xGMI
// hello so only peers of the same communicator use it.
uint64_t PlaneId();
// Abort the communicator (idempotent); pending waiters fail.
void Shutdown();

// Queue a send of [p, p+len) (HBM of the plane's device) to `peer`. `hold`
// keeps the bytes alive until RCCL is done with them. Returns the payload's
// sequence number for that destination, or -1.
int64_t Send(int peer, const void* p, size_t len, Buf&& hold);
// Receive payloads (src[i], seq[i], len[i]) into fresh HBM blocks outs[i];
// parks the calling fiber until all arrived. 0 on success.
int Recv(int n, const int* src, const uint64_t* seq, const size_t* len, Buf* outs);
// Payload the receiver will not consume: receive it into scratch and drop it.
void Discard(int src, uint64_t seq, size_t len);
// The sender queued payload `seq` for `peer` but will never announce it:
// the pair cannot be resynchronised, so the plane is aborted.
void Cancelled(int peer, uint64_t seq);

struct Stats {
    int64_t sent_payloads = 0, sent_bytes = 0, recv_payloads = 0, recv_bytes = 0;
    int64_t discarded = 0, groups = 0, aborts = 0;
    int64_t reorder_waits = 0;  // receives held back for an earlier sequence
};
Stats GetStats();

}  // namespace rccl
}  // namespace gpu
}  // namespace mrpc
