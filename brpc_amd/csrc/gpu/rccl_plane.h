// RCCL payload plane: large payloads of RPCs between ranks of one node move
// by ncclSend/ncclRecv over xGMI while the RPC meta (the payload's per-pair
// sequence number and length) travels on the TCP connection. The xGMI
// lending transport (gpu/xgmi.h) stays the default below -rccl_min_bytes.
// It is the analog of the reference's RDMA data path
// (src/brpc/rdma/rdma_endpoint.cpp:771-895: zero-copy SGEs, a sliding
// window per connection, ACK credits in imm_data, window sizes agreed in
// the handshake at :505-509,613-617), with RCCL as the fabric.
//
// Why pair rounds. RCCL send/recv kernels block until their partner runs,
// every op of one communicator is serialised, and streams beyond
// GPU_MAX_HW_QUEUES share in-order hardware queues. A plane that issues a
// send before its peer has committed to the matching receive can park it in
// front of work another rank needs (a cross-rank deadlock once payloads
// exceed RCCL's p2p buffering), and a plane that moves every rank in
// lockstep (round 3's) lets one slow rank stall the node. This plane
// decouples the pairs instead:
//  * the control traffic never touches RCCL: per unordered pair of ranks a
//    shm slot holds a round word, each side's payload list for the open
//    round, the landing credit each receiver grants and a cancel ring;
//  * a side with payloads within credit publishes its list and sets its
//    ready bit; the side that finds the other bit set fires the round (the
//    word moves to the next round). Idle pairs exchange nothing, and a
//    payload moves in the round it is listed in — the receiver granted the
//    landing bytes ahead of time (-rccl_window_bytes, the analog of the
//    reference's pre-posted receive blocks, rdma_endpoint.cpp:990-1006);
//  * every round a rank takes part in goes into ONE ncclGroupStart/End
//    group on its one stream, and the rank clears its ready bit on every
//    other pair first (a clear that fails means the peer fired it: it joins
//    the group). So each rank has at most one plane group in flight and
//    every group's partner ops sit in the partner's only group: no group
//    can wait behind another, and a group waits only for ranks that
//    already committed to it, never for an unrelated or slow rank.
// Flow control: a sender lists a payload only within the receiver's
// cumulative consumed bytes plus -rccl_window_bytes (or alone, once
// everything it sent was consumed); the receiver wakes a stalled sender
// when it consumes. Received payloads wait in a stash, keyed by (source,
// sequence), until the RPC layer claims them (Recv), gives them back
// (Discard) or -rccl_stash_ttl_ms expires.
// Failure: any rank that hits an RCCL error, a group older than
// -rccl_timeout_ms or a dead peer process sets the node's abort flag;
// every rank then aborts its communicator, waits (bounded) for its stream
// to drain before recycling payload memory, fails its waiters, and new
// payloads fall back to xGMI lending.
//
// On hosts without GPUs the plane runs on the stub library
// tests/stub/fake_rccl.cc (-rccl_library), moving host blocks.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

#include "base/buf.h"

namespace mrpc {
namespace policy {
class PlaneHello;
}  // namespace policy
namespace gpu {
namespace rccl {

// Generate a unique id (rank 0). Empty string when RCCL is unavailable.
std::string UniqueId(std::string* error = nullptr);
// Collective over the ranks of one node: create the communicator of
// `world` ranks on `device` (ignored on the stub library) and run the
// first round (connects every pair). 0 on success.
int Init(int rank, int world, const std::string& unique_id, int device, std::string* error = nullptr);
bool Active();
int Rank();
int World();
// Identity of the job's plane (hash of the unique id), carried in the
// connection hello so only peers of the same plane use it.
uint64_t PlaneId();
// The plane moves host blocks (stub library) rather than HBM blocks.
bool HostMemory();
// Whether a payload block of this kind/device can go over the plane.
bool AcceptsBlock(const BufBlock* b);
// Leave the plane (not collective: the other ranks fall back to lending).
void Shutdown();

// Connection hello (RpcMeta.plane_hello): this rank's identity, and the
// peer's plane rank from its hello (-1: not a rank of our plane).
bool FillHello(policy::PlaneHello* h);
int PeerRank(const policy::PlaneHello& h);

// Queue [p, p+len) for `peer`; `hold` keeps the bytes alive until RCCL is
// done with them. Returns the payload's sequence number for that
// destination (announced in the meta), or -1 when the plane is down.
int64_t Send(int peer, const void* p, size_t len, Buf&& hold);
// Claim payloads (src[i], seq[i], len[i]) into outs[i]; parks the calling
// fiber until all arrived (at most -rccl_timeout_ms). 0 on success.
int Recv(int n, const int* src, const uint64_t* seq, const size_t* len, Buf* outs);
// Payload the receiver will not consume: drop it (now or on arrival).
void Discard(int src, uint64_t seq, size_t len);
// The sender queued payload `seq` for `peer` but will never announce it in
// a meta: withdrawn if not yet announced in a round header, otherwise the
// receiver's stash expires it.
void Cancelled(int peer, uint64_t seq);

// Fault injection: raise the node's abort flag as if this rank had failed
// (every rank's poster aborts its plane).
void AbortForTest(const std::string& why);

struct Stats {
    int64_t sent_payloads = 0, sent_bytes = 0, recv_payloads = 0, recv_bytes = 0;
    int64_t discarded = 0, rounds = 0, payload_rounds = 0, aborts = 0;
    int64_t pair_rounds = 0;     // pair rounds fired (a group holds one per partner)
    int64_t withdrawals = 0;     // ready bits cleared because another pair fired first
    int64_t group_us = 0;        // wall time groups spent on the stream (issue to completion)
    int64_t credit_stalls = 0;   // rounds where a queued payload waited for credit
    int64_t stash_expired = 0;   // received payloads nobody claimed in time
    int64_t recv_timeouts = 0;   // Recv calls that gave up
    int64_t doorbells = 0;       // idle -> busy wake-ups of the poster by new payloads
    int64_t withdrawn = 0;       // Cancelled (before announcement, or told to the receiver after)
    int64_t stash_payloads = 0, stash_bytes = 0;  // landed, not yet claimed (now)
    int world = 0;
    bool host_memory = false;
};
Stats GetStats();

}  // namespace rccl
}  // namespace gpu
}  // namespace mrpc
