// xGMI device transport: HBM payloads move GPU-to-GPU over xGMI while only
// the RPC metadata travels on the TCP connection (the MI355X analog of the
// reference's RDMA endpoint, src/brpc/rdma/rdma_endpoint.cpp:771-895, whose
// SGEs point straight into registered IOBuf blocks).
//
// Zero-copy send, one pull per hop:
//  * every HBM block the framework allocates comes from the per-device
//    IPC-exported arena (gpu/hbm_pool.h), which each peer process maps once
//    during the per-connection hello (RpcMeta.xgmi_hello, both directions);
//  * sending a DEVICE attachment block LENDS it: the sender takes a
//    reference, assigns a release slot and puts (arena offset, length, slot,
//    seq) into RpcMeta.device_payload — no copy, no device work at all.
//    Blocks from outside the arena (a torch tensor, a user hipMalloc) are
//    first copied into an arena block;
//  * the receiver pulls every payload of a message into fresh blocks of its
//    own arena with the batched copy engine (gpu/copy_engine.h: one kernel
//    for the payloads of all concurrently arriving messages, reading across
//    xGMI when the sender sits on another GPU), then writes the seq into the
//    sender's POSIX-shm release table. The sender reaps released slots and
//    drops its references; slots whose connection died are reaped too.
// Received blocks are arena memory again, so a server that forwards or
// echoes them lends them onward without another copy.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

namespace mrpc {
class Socket;
namespace policy {
class XgmiHello;
}  // namespace policy

namespace gpu {

// Registers the transport hooks and creates this process's arena on
// `device` (idempotent). Returns 0, or -1 when no GPU / IPC is available.
int EnableXgmiTransport(int device, std::string* error = nullptr);
bool XgmiEnabled();
int XgmiDevice();
// Fill the local hello (arena of the enabled device).
bool FillXgmiHello(policy::XgmiHello* hello);
// Map the peer described by `hello` and attach the endpoint to `sock`.
// Same-process peers use the local arena directly. Returns 0 on success.
int AttachXgmiPeer(Socket* sock, const policy::XgmiHello& hello, std::string* error = nullptr);
// Drop references of every lent block the peers have released. Runs on
// every send; exposed for tests and idle-time housekeeping.
void ReapLentBlocks();

struct XgmiStats {
    int64_t sent_bytes = 0, recv_bytes = 0, sent_payloads = 0, recv_payloads = 0;
    int64_t ring_full_fallbacks = 0, crc_failures = 0;
    int64_t lent_outstanding = 0, copied_into_arena = 0, released_unconsumed = 0;
    // pulls whose source sat on ANOTHER GPU (true xGMI traffic), as opposed
    // to HBM-local lends between processes/sockets of one device
    int64_t cross_device_payloads = 0, cross_device_bytes = 0, cross_device_pull_failures = 0;
    int64_t peer_access_enabled = 0;  // hipDeviceEnablePeerAccess successes
    int64_t attach_failures = 0;      // hellos that could not be mapped (fallback: staged over TCP)
    int64_t peer_maps = 0;            // peer arenas mapped
    // device-compressed payloads (Controller::set_device_payload_compress_type):
    // lent encoded, decoded on arrival, lent raw because incompressible, or
    // lent raw because the device encode failed
    int64_t compressed_sent = 0, compressed_recv = 0, compress_skipped_raw = 0, compress_failures = 0;
    // lent raw without an encode: the connection's recent payloads were incompressible
    int64_t compress_skipped_adaptive = 0;
};
XgmiStats GetXgmiStats();

}  // namespace gpu
}  // namespace mrpc
