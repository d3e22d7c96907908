// xGMI device transport: HBM payloads move GPU-to-GPU over xGMI while only
// the RPC metadata travels on the TCP connection (the MI355X analog of the
// reference's RDMA endpoint, src/brpc/rdma/rdma_endpoint.cpp +
// block_pool.cpp, which zero-copies IOBuf blocks over verbs).
//
// Each process owns one IPC arena per device: a large HBM region exported
// with hipIpcGetMemHandle plus a POSIX-shm release table. Sending a DEVICE
// attachment block = one D2D copy into a ring region of the sender's arena;
// the descriptor (offset, length, slot, seq) rides in RpcMeta. The receiver
// mapped the sender's arena during the per-connection hello
// (RpcMeta.xgmi_hello, both directions), pulls the region peer-to-peer into
// a pooled HBM block of its own device (xGMI DMA), verifies the optional
// CRC32C on device (MFMA kernel) and writes the region's sequence number
// into the sender's release table; the sender reclaims its ring in FIFO
// order. Nothing is sent over TCP for the payload bytes.
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
// Fill the local hello (arena of the enabled device).
bool FillXgmiHello(policy::XgmiHello* hello);
// Map the peer described by `hello` and attach the endpoint to `sock`.
// Same-process peers use the local arena directly. Returns 0 on success.
int AttachXgmiPeer(Socket* sock, const policy::XgmiHello& hello, std::string* error = nullptr);

// Pooled HBM blocks (size classes) so received payloads never hit hipMalloc
// on the hot path.
void* PoolAlloc(size_t n, int device);
void PoolFree(void* p);

struct XgmiStats {
    int64_t sent_bytes = 0, recv_bytes = 0, sent_payloads = 0, recv_payloads = 0;
    int64_t ring_full_fallbacks = 0, crc_failures = 0;
};
XgmiStats GetXgmiStats();

}  // namespace gpu
}  // namespace mrpc
