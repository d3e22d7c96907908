// Device (HBM) attachment handling for baidu_std (MI355X-native).
// An attachment may contain DEVICE/PEER blocks (Buf::append_user_data with
// MemKind::DEVICE). When the socket has a device transport (the xGMI
// endpoint in gpu/xgmi_transport.cc) those blocks are written straight into
// the peer GPU's receive ring and described by RpcMeta.device_payload —
// they never touch the TCP byte stream. Without a transport the blocks are
// staged to host memory and sent inline (always correct, just slower).
#pragma once

#include <cstddef>

#include "base/buf.h"

namespace mrpc {

class Controller;
class Socket;
namespace policy {
class RpcMeta;
class DevicePayload;
}  // namespace policy

struct DeviceTransportHooks {
    // Copy [dev_ptr, dev_ptr+len) on `device` into the peer ring of `sock`.
    // Fill desc (ring_offset/length/src_device). 0 on success, >0 when the
    // transport cannot take the block right now (sent inline instead), <0 on
    // error.
    int (*send)(Socket* sock, const void* dev_ptr, size_t len, int device, bool with_crc, policy::DevicePayload* desc) = nullptr;
    // Append a block referencing the received ring region to *out.
    int (*recv)(Socket* sock, const policy::DevicePayload& desc, Buf* out) = nullptr;
};
void SetDeviceTransportHooks(const DeviceTransportHooks& h);
bool HasDeviceTransport(Socket* sock);

// Copies every non-host block of `in` to host memory (appends to *out).
void StageDeviceBufToHost(const Buf& in, Buf* out);

namespace policy {
bool SplitDevicePayload(Controller* cntl, bool request, const Buf& attachment, Buf* host_out, RpcMeta* meta,
                        Socket* sock = nullptr);
bool MergeDevicePayload(Controller* cntl, Socket* sock, const RpcMeta& meta, bool request, Buf* attachment);
}  // namespace policy

}  // namespace mrpc
