// Device (HBM) attachment handling for baidu_std (MI355X-native).
// An attachment may contain DEVICE blocks (Buf::append_user_data with
// MemKind::DEVICE). When the socket has a device transport (the xGMI
// endpoint in gpu/xgmi.cc) those blocks are lent to the peer and described
// by RpcMeta.device_payload — they never touch the TCP byte stream. Without
// a transport the blocks are staged to host memory and sent inline (always
// correct, just slower).
//
// Every received descriptor must end in exactly one of: a pull
// (MergeDevicePayload) or a release (ReleaseDevicePayload) — otherwise the
// sender keeps the lent block until the connection dies.
#pragma once

#include <cstddef>
#include <cstdint>

#include <string>
#include <utility>
#include <vector>

#include "base/buf.h"
#include "pb/message.h"

namespace mrpc {

class Controller;
class Socket;
namespace policy {
class RpcMeta;
class DevicePayload;
}  // namespace policy

// How the sender lends device blocks (Controller::verify_device_payload,
// device_payload_compress_type, device_payload_scan).
struct DeviceLendOptions {
    bool verify = false;  // CRC32C of the payload, checked by the receiver on the device
    int compress = 0;     // CompressType: 1 = snappy-encode on the device before lending
    bool scan = false;    // the payload is one protobuf message: the receiver indexes it
};

// Top-level field table of a device payload that arrived with pb_scan
// (pb_scan layout: fields[2k] = (number << 3) | wire type, fields[2k+1] =
// the value, or the (offset << 32 | length) of a length-delimited field).
// nfields < 0: not scanned (or a malformed message, pb_scan's code).
struct DevicePayloadIndex {
    int nfields = -1;
    std::vector<uint64_t> fields;
};

struct DeviceTransportHooks {
    // Lend [block->data+offset, +len) to the peer of `sock` and fill desc
    // (ring_offset/length/slot/seq/src_device, and the block table of a
    // device-compressed payload). 0 on success, >0 when the transport cannot
    // take the block right now (sent inline instead), <0 on error.
    int (*send)(Socket* sock, BufBlock* block, uint32_t offset, uint32_t len, const DeviceLendOptions& opt,
                policy::DevicePayload* desc) = nullptr;
    // Pull (or decode, when device-compressed) the n described payloads into
    // fresh local HBM blocks (outs[i] receives payload i) and release them to
    // the sender. With `index`, index[i] receives payload i's field table
    // when its descriptor asked for pb_scan. 0 on success.
    int (*recv)(Socket* sock, const policy::DevicePayload* const* descs, int n, Buf* outs,
                DevicePayloadIndex* index) = nullptr;
    // The receiver will not consume `desc`: give it back to the sender.
    void (*release)(Socket* sock, const policy::DevicePayload& desc) = nullptr;
    // The sender lent `desc` but the message carrying it is never sent.
    void (*cancel)(const policy::DevicePayload& desc) = nullptr;
};
void SetDeviceTransportHooks(const DeviceTransportHooks& h);
bool HasDeviceTransport(Socket* sock);

// Copies every non-host block of `in` to host memory (appends to *out).
// Device payloads staged inline on the connection so far (count, bytes).
void GetStagedStats(int64_t* payloads, int64_t* bytes);
void StageDeviceBufToHost(const Buf& in, Buf* out);
// Batched staging implementation (gpu/device_handler.h), installed when a
// device is enabled; returns non-zero to fall back to per-block copies.
void SetStageToHostHook(int (*fn)(const Buf& in, Buf* out));

namespace policy {
using DevicePayloads = pb::RepeatedPtrField<DevicePayload>;

// A request's packed descriptors, kept by its controller until the write
// is accepted (rpc/controller.h _packed_payloads).
struct PackedPayloads {
    DevicePayloads descs;
};
// Protocol-neutral core (baidu_std metas and STRM frames): lend the device
// blocks of `in` into *descs (host blocks go to *host_out, positions are
// relative to `in`); pull `descs` into *attachment, whose current content
// is the inline host part; release descriptors that will not be pulled.
int LendDeviceBlocks(Socket* sock, const Buf& in, const DeviceLendOptions& opt, Buf* host_out,
                     DevicePayloads* descs, std::string* err);
// With `index`: the field table of the first payload that asked for pb_scan.
int PullDeviceBlocks(Socket* sock, const DevicePayloads& descs, Buf* attachment, std::string* err,
                     DevicePayloadIndex* index = nullptr);
// Several messages of one connection at once (one batched pull launch);
// `indexes` (optional) gets one entry per item.
int PullDeviceBlocksBatch(Socket* sock, const std::vector<std::pair<const DevicePayloads*, Buf*>>& items,
                          std::string* err, std::vector<DevicePayloadIndex>* indexes = nullptr);
void ReleaseDeviceBlocks(Socket* sock, const DevicePayloads& descs);
void CancelDeviceBlocks(const DevicePayloads& descs);

bool SplitDevicePayload(Controller* cntl, bool request, const Buf& attachment, Buf* host_out, RpcMeta* meta,
                        Socket* sock = nullptr);
bool MergeDevicePayload(Controller* cntl, Socket* sock, const RpcMeta& meta, bool request, Buf* attachment);
// Give back every device payload of `meta` without pulling it (rejected
// requests, stale or failed responses).
void ReleaseDevicePayload(Socket* sock, const RpcMeta& meta);
// Un-lend the payloads a sender put into `meta` for a message it will not
// send after all.
void CancelDevicePayload(const RpcMeta& meta);
}  // namespace policy

}  // namespace mrpc
