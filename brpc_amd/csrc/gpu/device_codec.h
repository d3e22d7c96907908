// Device-payload codec: snappy for HBM-resident attachments, end to end in
// HBM (MI355X-native; reference analog: the body codec of
// src/brpc/compress.cpp:79-92 and src/brpc/policy/snappy_compress.cpp:28-64,
// which runs on the host over IOBuf bytes).
//
// The sender encodes the payload in HBM into independent raw snappy blocks
// (one wave each, gpu/snappy_kernels.hip snappy_compress_kernel) laid out at
// a fixed stride inside one lendable arena block, and lends that block. Only
// the block table (compressed size per block) goes into the meta. The
// receiver decodes every block straight out of the lent region — local HBM,
// or the peer's HBM across xGMI — into its own HBM with the piece decoder
// (snappy_decompress_pieces_par_kernel), optionally pb_scan-indexing the
// result, and only then releases the lend. No byte of the payload crosses
// PCIe or touches a host cache, and both sides join the cross-RPC codec
// batch (gpu/codec_batch.h): one launch sequence and one event for every
// RPC's codec work that arrived meanwhile.
#pragma once

#include <cstddef>
#include <cstdint>

namespace mrpc {
struct DevicePayloadIndex;
namespace gpu {

struct DeviceSnappyLayout {
    uint32_t block_ulen = 0;  // uncompressed bytes per block (the last: the rest)
    uint32_t stride = 0;      // bytes between block starts (>= worst-case block)
    uint32_t nblocks = 0;
    uint64_t region() const { return (uint64_t)stride * nblocks; }
};
// -device_payload_block_kb blocks for a payload of `len` bytes.
DeviceSnappyLayout DeviceSnappyLayoutFor(size_t len);

// Encode [src, +len) (device memory) into `dst` (device, >= lay.region()
// bytes). clen[i] receives block i's size, its varint header included.
// Blocks the calling fiber on the codec batch; 0 on success.
int DeviceSnappyEncode(const void* src, size_t len, void* dst, const DeviceSnappyLayout& lay, uint32_t* clen,
                       int device);

// One received payload: blocks at region + i*stride of clen[i] bytes each
// (header included), decoded into dst (len bytes, device memory).
struct DeviceSnappyBlocks {
    const char* region = nullptr;
    uint64_t region_len = 0;
    DeviceSnappyLayout lay;
    const uint32_t* clen = nullptr;
    void* dst = nullptr;
    uint64_t len = 0;
    bool scan = false;  // pb_scan the decoded message into index[i]
};
// Validates every block table against its region (a bad table fails that
// job without launching anything for it), then decodes all jobs in one codec
// request. err[i] = 0, or nonzero when job i was malformed. `index` (may be
// null) gets job i's field table when jobs[i].scan. Returns -1 only on a
// device error.
int DeviceSnappyDecode(const DeviceSnappyBlocks* jobs, int n, int* err, DevicePayloadIndex* index, int device);

// Index already-decoded device messages (one codec request). 0 on success.
int DevicePbScan(const void* const* bufs, const uint64_t* lens, int n, DevicePayloadIndex* index, int device);

// The field table entry of length-delimited field `number` (the first one
// when repeated): its bytes are [*off, *off + *len) of the scanned payload.
// False when the index holds no such field.
bool DevicePayloadField(const DevicePayloadIndex& index, uint32_t number, uint64_t* off, uint64_t* len);

// A packed repeated numeric field whose bytes are already in device memory
// (a device payload located by its DevicePayloadIndex), decoded into a device
// array in the field's vector layout (kind: gpu::PbRunKind; 4 bytes per
// element for the 32-bit kinds, 8 for the 64-bit ones, 1 for bool). dst needs
// room for every element of the run (never more than `len`). The reference
// parses such fields element by element on the host
// (src/brpc/protocol.cpp:349-360 ParsePbFromIOBuf); here the bytes never
// leave HBM.
struct DevicePackedRun {
    const void* src = nullptr;
    uint64_t len = 0;
    uint32_t kind = 0;
    void* dst = nullptr;
    uint64_t count = 0;  // out: elements written
    int err = 0;         // out: 0 ok, 1 malformed or truncated varint, 2 refused (bad arguments)
};
// All runs in one codec request (two launches: count, then place). Returns
// -1 only on a device error; per-run codes in runs[i].err.
int DeviceDecodePackedRuns(DevicePackedRun* runs, int n, int device);

struct DeviceCodecStats {
    int64_t encodes = 0, encoded_bytes = 0, encoded_out_bytes = 0;
    int64_t decodes = 0, decoded_bytes = 0, bad_tables = 0, decode_errors = 0;
    int64_t scans = 0;
    int64_t packed_runs = 0, packed_bytes = 0, packed_elems = 0, packed_errors = 0;
};
DeviceCodecStats GetDeviceCodecStats();

}  // namespace gpu
}  // namespace mrpc
