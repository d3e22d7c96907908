// Host-side launch API of the hand-written CDNA4 kernels in kernels.hip.
// All launches are stream-ordered and asynchronous; pointers are device (or
// device-accessible pinned) addresses.
#pragma once

#include <cstddef>
#include <cstdint>

#include "gpu/gpu.h"

namespace mrpc {
namespace gpu {

struct Segment {
    const void* src;
    void* dst;   // used by copies; ignored by crc
    uint64_t len;
};

// Maximum number of segments one launch carries inline in its kernel
// arguments (no descriptor upload); launchers split larger batches.
constexpr int kInlineSegments = 32;
// Bytes covered by one workgroup (256 lanes x 64 bytes).
constexpr uint64_t kChunkBytes = 16384;

// Standard (finalized) CRC32C of every segment into out_dev[i] — the
// MFMA (GF(2) matmul on v_mfma_i32_32x32x32_i8) kernel. Segment table lives
// in device memory: starts_dev[i] = address, lens_dev[i] = bytes.
// total_bytes bounds the sum of lengths (sizes the grid); max_seg_len
// bounds any one length. scratch: Crc32cScratchBytes(nseg) of device memory.
size_t Crc32cScratchBytes(int64_t nseg);
int LaunchCrc32cSegments(const uint64_t* starts_dev, const uint64_t* lens_dev, int64_t nseg, uint64_t total_bytes,
                         uint64_t max_seg_len, uint32_t* out_dev, void* scratch, hipStream_t s);
// Same result from the LDS slicing-by-8 kernel (segments passed inline;
// kept as an independent implementation for cross-checks and A/B timing).
// `out` needs no initialisation and may be pinned host memory (the kernel
// stores each finished CRC; read it after the stream's event).
int LaunchCrc32c(const Segment* segs, int nseg, uint32_t* out, hipStream_t s);
// One lane stores the GPU wall clock (100 MHz) into *out_pinned (pinned host
// memory, system scope): clock correlation for diagnostics.
int LaunchClockProbe(uint64_t* out_pinned, hipStream_t s);
// One wave that sleeps `us` microseconds of GPU wall clock (capped at 10 s).
int LaunchSleepKernel(uint64_t us, hipStream_t s);
// Completion word of a launch: the kernel's last workgroup to finish
// stores `seq` into *word (pinned host memory, system-scope release, after
// every workgroup's stores were released at agent scope), so the host sees
// the batch done by reading one word — no hipEvent in the completion path.
// `counter` (device memory, zero between launches) counts finished
// workgroups; the last one resets it. Launchers that split a batch into
// several launches on one stream pass the word to the last launch only.
// word[1] / word[2] receive the GPU wall clock (hipDeviceAttributeWallClockRate)
// when workgroup 0 started and when the last workgroup finished.
struct DoneWord {
    uint32_t* counter = nullptr;
    uint64_t* word = nullptr;
    uint64_t seq = 0;
};
// Copy every segment src -> dst (one launch for many small copies).
int LaunchBatchedCopy(const Segment* segs, int nseg, hipStream_t s, const DoneWord* done = nullptr);
// Fused: copy every segment AND write its standard CRC32C to out[i]
// (one read of the bytes; sources may be local/peer HBM or pinned host).
// One launch per 32 segments and nothing else: no memset of `out`, which
// may be pinned host memory read after the stream's event.
// mfma: the CRC runs on the matrix cores (copy_crc32c_mfma_kernel, the
// default), else on the byte-table kernel.
int LaunchBatchedCopyCrc32c(const Segment* segs, int nseg, uint32_t* out, hipStream_t s, bool mfma = true);
// Same copy, but consecutive segments with equal msg_of[] (non-decreasing,
// starting anywhere) form a MESSAGE and out[msg_of[i]] receives the CRC32C
// of the message's bytes (its segments concatenated), folded on the device.
// A message may have at most kInlineSegments segments (else -2, nothing
// launched for it).
int LaunchBatchedCopyCrc32cMessages(const Segment* segs, const int* msg_of, int nseg, uint32_t* out, hipStream_t s,
                                    const DoneWord* done = nullptr, bool mfma = true);

// Packed-varint decode (protobuf wire type 0, packed repeated field):
// `in` holds n bytes of concatenated varints; out receives the values
// (uint64, zigzag-decoded to int64 when zigzag). count_dev receives the
// number of values; err_dev gets 1 if the stream is malformed (value longer
// than 10 bytes or truncated). scratch must hold VarintScratchBytes(n).
size_t VarintScratchBytes(uint64_t n);
int LaunchVarintDecode(const uint8_t* in, uint64_t n, uint64_t* out, uint64_t max_out, bool zigzag,
                       uint64_t* count_dev, int* err_dev, void* scratch, hipStream_t s);
// Packed-varint encode: values -> bytes. out must hold 10*n bytes; bytes_dev
// receives the encoded size. scratch must hold VarintScratchBytes(n).
int LaunchVarintEncode(const uint64_t* in, uint64_t n, bool zigzag, uint8_t* out, uint64_t* bytes_dev,
                       void* scratch, hipStream_t s);

// Batched snappy decompression (gpu/snappy_kernels.hip): every job is an
// independent raw snappy stream of at most kSnappyMaxBlock uncompressed
// bytes. jobs_dev is a device array; out_len_dev[i] / err_dev[i] receive
// the decoded size and 0 (or a nonzero malformed-input code) per job.
constexpr uint32_t kSnappyMaxBlock = 65536;
struct SnappyJob {
    const void* src;    // compressed stream (device)
    void* dst;          // output (device), dst_cap bytes
    uint64_t src_len;
    uint64_t dst_cap;
};
// max_ulen (>= every job's uncompressed size) sizes the LDS per wave: 32 KiB
// blocks run 5 waves per CU, 64 KiB blocks 2.
int LaunchSnappyDecompress(const SnappyJob* jobs_dev, int n, uint32_t max_ulen, uint32_t* out_len_dev, int* err_dev,
                           hipStream_t s);
// Whole raw streams of any length, cut on the device (no host tag walk):
// one wave per stream walks its element headers and cuts it into pieces of
// at most piece_limit uncompressed bytes whose copies stay inside the piece
// (every fragmenting encoder's output: ours cuts at -gpu_snappy_block_kb,
// CPU encoders at 64 KiB; a stream that does not cut at piece_limit is
// retried at kSnappyMaxBlock). Pieces land in pieces[first, first +
// max_pieces) (unused slots get ulen 0); stream_err[i] = 0 or a code
// (malformed, longer than dst_cap, not cuttable). A piece is headerless: its
// ulen is known, its src points into the stream.
struct SnappyStream {
    const void* src;  // whole compressed stream (device)
    void* dst;        // output, dst_cap bytes (device-accessible)
    uint32_t src_len, dst_cap;
    uint32_t first, max_pieces;
};
struct SnappyPiece {
    const void* src;
    void* dst;
    uint32_t src_len, ulen;
};
// Slots a stream of ulen bytes can need: consecutive pieces sum to more
// than the limit, so there are at most 2*ceil(ulen/limit) of them.
constexpr uint32_t SnappyMaxPieces(uint64_t ulen, uint32_t limit) {
    return (uint32_t)(2 * ((ulen + limit - 1) / limit) + 1);
}
int LaunchSnappySplit(const SnappyStream* streams_dev, int n, uint32_t piece_limit, SnappyPiece* pieces_dev,
                      int* stream_err_dev, hipStream_t s);
// Decodes the pieces with lo < ulen <= hi (LDS per wave = hi, so small
// pieces run many waves per CU; a second launch takes the large ones) and
// writes their err (0 or a code); the launch with lo == 0 also writes 0 for
// empty slots.
int LaunchSnappyDecompressPieces(const SnappyPiece* pieces_dev, int n, uint32_t lo, uint32_t hi, int* err_dev,
                                 hipStream_t s);
// The serial decoder (one element per wave step) for every size: A/B and
// tests; LaunchSnappyDecompressPieces takes the parallel decoder (source map
// + pointer jumping) for pieces up to 8 KiB.
int LaunchSnappyDecompressPiecesSerial(const SnappyPiece* pieces_dev, int n, uint32_t lo, uint32_t hi, int* err_dev,
                                       hipStream_t s);
// With phase stamps (shader clock, block 0) written to stamps[0..4].
int LaunchSnappyDecompressPiecesStamped(const SnappyPiece* pieces_dev, int n, uint32_t lo, uint32_t hi, int* err_dev,
                                        uint64_t* stamps, hipStream_t s);
// Batched snappy compression: job.src = raw block (<= kSnappyMaxBlock),
// job.dst = output with job.dst_cap >= SnappyMaxCompressedLength(src_len).
// scratch: n * SnappyCompressScratchPerBlock() bytes of device memory.
// out_len_dev[i] = compressed size, err_dev[i] = 0 or an error code.
constexpr uint32_t SnappyCompressSlot() { return ((kSnappyMaxBlock / 64) + 32 + 63) & ~63u; }
constexpr uint64_t SnappyCompressScratchPerBlock() { return 64ull * SnappyCompressSlot(); }
constexpr uint64_t SnappyMaxCompressedLength(uint64_t n) { return 32 + n + n / 6; }
// max_ulen (>= every job's src_len) sizes the LDS: the block is staged in
// LDS, and blocks up to 16 KiB keep their output slots there too (scratch
// is then unused).
int LaunchSnappyCompress(const SnappyJob* jobs_dev, int n, uint32_t max_ulen, void* scratch, uint32_t* out_len_dev,
                         int* err_dev, hipStream_t s);
// Same, stamping block 0's phases (shader clock) into stamps[0..4]: start,
// staged, earliest-position table built, matched, written.
int LaunchSnappyCompressStamped(const SnappyJob* jobs_dev, int n, uint32_t max_ulen, void* scratch,
                                uint32_t* out_len_dev, int* err_dev, uint64_t* stamps, hipStream_t s);
// Whether a launch with this max_ulen writes the global scratch (blocks
// above 16 KiB); otherwise scratch may be null.
constexpr bool SnappyCompressUsesScratch(uint32_t max_ulen) { return max_ulen > 16384; }

// Batched protobuf wire scan (gpu/pb_kernels.hip): message i is
// buf[offsets[i], offsets[i+1]); its top-level fields land in
// fields[i * max_fields * 2 + 2k] = tag, [.. + 1] = value (varint / fixed /
// (offset << 32) | length); nfields[i] = count or a negative error code
// (-5: the offsets of message i leave [0, buf_len) or descend).
int LaunchPbScan(const uint8_t* buf, uint64_t buf_len, const int64_t* offsets_dev, int64_t n, uint32_t max_fields,
                 uint64_t* fields, int32_t* nfields, hipStream_t s);
// Same scan for messages in separate buffers: job i is buf[0, len) (device
// or device-readable pinned table).
struct PbScanJob {
    const uint8_t* buf;
    uint64_t len;
};
int LaunchPbScanPtrs(const PbScanJob* jobs, int64_t n, uint32_t max_fields, uint64_t* fields, int32_t* nfields,
                     hipStream_t s);

// Fused device-body codec launch (codec_waves_kernel, snappy_kernels.hip):
// ONE launch runs a codec batch's compress blocks and headerless decode
// pieces, each at most kFusedMaxBlock uncompressed bytes, one wave per block
// or piece (the per-lane-segment compressor and the wave decoder); a
// message's field table follows as a pb-scan launch, or (opt-in) the wave
// that finished its last piece scans it.
constexpr uint32_t kFusedMaxBlock = 8192;
constexpr uint32_t kFusedNoGroup = 0xFFFFFFFFu;
struct FusedCodecArgs {
    const SnappyJob* comp = nullptr;  // compress jobs (device-readable table)
    int ncomp = 0;
    uint32_t* comp_len = nullptr;
    int* comp_err = nullptr;          // 0, 1 (block too large), 2 (output exceeds dst_cap)
    const SnappyPiece* pieces = nullptr;
    int npieces = 0;
    int* piece_err = nullptr;         // 0, 1 (too large), 3 (element chain leaves the piece), 4 (size), 6 (offset)
    const uint32_t* piece_group = nullptr;  // per piece: scan group, or kFusedNoGroup
    const PbScanJob* scans = nullptr;       // per group: the message its pieces form
    const uint32_t* group_pieces = nullptr; // per group: how many pieces decode into it
    uint32_t* group_done = nullptr;         // per group: HBM counter, zero between launches
    uint64_t* scan_fields = nullptr;        // per group: max_fields {tag, value} rows
    int32_t* scan_n = nullptr;
    uint32_t max_fields = 0;
    uint32_t max_ulen = 0;                  // >= every block's and piece's size
};
int LaunchCodecWaves(const FusedCodecArgs& a, hipStream_t s);


// Batched encoder of repeated numeric runs (SURVEY K2, and the number
// arrays of pb2json, K6): one workgroup per chunk of <= kPbRunChunkElems
// elements, read in the std::vector layout of the field (1/4/8 bytes per
// element), written as protobuf varints (the payload of a packed field) or
// as comma-separated JSON numbers. The host knows every chunk's output size
// (its size pass) and so its destination: chunks of many runs of many
// messages go into one launch with no device-side scan across chunks.
constexpr uint32_t kPbRunChunkElems = 2048;
enum PbRunKind : uint32_t {
    PB_RUN_INT32 = 0,   // int32/enum: sign-extended to 64 bits (negative -> 10 bytes)
    PB_RUN_UINT32 = 1,
    PB_RUN_SINT32 = 2,  // zigzag32
    PB_RUN_INT64 = 3,
    PB_RUN_UINT64 = 4,
    PB_RUN_SINT64 = 5,  // zigzag64
    PB_RUN_BOOL = 6,    // one byte per element
};
enum PbRunFormat : uint32_t {
    PB_RUN_VARINT = 0,
    PB_RUN_DECIMAL = 1,  // JSON: "v,v,...,v" (true/false for bools); no trailing comma on a run's last chunk
};
struct PbRunChunk {
    const void* src;  // this chunk's first element (device-readable)
    uint8_t* dst;     // this chunk's first output byte (device-writable)
    uint32_t count;   // elements, 1..kPbRunChunkElems
    uint32_t kind;    // PbRunKind
    uint32_t format;  // PbRunFormat
    uint32_t last;    // 1: the run's last chunk (decimal: no trailing comma)
    uint32_t bytes;   // output size the host computed; a mismatch is reported and nothing is written
    uint32_t pad;
};
// err[i] is set to 0 (ok) or 1 (size mismatch) for every chunk.
int LaunchPbRunEncode(const PbRunChunk* chunks, int n, int32_t* err, hipStream_t s);

// Batched decoder of packed varint runs (the parse half of K2: large packed
// fields of a body the device already decoded): a run is cut into chunks of
// <= kPbRunDecodeChunkBytes; pass 1 counts the varints ending in each chunk
// (into counts, and into `prefix`, device memory of n entries, which one
// workgroup then scans), pass 2 gives every chunk its first element index
// (prefix[chunk] - prefix[run's first chunk]) and writes each varint ending in it,
// converted to the field's vector layout, at dst[index]. A varint belongs
// to the chunk its last byte is in, so one may start up to 9 bytes into the
// previous chunk (read from there). Codes in err: 0 ok, 1 a varint longer
// than 10 bytes (or a 10th byte above 1).
constexpr uint32_t kPbRunDecodeChunkBytes = 4096;
struct PbRunDecodeChunk {
    const uint8_t* run;  // the run's first byte (device-readable)
    void* dst;           // the run's output array (kind's vector layout)
    uint32_t offset;     // this chunk's first byte within the run
    uint32_t len;        // bytes in the chunk, 1..kPbRunDecodeChunkBytes
    uint32_t first;      // table index of the run's first chunk
    uint32_t kind;       // PbRunKind
};
int LaunchPbRunDecode(const PbRunDecodeChunk* chunks, int n, uint32_t* counts, uint32_t* prefix, int32_t* err,
                      hipStream_t s);

// JSON structural index (gpu/json_kernels.hip): out_pos receives, in order,
// the byte offsets of every unescaped '"' and of every { } [ ] : , outside
// strings; count_dev the number found (positions past max_out are dropped
// and err |= 2); err |= 1 when a string is left open at the end. n < 4 GiB.
// JSON integer arrays (K6 parse half): element i of an array is the text
// between separators seps[i] and seps[i+1] (the '[' / ',' / ']' positions of
// the structural index); one lane per element trims whitespace and parses
// -?[0-9]+ into out[i] as int64. Any element that is not such an integer
// (a float, a literal, out of int64 range) sets *bad = 1: the host then
// parses the array itself. *bad must be 0 before the launch.
int LaunchJsonIntArray(const char* text, const uint32_t* seps, uint32_t n, int64_t* out, int32_t* bad,
                       hipStream_t s);
// scratch must hold JsonIndexScratchBytes(n).
size_t JsonIndexScratchBytes(uint64_t n);
int LaunchJsonIndex(const uint8_t* in, uint64_t n, uint32_t* out_pos, uint64_t max_out, uint64_t* count_dev,
                    int* err_dev, void* scratch, hipStream_t s);

// ---- resident copy worker (persistent kernel fed from a pinned ring;
// kernels.hip explains the protocol). Created on first use per device
// (nullptr: unavailable); instances exit after idle_us without work or
// max_us of life and are relaunched on demand.
struct ResidentRing;
ResidentRing* ResidentRingFor(int device, uint32_t idle_us, uint32_t max_us, uint32_t groups);
// Publish segs as ring batches (groups of <= kInlineSegments segments that
// never split a message; msg_of as in LaunchBatchedCopyCrc32cMessages, null:
// one message per segment). crc_out (pinned host, null: copy only) receives
// one CRC32C per message; a null segment dst only checksums. [first, last]
// are the batches' sequence numbers. 0 on success.
int ResidentSubmit(ResidentRing* r, const Segment* segs, const int* msg_of, int nseg, uint32_t* crc_out,
                   uint64_t* first_seq, uint64_t* last_seq);
// Whether every batch of [first, last] is complete (reads pinned memory).
bool ResidentDone(ResidentRing* r, uint64_t first_seq, uint64_t last_seq);
// Watchdog: relaunch when no instance is on the device but a batch waits.
void ResidentKick(ResidentRing* r);
// Stop every instance and wait for them (process exit).
void ResidentShutdown();
struct ResidentStats {
    int64_t launches = 0, batches = 0, ring_full_waits = 0;
};
ResidentStats GetResidentStats();

// ---- synchronous helpers (fiber-friendly waits)
// CRC32C of device buffers; results to host.
int Crc32cDevice(const void* const* ptrs, const uint64_t* lens, int n, uint32_t* out_host, int device);
int Crc32cOfBuf(const Buf& b, uint32_t* out, int device);  // any block kinds

}  // namespace gpu
}  // namespace mrpc
