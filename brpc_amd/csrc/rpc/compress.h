// Compression registry (role of src/brpc/compress.cpp:29-92,
// policy/snappy_compress.cpp, policy/gzip_compress.cpp): snappy (own
// implementation, optionally on GPU via ops/snappy.hip for large bodies),
// gzip and zlib (zlib library).
#pragma once

#include <string>

#include "base/buf.h"
#include "mrpc/proto/options.pb.h"

namespace mrpc {

struct CompressHandler {
    // Compress `in` into *out (appends). false on failure.
    bool (*Compress)(const Buf& in, Buf* out) = nullptr;
    bool (*Decompress)(const Buf& in, Buf* out) = nullptr;
    const char* name = nullptr;
};

int RegisterCompressHandler(CompressType type, const CompressHandler& h);
const CompressHandler* FindCompressHandler(CompressType type);
const char* CompressTypeToCStr(CompressType type);
void RegisterBuiltinCompressHandlers();

bool CompressBuf(CompressType type, const Buf& in, Buf* out);
bool DecompressBuf(CompressType type, const Buf& in, Buf* out);

// Hook so that the GPU module can take over snappy for large buffers.
typedef bool (*SnappyOffload)(const Buf& in, Buf* out, bool compress);
void SetSnappyOffload(SnappyOffload fn, size_t min_bytes);

// Hook for decompress + parse in one device pass (GPU snappy decode, then
// the pb wire-scan kernel indexes the message's top-level fields, so the
// host merges fields from a table instead of walking the bytes). Returns
// 1 when *msg is parsed, 0 when the hook declines (the CPU path runs), -1
// when the data is malformed.
namespace pb {
class Message;
}
// Serialize-and-compress offload for snappy bodies of at least min_bytes
// (serialized size): the device codec serializes the message straight into
// memory its kernel reads (pinned) and compresses from there, so the body
// is written once on the host instead of serialized and then copied.
// Returns false to fall back to serialize + CompressBuf.
typedef bool (*SnappyPackOffload)(const pb::Message& msg, size_t serialized_size, Buf* out);
void SetSnappyPackOffload(SnappyPackOffload fn, size_t min_bytes);
bool TrySnappyPackOffload(const pb::Message& msg, Buf* out);

typedef int (*PbParseOffload)(const Buf& compressed, CompressType type, pb::Message* msg);
void SetPbParseOffload(PbParseOffload fn, size_t min_bytes);
// Runs the hook for `type` if one is installed and the body is large
// enough; same return codes, 0 without a hook.
int TryPbParseOffload(const Buf& compressed, CompressType type, pb::Message* msg);

}  // namespace mrpc
