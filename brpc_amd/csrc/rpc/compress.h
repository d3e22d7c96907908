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

}  // namespace mrpc
