// Snappy-format block compression (own implementation of the public snappy
// format; the reference vendors google snappy, butil/third_party/snappy).
// Input is processed in independent 64 KB fragments, which is also the unit
// of parallelism of the HIP kernels in ops/snappy.hip.
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>

namespace mrpc {
namespace snappy {

size_t MaxCompressedLength(size_t n);
// Returns compressed size written to out (must hold MaxCompressedLength).
size_t RawCompress(const char* in, size_t n, char* out);
bool Compress(const char* in, size_t n, std::string* out);
bool GetUncompressedLength(const char* in, size_t n, size_t* result);
// out must hold the uncompressed length.
bool RawUncompress(const char* in, size_t n, char* out);
bool Uncompress(const char* in, size_t n, std::string* out);
bool IsValidCompressedBuffer(const char* in, size_t n);

// Compress one fragment (<= 64KB) without the length preamble. Used by the
// device path which emits fragments independently then stitches.
size_t CompressFragment(const char* in, size_t n, char* out);

}  // namespace snappy
}  // namespace mrpc
