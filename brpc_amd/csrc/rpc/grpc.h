// gRPC conventions over HTTP/2 (role of the reference's src/brpc/grpc.h,
// grpc.cpp:29-171): status codes, the mapping to/from RPC error codes,
// grpc-timeout values, grpc-message percent encoding and the 5-byte
// length-prefixed message framing.
#pragma once

#include <cstdint>
#include <string>

#include "base/buf.h"

namespace mrpc {

enum GrpcStatus {
    GRPC_OK = 0,
    GRPC_CANCELED = 1,
    GRPC_UNKNOWN = 2,
    GRPC_INVALIDARGUMENT = 3,
    GRPC_DEADLINEEXCEEDED = 4,
    GRPC_NOTFOUND = 5,
    GRPC_ALREADYEXISTS = 6,
    GRPC_PERMISSIONDENIED = 7,
    GRPC_RESOURCEEXHAUSTED = 8,
    GRPC_FAILEDPRECONDITION = 9,
    GRPC_ABORTED = 10,
    GRPC_OUTOFRANGE = 11,
    GRPC_UNIMPLEMENTED = 12,
    GRPC_INTERNAL = 13,
    GRPC_UNAVAILABLE = 14,
    GRPC_DATALOSS = 15,
    GRPC_UNAUTHENTICATED = 16,
};

GrpcStatus ErrorCodeToGrpcStatus(int error_code);
int GrpcStatusToErrorCode(int grpc_status);
// "100m", "2S", "5000u" ... -> microseconds (-1 if malformed)
int64_t ConvertGrpcTimeoutToUS(const std::string& v);
std::string ConvertUSToGrpcTimeout(int64_t us);
std::string PercentEncode(const std::string& s);
std::string PercentDecode(const std::string& s);
// 5-byte prefix: compressed flag + big-endian length
void AddGrpcPrefix(Buf* out, const Buf& message, bool compressed);
// Cuts one length-prefixed message from `in`. Returns 1 ok, 0 not enough
// data, -1 malformed.
int RemoveGrpcPrefix(Buf* in, Buf* message, bool* compressed);
// grpc-encoding names <-> compress types ("identity" = none, "gzip",
// "deflate" = zlib, "snappy"). Unknown names map to -1.
int GrpcEncodingToCompressType(const std::string& name);
const char* CompressTypeToGrpcEncoding(int type);

}  // namespace mrpc
