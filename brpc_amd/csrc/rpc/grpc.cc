#include "rpc/grpc.h"

#include "rpc/compress.h"

#include <cerrno>
#include <cstdio>
#include <cstdlib>

#include "rpc/errno.h"

namespace mrpc {

GrpcStatus ErrorCodeToGrpcStatus(int ec) {
    switch (ec) {
    case 0: return GRPC_OK;
    case ENOSERVICE:
    case ENOMETHOD: return GRPC_UNIMPLEMENTED;
    case ERPCAUTH: return GRPC_UNAUTHENTICATED;
    case EREQUEST:
    case EINVAL: return GRPC_INVALIDARGUMENT;
    case ELIMIT:
    case EOVERCROWDED: return GRPC_RESOURCEEXHAUSTED;
    case ELOGOFF:
    case EFAILEDSOCKET:
    case EHOSTDOWN: return GRPC_UNAVAILABLE;
    case ERPCTIMEDOUT:
    case ETIMEDOUT: return GRPC_DEADLINEEXCEEDED;
    case ECANCELED: return GRPC_CANCELED;
    case EPERM: return GRPC_PERMISSIONDENIED;
    case ERESPONSE:
    case EINTERNAL: return GRPC_INTERNAL;
    default: return GRPC_UNKNOWN;
    }
}

int GrpcStatusToErrorCode(int s) {
    switch (s) {
    case GRPC_OK: return 0;
    case GRPC_CANCELED: return ECANCELED;
    case GRPC_INVALIDARGUMENT: return EREQUEST;
    case GRPC_DEADLINEEXCEEDED: return ERPCTIMEDOUT;
    case GRPC_NOTFOUND: return ENOENT;
    case GRPC_PERMISSIONDENIED: return EPERM;
    case GRPC_RESOURCEEXHAUSTED: return ELIMIT;
    case GRPC_UNIMPLEMENTED: return ENOMETHOD;
    case GRPC_UNAVAILABLE: return EFAILEDSOCKET;
    case GRPC_UNAUTHENTICATED: return ERPCAUTH;
    case GRPC_INTERNAL: return EINTERNAL;
    default: return EINTERNAL;
    }
}

int64_t ConvertGrpcTimeoutToUS(const std::string& v) {
    if (v.size() < 2 || v.size() > 9) return -1;
    char* end = nullptr;
    const long long n = strtoll(v.c_str(), &end, 10);
    if (end != v.c_str() + v.size() - 1 || n < 0) return -1;
    switch (v.back()) {
    case 'H': return n * 3600LL * 1000000;
    case 'M': return n * 60LL * 1000000;
    case 'S': return n * 1000000LL;
    case 'm': return n * 1000LL;
    case 'u': return n;
    case 'n': return (n + 999) / 1000;
    default: return -1;
    }
}

std::string ConvertUSToGrpcTimeout(int64_t us) {
    if (us <= 0) return "0u";
    if (us < 100000000LL) return std::to_string(us) + "u";  // at most 8 digits
    const int64_t ms = us / 1000;
    if (ms < 100000000LL) return std::to_string(ms) + "m";
    const int64_t s = us / 1000000;
    if (s < 100000000LL) return std::to_string(s) + "S";
    return std::to_string(s / 60) + "M";
}

std::string PercentEncode(const std::string& s) {
    std::string out;
    for (unsigned char c : s) {
        if (c >= 0x20 && c <= 0x7e && c != '%') {
            out.push_back((char)c);
        } else {
            char buf[4];
            snprintf(buf, sizeof(buf), "%%%02X", c);
            out.append(buf);
        }
    }
    return out;
}

std::string PercentDecode(const std::string& s) {
    std::string out;
    for (size_t i = 0; i < s.size(); ++i) {
        if (s[i] == '%' && i + 2 < s.size()) {
            const std::string hex = s.substr(i + 1, 2);
            char* end = nullptr;
            const long v = strtol(hex.c_str(), &end, 16);
            if (end == hex.c_str() + 2) {
                out.push_back((char)v);
                i += 2;
                continue;
            }
        }
        out.push_back(s[i]);
    }
    return out;
}

void AddGrpcPrefix(Buf* out, const Buf& message, bool compressed) {
    char head[5];
    head[0] = compressed ? 1 : 0;
    const uint32_t n = (uint32_t)message.size();
    head[1] = (char)(n >> 24);
    head[2] = (char)(n >> 16);
    head[3] = (char)(n >> 8);
    head[4] = (char)n;
    out->append(head, 5);
    out->append(message);
}

int RemoveGrpcPrefix(Buf* in, Buf* message, bool* compressed) {
    if (in->size() < 5) return 0;
    unsigned char head[5];
    in->copy_to(head, 5);
    if (head[0] > 1) return -1;
    const uint32_t n = ((uint32_t)head[1] << 24) | ((uint32_t)head[2] << 16) | ((uint32_t)head[3] << 8) | head[4];
    if (in->size() < 5 + (size_t)n) return 0;
    in->pop_front(5);
    in->cutn(message, n);
    if (compressed) *compressed = head[0] == 1;
    return 1;
}

int GrpcEncodingToCompressType(const std::string& name) {
    if (name.empty() || name == "identity") return COMPRESS_TYPE_NONE;
    if (name == "gzip") return COMPRESS_TYPE_GZIP;
    if (name == "deflate") return COMPRESS_TYPE_ZLIB;
    if (name == "snappy") return COMPRESS_TYPE_SNAPPY;
    return -1;
}

const char* CompressTypeToGrpcEncoding(int type) {
    switch (type) {
    case COMPRESS_TYPE_GZIP: return "gzip";
    case COMPRESS_TYPE_ZLIB: return "deflate";
    case COMPRESS_TYPE_SNAPPY: return "snappy";
    default: return "identity";
    }
}

}  // namespace mrpc
