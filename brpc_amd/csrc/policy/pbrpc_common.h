// Shared server/client plumbing of the "binary header + pb meta + pb body
// (+ attachment)" protocol family: hulu_pbrpc, sofa_pbrpc, nova_pbrpc,
// public_pbrpc, nshead+pb adaptors. Each protocol only decodes/encodes its
// own framing and meta; admission control, method-status accounting,
// request parsing/decompression, rpcz spans, the user callback and the
// response write are done once here. (The reference repeats this sequence in
// every policy/*_protocol.cpp, e.g. hulu_pbrpc_protocol.cpp:369-540,
// sofa_pbrpc_protocol.cpp:336-470.)
#pragma once

#include <cstdint>
#include <functional>
#include <string>

#include "base/buf.h"
#include "fiber/call_id.h"
#include "mrpc/proto/options.pb.h"
#include "rpc/server.h"

namespace mrpc {
class Socket;
class Controller;
namespace policy {

// What a protocol's process_request knows after decoding its meta.
struct PbServerRequest {
    Server* server = nullptr;
    Socket* socket = nullptr;
    int64_t received_us = 0;
    ProtocolType protocol = PROTOCOL_UNKNOWN;
    // The method, resolved by the protocol (service name+index, full name...).
    // When null, `error_code`/`error_text` say why (ENOSERVICE/ENOMETHOD...).
    const Server::MethodProperty* mp = nullptr;
    int error_code = 0;
    std::string error_text;
    Buf body;        // serialized (possibly compressed) request message
    Buf attachment;  // raw bytes after the message
    CompressType compress_type = COMPRESS_TYPE_NONE;
    int response_compress = -1;  // <0: answer with the request's compression
    bool has_log_id = false;
    uint64_t log_id = 0;
    uint64_t trace_id = 0, span_id = 0, parent_span_id = 0;
    int64_t timeout_ms = 0;
    std::string span_method_name;  // for rpcz when mp is null
    std::string auth_data;         // credential carried by the meta, if any
};

// Builds the protocol-specific response packet. `cntl` carries the error
// (if any); `body` is the serialized+compressed response (empty on error),
// `attachment` the response attachment.
typedef std::function<void(Controller* cntl, Buf* body, Buf* attachment, Buf* packet)> PbResponsePacker;

// Runs the whole server-side call; the request's buffers are consumed.
// Resolves server-wide & per-method admission, parses the request, invokes
// the service, and when done->Run() is called writes `packer`'s packet.
void RunPbServerCall(PbServerRequest* req, PbResponsePacker packer);

// Looks up "service.method" by the short (or full) service name and a
// method index, as hulu/nova/public_pbrpc address methods.
const Server::MethodProperty* FindMethodByIndex(const Server* server, const std::string& service_name,
                                                int method_index, int* error_code, std::string* error_text);
const Server::MethodProperty* FindMethodByFullName(const Server* server, const std::string& full_method_name,
                                                   int* error_code, std::string* error_text);

// Client side: finish call `cid` with the response bytes of one attempt.
// Locks the id, drops stale versions, parses `body` (decompressing by
// `ct`) into the controller's response, moves `attachment` into
// response_attachment and hands over to OnVersionedRPCReturned.
void CompletePbClientCall(fiber::CallId cid, int error_code, const std::string& error_text, Buf* body,
                          Buf* attachment, CompressType ct, Socket* sock);

// Same, for responses whose payload the protocol converts itself (e.g.
// mcpack -> pb). `fill` runs with the id locked and returns an error code
// (0 on success) after writing into cntl->_response.
void CompleteClientCallWith(fiber::CallId cid, Socket* sock, const std::function<int(Controller*)>& fill);

// Little-endian raw packing used by hulu/sofa/nshead (not network order).
inline void pack_le32(char* p, uint32_t v) {
    p[0] = (char)v; p[1] = (char)(v >> 8); p[2] = (char)(v >> 16); p[3] = (char)(v >> 24);
}
inline void pack_le64(char* p, uint64_t v) {
    pack_le32(p, (uint32_t)v);
    pack_le32(p + 4, (uint32_t)(v >> 32));
}
inline uint32_t unpack_le32(const char* p) {
    const unsigned char* u = (const unsigned char*)p;
    return (uint32_t)u[0] | ((uint32_t)u[1] << 8) | ((uint32_t)u[2] << 16) | ((uint32_t)u[3] << 24);
}
inline uint64_t unpack_le64(const char* p) { return (uint64_t)unpack_le32(p) | ((uint64_t)unpack_le32(p + 4) << 32); }

}  // namespace policy
}  // namespace mrpc
