// sofa_pbrpc (role of the reference's src/brpc/policy/sofa_pbrpc_protocol.cpp):
//   "SOFA" | meta_size (u32 LE) | body_size (u64 LE) | meta_size+body_size (u64 LE) | SofaRpcMeta | body
// Methods are addressed by their full name; the format has no attachment.
// Sofa numbers compressors differently (gzip=1, zlib=2, snappy=3).
#include "base/flags.h"
#include "base/logging.h"
#include "mrpc/proto/legacy_meta.pb.h"
#include "policy/pbrpc_common.h"
#include "policy/policies.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/protocol.h"
#include "rpc/server.h"

DECLARE_uint64(max_body_size);

namespace mrpc {
namespace policy {

static const size_t kSofaHeader = 24;

static CompressType FromSofa(int t) {
    switch (t) {
    case SOFA_COMPRESS_TYPE_GZIP: return COMPRESS_TYPE_GZIP;
    case SOFA_COMPRESS_TYPE_ZLIB: return COMPRESS_TYPE_ZLIB;
    case SOFA_COMPRESS_TYPE_SNAPPY: return COMPRESS_TYPE_SNAPPY;
    case SOFA_COMPRESS_TYPE_LZ4: return COMPRESS_TYPE_LZ4;
    default: return COMPRESS_TYPE_NONE;
    }
}

static SofaCompressType ToSofa(CompressType t) {
    switch (t) {
    case COMPRESS_TYPE_GZIP: return SOFA_COMPRESS_TYPE_GZIP;
    case COMPRESS_TYPE_ZLIB: return SOFA_COMPRESS_TYPE_ZLIB;
    case COMPRESS_TYPE_SNAPPY: return SOFA_COMPRESS_TYPE_SNAPPY;
    case COMPRESS_TYPE_LZ4: return SOFA_COMPRESS_TYPE_LZ4;
    default: return SOFA_COMPRESS_TYPE_NONE;
    }
}

static void PackSofaFrame(Buf* out, const SofaRpcMeta& meta, const Buf& body) {
    const uint32_t meta_size = (uint32_t)meta.ByteSizeLong();
    char* p = out->append_contiguous(kSofaHeader + meta_size);
    memcpy(p, "SOFA", 4);
    pack_le32(p + 4, meta_size);
    pack_le64(p + 8, body.size());
    pack_le64(p + 16, meta_size + body.size());
    meta.SerializeWithCachedSizesToArray((uint8_t*)p + kSofaHeader);
    out->append(body);
}

ParseResult ParseSofaMessage(Buf* source, Socket* socket, bool, const void*) {
    char h[kSofaHeader];
    const size_t n = source->copy_to(h, sizeof(h));
    if (memcmp(h, "SOFA", n < 4 ? n : 4) != 0) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    if (n < kSofaHeader) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    const uint32_t meta_size = unpack_le32(h + 4);
    const uint64_t body_size = unpack_le64(h + 8);
    const uint64_t total = unpack_le64(h + 16);
    if (total != meta_size + body_size) {
        LOG(ERROR) << "sofa: inconsistent sizes meta=" << meta_size << " body=" << body_size << " total=" << total;
        return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
    }
    if (total > FLAGS_max_body_size) {
        LOG(ERROR) << "sofa body of " << total << " bytes from " << socket->remote_side() << " is too large";
        return MakeParseError(PARSE_ERROR_TOO_BIG_DATA);
    }
    if (source->size() < kSofaHeader + total) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    source->pop_front(kSofaHeader);
    MostCommonMessage* msg = MostCommonMessage::Get();
    source->cutn(&msg->meta, meta_size);
    source->cutn(&msg->payload, body_size);
    return MakeMessage(msg);
}

void ProcessSofaRequest(InputMessageBase* base) {
    MostCommonMessage* msg = static_cast<MostCommonMessage*>(base);
    Socket* socket = msg->socket();
    SofaRpcMeta meta;
    if (!ParsePbFromBuf(&meta, msg->meta) || meta.type() != SofaRpcMeta::REQUEST) {
        socket->SetFailed(EREQUEST, "fail to parse SofaRpcMeta");
        msg->Destroy();
        return;
    }
    PbServerRequest r;
    r.server = const_cast<Server*>(static_cast<const Server*>(msg->arg()));
    r.socket = socket;
    r.received_us = msg->received_us();
    r.protocol = PROTOCOL_SOFA_PBRPC;
    r.mp = FindMethodByFullName(r.server, meta.method(), &r.error_code, &r.error_text);
    r.span_method_name = meta.method();
    r.compress_type = FromSofa(meta.compress_type());
    r.body.swap(msg->payload);
    if (meta.has_expected_response_compress_type()) r.response_compress = FromSofa(meta.expected_response_compress_type());
    const uint64_t seq = meta.sequence_id();
    msg->Destroy();
    RunPbServerCall(&r, [seq](Controller* cntl, Buf* body, Buf*, Buf* packet) {
        SofaRpcMeta rm;
        rm.set_type(SofaRpcMeta::RESPONSE);
        rm.set_sequence_id(seq);
        if (cntl->Failed()) {
            rm.set_failed(true);
            rm.set_error_code(cntl->ErrorCode());
            rm.set_reason(cntl->ErrorText());
        } else {
            rm.set_compress_type(ToSofa(cntl->response_compress_type()));
        }
        PackSofaFrame(packet, rm, *body);
    });
}

void ProcessSofaResponse(InputMessageBase* base) {
    MostCommonMessage* msg = static_cast<MostCommonMessage*>(base);
    SofaRpcMeta meta;
    if (!ParsePbFromBuf(&meta, msg->meta) || meta.type() != SofaRpcMeta::RESPONSE) {
        LOG(WARNING) << "Fail to parse SofaRpcMeta from " << msg->socket()->remote_side();
        msg->Destroy();
        return;
    }
    int err = 0;
    if (meta.failed()) err = meta.error_code() ? meta.error_code() : EINTERNAL;
    CompletePbClientCall(fiber::CallId{meta.sequence_id()}, err, meta.reason(), &msg->payload, nullptr,
                         FromSofa(meta.compress_type()), msg->socket());
    msg->Destroy();
}

void SerializeSofaRequest(Buf* buf, Controller* cntl, const pb::Message* request) {
    if (!request || !request->IsInitialized()) {
        cntl->SetFailed(EREQUEST, "request is NULL or missing required fields");
        return;
    }
    if (!cntl->request_attachment().empty()) {
        cntl->SetFailed(EREQUEST, "sofa_pbrpc does not support attachment");
        return;
    }
    if (!SerializeAsCompressedData(*request, buf, cntl->request_compress_type())) {
        cntl->SetFailed(EREQUEST, "Fail to compress request");
    }
}

void PackSofaRequest(Buf* packet, uint64_t correlation_id, const pb::MethodDescriptor* method, Controller* cntl,
                     const Buf& request_buf, const Authenticator*) {
    if (!method) {
        cntl->SetFailed(EREQUEST, "sofa_pbrpc needs a method");
        return;
    }
    SofaRpcMeta meta;
    meta.set_type(SofaRpcMeta::REQUEST);
    meta.set_sequence_id(correlation_id);
    meta.set_method(method->full_name);
    meta.set_compress_type(ToSofa(cntl->request_compress_type()));
    meta.set_expected_response_compress_type(ToSofa(cntl->response_compress_type()));
    PackSofaFrame(packet, meta, request_buf);
}

void RegisterSofaProtocol() {
    Protocol p;
    p.parse = ParseSofaMessage;
    p.serialize_request = SerializeSofaRequest;
    p.pack_request = PackSofaRequest;
    p.process_request = ProcessSofaRequest;
    p.process_response = ProcessSofaResponse;
    p.supported_connection_type = CONNECTION_TYPE_SINGLE | CONNECTION_TYPE_POOLED | CONNECTION_TYPE_SHORT;
    p.name = "sofa_pbrpc";
    RegisterProtocol(PROTOCOL_SOFA_PBRPC, p);
}

}  // namespace policy
}  // namespace mrpc
