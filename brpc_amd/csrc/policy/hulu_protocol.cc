// hulu_pbrpc (role of the reference's src/brpc/policy/hulu_pbrpc_protocol.cpp):
//   "HULU" | body_size (u32, little endian) | meta_size (u32, LE) | meta | message | attachment
// Methods are addressed by the SHORT service name + the method's index in the
// service; `user_message_size` separates the pb message from a raw
// attachment. Hulu's compress numbering (none/snappy/gzip/zlib = 0..3)
// coincides with CompressType, so no translation table is needed.
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

static const size_t kHuluHeader = 12;

static void PackHuluFrame(Buf* out, const pb::Message& meta, const Buf& body, const Buf& attachment) {
    const uint32_t meta_size = (uint32_t)meta.ByteSizeLong();
    char* p = out->append_contiguous(kHuluHeader + meta_size);
    memcpy(p, "HULU", 4);
    pack_le32(p + 4, (uint32_t)(meta_size + body.size() + attachment.size()));
    pack_le32(p + 8, meta_size);
    meta.SerializeWithCachedSizesToArray((uint8_t*)p + kHuluHeader);
    out->append(body);
    out->append(attachment);
}

ParseResult ParseHuluMessage(Buf* source, Socket* socket, bool, const void*) {
    char h[kHuluHeader];
    const size_t n = source->copy_to(h, sizeof(h));
    if (memcmp(h, "HULU", n < 4 ? n : 4) != 0) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    if (n < kHuluHeader) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    const uint32_t body_size = unpack_le32(h + 4);
    const uint32_t meta_size = unpack_le32(h + 8);
    if (body_size > FLAGS_max_body_size) {
        LOG(ERROR) << "hulu body_size=" << body_size << " from " << socket->remote_side() << " is too large";
        return MakeParseError(PARSE_ERROR_TOO_BIG_DATA);
    }
    if (meta_size > body_size) return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
    if (source->size() < kHuluHeader + body_size) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    source->pop_front(kHuluHeader);
    MostCommonMessage* msg = MostCommonMessage::Get();
    source->cutn(&msg->meta, meta_size);
    source->cutn(&msg->payload, body_size - meta_size);
    return MakeMessage(msg);
}

// Splits payload into (message, attachment) by the meta's user_message_size.
static bool SplitUserMessage(Buf* payload, bool has_size, int32_t size, Buf* body, Buf* attachment) {
    if (!has_size) {
        body->swap(*payload);
        return true;
    }
    if (size < 0 || (size_t)size > payload->size()) return false;
    payload->cutn(body, (size_t)size);
    attachment->swap(*payload);
    return true;
}

void ProcessHuluRequest(InputMessageBase* base) {
    MostCommonMessage* msg = static_cast<MostCommonMessage*>(base);
    Socket* socket = msg->socket();
    HuluRpcRequestMeta meta;
    if (!ParsePbFromBuf(&meta, msg->meta)) {
        socket->SetFailed(EREQUEST, "fail to parse HuluRpcRequestMeta");
        msg->Destroy();
        return;
    }
    PbServerRequest r;
    r.server = const_cast<Server*>(static_cast<const Server*>(msg->arg()));
    r.socket = socket;
    r.received_us = msg->received_us();
    r.protocol = PROTOCOL_HULU_PBRPC;
    r.mp = FindMethodByIndex(r.server, meta.service_name(), meta.method_index(), &r.error_code, &r.error_text);
    r.span_method_name = meta.service_name() + "." + std::to_string(meta.method_index());
    r.compress_type = (CompressType)meta.compress_type();
    r.has_log_id = meta.has_log_id();
    r.log_id = (uint64_t)meta.log_id();
    r.trace_id = (uint64_t)meta.trace_id();
    r.span_id = (uint64_t)meta.span_id();
    r.parent_span_id = (uint64_t)meta.parent_span_id();
    r.auth_data = meta.credential_data();
    if (!SplitUserMessage(&msg->payload, meta.has_user_message_size(), meta.user_message_size(), &r.body,
                          &r.attachment)) {
        r.mp = nullptr;
        r.error_code = EREQUEST;
        r.error_text = "user_message_size is larger than the payload";
    }
    const int64_t corr = meta.correlation_id();
    msg->Destroy();
    RunPbServerCall(&r, [corr](Controller* cntl, Buf* body, Buf* attachment, Buf* packet) {
        HuluRpcResponseMeta rm;
        rm.set_correlation_id(corr);
        if (cntl->Failed()) {
            rm.set_error_code(cntl->ErrorCode());
            rm.set_error_text(cntl->ErrorText());
        } else {
            rm.set_compress_type((int32_t)cntl->response_compress_type());
            if (!attachment->empty()) rm.set_user_message_size((int32_t)body->size());
        }
        PackHuluFrame(packet, rm, *body, *attachment);
    });
}

void ProcessHuluResponse(InputMessageBase* base) {
    MostCommonMessage* msg = static_cast<MostCommonMessage*>(base);
    HuluRpcResponseMeta meta;
    if (!ParsePbFromBuf(&meta, msg->meta)) {
        LOG(WARNING) << "Fail to parse HuluRpcResponseMeta from " << msg->socket()->remote_side();
        msg->Destroy();
        return;
    }
    Buf body, attachment;
    int err = meta.error_code();
    std::string text = meta.error_text();
    if (!err && !SplitUserMessage(&msg->payload, meta.has_user_message_size(), meta.user_message_size(), &body,
                                  &attachment)) {
        err = ERESPONSE;
        text = "user_message_size is larger than the payload";
    }
    CompletePbClientCall(fiber::CallId{(uint64_t)meta.correlation_id()}, err, text, &body, &attachment,
                         (CompressType)meta.compress_type(), msg->socket());
    msg->Destroy();
}

void SerializeHuluRequest(Buf* buf, Controller* cntl, const pb::Message* request) {
    if (!request || !request->IsInitialized()) {
        cntl->SetFailed(EREQUEST, "request is NULL or missing required fields");
        return;
    }
    if (!SerializeAsCompressedData(*request, buf, cntl->request_compress_type())) {
        cntl->SetFailed(EREQUEST, "Fail to compress request");
    }
}

void PackHuluRequest(Buf* packet, uint64_t correlation_id, const pb::MethodDescriptor* method, Controller* cntl,
                     const Buf& request_buf, const Authenticator* auth) {
    if (!method) {
        cntl->SetFailed(EREQUEST, "hulu_pbrpc needs a method");
        return;
    }
    HuluRpcRequestMeta meta;
    meta.set_service_name(method->service->name);
    meta.set_method_index(method->index);
    meta.set_method_name(method->name);
    meta.set_compress_type((int32_t)cntl->request_compress_type());
    meta.set_correlation_id((int64_t)correlation_id);
    if (cntl->log_id()) meta.set_log_id((int64_t)cntl->log_id());
    if (cntl->trace_id()) {
        meta.set_trace_id((int64_t)cntl->trace_id());
        meta.set_span_id((int64_t)cntl->span_id());
        if (cntl->_parent_span_id) meta.set_parent_span_id((int64_t)cntl->_parent_span_id);
    }
    if (!cntl->request_attachment().empty()) meta.set_user_message_size((int32_t)request_buf.size());
    if (auth) {
        std::string cred;
        if (auth->GenerateCredential(&cred) != 0) {
            cntl->SetFailed(ERPCAUTH, "Fail to generate credential");
            return;
        }
        meta.set_credential_data(cred);
    }
    PackHuluFrame(packet, meta, request_buf, cntl->request_attachment());
}

void RegisterHuluProtocol() {
    Protocol p;
    p.parse = ParseHuluMessage;
    p.serialize_request = SerializeHuluRequest;
    p.pack_request = PackHuluRequest;
    p.process_request = ProcessHuluRequest;
    p.process_response = ProcessHuluResponse;
    p.supported_connection_type = CONNECTION_TYPE_SINGLE | CONNECTION_TYPE_POOLED | CONNECTION_TYPE_SHORT;
    p.name = "hulu_pbrpc";
    RegisterProtocol(PROTOCOL_HULU_PBRPC, p);
}

}  // namespace policy
}  // namespace mrpc
