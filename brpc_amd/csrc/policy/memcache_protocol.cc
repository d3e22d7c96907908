// Memcache binary protocol client (role of the reference's
// src/brpc/policy/memcache_binary_protocol.cpp): operations are pipelined;
// responses map to calls through the socket's pipelined-info queue.
#include <memory>

#include "base/logging.h"
#include "fiber/call_id.h"
#include "net/input_messenger.h"
#include "policy/authenticators.h"
#include "policy/policies.h"
#include "redis/memcache.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/protocol.h"

namespace mrpc {
namespace policy {

namespace {
class McContext : public ParsingContext {
public:
    static const int kTag = 0x4D43434C;  // "MCCL"
    int protocol_tag() const override { return kTag; }
    MemcacheResponse partial;
    PipelinedInfo pi;
    bool has_pi = false;
};

class McMessage : public InputMessageBase {
public:
    MemcacheResponse response;
    PipelinedInfo pi;
};
}  // namespace

ParseResult ParseMemcacheMessage(Buf* source, Socket* socket, bool, const void*) {
    if (source->empty()) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    if (socket->user() != get_client_side_messenger()) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    ParsingContext* pc = socket->parsing_context();
    McContext* ctx;
    if (pc) {
        if (pc->protocol_tag() != McContext::kTag) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        ctx = static_cast<McContext*>(pc);
    } else {
        unsigned char magic;
        source->copy_to(&magic, 1);
        PipelinedInfo peek;
        if (magic != 0x81 || !socket->PeekPipelinedInfo(&peek) || peek.protocol != PROTOCOL_MEMCACHE) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        ctx = new McContext;
        if (!socket->InstallParsingContext(ctx)) {
            delete ctx;
            return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        }
    }
    if (!ctx->has_pi) {
        if (!socket->PopPipelinedInfo(&ctx->pi)) return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
        ctx->has_pi = true;
        ctx->partial.Clear();
    }
    if (ctx->pi.auth_replies > 0) {
        // the SASL reply to the bucket credential sent in front of this
        // request (reference: memcache_binary_protocol.cpp:130-138)
        unsigned char h[24];
        if (source->copy_to(h, sizeof(h)) < sizeof(h)) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
        const uint32_t body = ((uint32_t)h[8] << 24) | ((uint32_t)h[9] << 16) | ((uint32_t)h[10] << 8) | h[11];
        if (source->size() < sizeof(h) + body) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
        const uint16_t status = (uint16_t)((h[6] << 8) | h[7]);
        if (h[1] != kMemcacheSaslAuth || status != 0) {
            LOG(ERROR) << "couchbase bucket authentication failed (status " << status << ")";
            return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
        }
        source->pop_front(sizeof(h) + body);
        ctx->pi.auth_replies = 0;
        if (source->empty()) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    }
    const int rc = ctx->partial.ConsumePartial(source, ctx->pi.count);
    if (rc < 0) return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
    if (rc == 0) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    McMessage* m = new McMessage;
    std::swap(m->response, ctx->partial);
    m->pi = ctx->pi;
    ctx->has_pi = false;
    return MakeMessage(m);
}

void SerializeMemcacheRequest(Buf* buf, Controller* cntl, const pb::Message* request) {
    const MemcacheRequest* r = dynamic_cast<const MemcacheRequest*>(request);
    if (!r || r->op_count() == 0) {
        cntl->SetFailed(EREQUEST, "request must be a non-empty MemcacheRequest");
        return;
    }
    buf->append(r->raw());
    cntl->_pipelined_count = r->op_count();
}

void PackMemcacheRequest(Buf* packet, uint64_t, const pb::MethodDescriptor*, Controller* cntl, const Buf& request_buf,
                         const Authenticator* auth) {
    if (auth) {  // first request of the connection: SASL credential in front
        std::string cred;
        if (auth->GenerateCredential(&cred) != 0) {
            cntl->SetFailed(ERPCAUTH, "fail to generate memcache credential");
            return;
        }
        packet->append(cred);
        cntl->_auth_replies = 1;
    }
    packet->append(request_buf);
    if (cntl->_pipelined_count <= 0) cntl->_pipelined_count = 1;
}

void ProcessMemcacheResponse(InputMessageBase* msg_base) {
    std::unique_ptr<McMessage> msg(static_cast<McMessage*>(msg_base));
    const fiber::CallId cid = msg->pi.id_wait;
    Controller* cntl = nullptr;
    if (fiber::call_id_lock(cid, (void**)&cntl) != 0) return;
    if (cid != cntl->current_id() && cid != cntl->_unfinished_call.id) {
        fiber::call_id_unlock(cid);
        return;
    }
    int saved_error = 0;
    if (MemcacheResponse* res = dynamic_cast<MemcacheResponse*>(cntl->_response)) {
        std::swap(*res, msg->response);
    } else if (cntl->_response) {
        saved_error = ERESPONSE;
        cntl->SetFailed(ERESPONSE, "response must be a MemcacheResponse");
    }
    msg.reset();
    cntl->OnVersionedRPCReturned(cid, saved_error);
}

void RegisterMemcacheProtocol() {
    Protocol p;
    p.parse = ParseMemcacheMessage;
    p.serialize_request = SerializeMemcacheRequest;
    p.pack_request = PackMemcacheRequest;
    p.process_response = ProcessMemcacheResponse;
    p.supported_connection_type = CONNECTION_TYPE_SINGLE | CONNECTION_TYPE_POOLED | CONNECTION_TYPE_SHORT;
    p.name = "memcache";
    RegisterProtocol(PROTOCOL_MEMCACHE, p);
}

}  // namespace policy
}  // namespace mrpc
