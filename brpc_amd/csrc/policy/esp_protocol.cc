// ESP client protocol (role of the reference's src/brpc/policy/esp_protocol.cpp).
// The reference ties one outstanding call to a connection
// (Socket::correlation_id); here each write records (call id, ESP tag) in
// the socket's pipelined-info queue, so a single connection can carry
// pipelined ESP calls answered in order.
#include "base/flags.h"
#include "base/logging.h"
#include "net/input_messenger.h"
#include "policy/pbrpc_common.h"
#include "policy/policies.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/esp.h"
#include "rpc/protocol.h"

DECLARE_uint64(max_body_size);

namespace mrpc {
namespace policy {

static const uint32_t kEspTag = 0x45535001;  // "ESP\1"

namespace {
class EspInputMessage : public InputMessageBase {
public:
    EspHead head;
    Buf body;
    PipelinedInfo pi;
};
}  // namespace

ParseResult ParseEspMessage(Buf* source, Socket* socket, bool, const void*) {
    if (socket->user() != get_client_side_messenger()) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    PipelinedInfo pi;
    if (!socket->PeekPipelinedInfo(&pi) || pi.tag != kEspTag) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    EspHead head;
    if (source->copy_to(&head, sizeof(head)) < sizeof(head)) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    if (head.body_len < 0 || (uint64_t)head.body_len > FLAGS_max_body_size) {
        return MakeParseError(PARSE_ERROR_TOO_BIG_DATA);
    }
    if (source->size() < sizeof(head) + (size_t)head.body_len) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    EspInputMessage* m = new EspInputMessage;
    if (!socket->PopPipelinedInfo(&m->pi)) {
        delete m;
        return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
    }
    m->head = head;
    source->pop_front(sizeof(head));
    source->cutn(&m->body, (size_t)head.body_len);
    return MakeMessage(m);
}

void SerializeEspRequest(Buf* buf, Controller* cntl, const pb::Message* request) {
    const EspMessage* req = dynamic_cast<const EspMessage*>(request);
    if (!req) return cntl->SetFailed(EREQUEST, "request of esp must be EspMessage");
    EspHead h = req->head;
    h.body_len = (int32_t)req->body.size();
    buf->append(&h, sizeof(h));
    buf->append(req->body);
}

void PackEspRequest(Buf* packet, uint64_t, const pb::MethodDescriptor*, Controller* cntl, const Buf& request_buf,
                    const Authenticator* auth) {
    if (auth) {  // first request of the connection carries the ESP preamble
        std::string cred;
        auth->GenerateCredential(&cred);
        packet->append(cred);
    }
    packet->append(request_buf);
    cntl->_pipelined_count = 1;
    cntl->_pipelined_tag = kEspTag;
}

void ProcessEspResponse(InputMessageBase* base) {
    std::unique_ptr<EspInputMessage> m(static_cast<EspInputMessage*>(base));
    CompleteClientCallWith(m->pi.id_wait, m->socket(), [&](Controller* cntl) -> int {
        EspMessage* res = dynamic_cast<EspMessage*>(cntl->_response);
        if (!res) {
            if (!cntl->_response) return 0;
            cntl->SetFailed(ERESPONSE, "response of esp must be EspMessage");
            return ERESPONSE;
        }
        res->head = m->head;
        res->body.swap(m->body);
        if (res->head.msg != 0) {
            cntl->SetFailed(ENOENT, "esp response head msg=%u", res->head.msg);
            return ENOENT;
        }
        return 0;
    });
}

void RegisterEspProtocol() {
    Protocol p;
    p.parse = ParseEspMessage;
    p.serialize_request = SerializeEspRequest;
    p.pack_request = PackEspRequest;
    p.process_response = ProcessEspResponse;
    p.supported_connection_type = CONNECTION_TYPE_SINGLE | CONNECTION_TYPE_POOLED | CONNECTION_TYPE_SHORT;
    p.name = "esp";
    RegisterProtocol(PROTOCOL_ESP, p);
}

}  // namespace policy
}  // namespace mrpc
