// Framed thrift (TBinaryProtocol) client and server (role of the
// reference's src/brpc/policy/thrift_protocol.cpp). The server hands calls
// to ServerOptions.thrift_service; responses of one connection leave in
// request order (OrderedResponseWriter) so the client can pipeline calls
// on a single connection through the socket's pipelined-info queue, and
// additionally checks that the reply's seqid matches its call.
#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "net/input_messenger.h"
#include "policy/pbrpc_common.h"
#include "policy/policies.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/method_status.h"
#include "rpc/ordered_response.h"
#include "rpc/protocol.h"
#include "rpc/server.h"
#include "thrift/thrift.h"

DECLARE_uint64(max_body_size);

namespace mrpc {
namespace policy {

namespace {

class ThriftServerContext : public ParsingContext {
public:
    static const int kTag = 0x54485246;  // "THRF"
    int protocol_tag() const override { return kTag; }
    std::shared_ptr<OrderedResponseWriter> seq = std::make_shared<OrderedResponseWriter>();
};

class ThriftInputMessage : public InputMessageBase {
public:
    std::string frame;  // the message, without the 4-byte length
    uint64_t seq = 0;
    std::shared_ptr<OrderedResponseWriter> writer;
    PipelinedInfo pi;    // client side
};

bool is_client_socket(Socket* s) { return s->user() == get_client_side_messenger(); }

void PackFrame(Buf* out, const std::string& msg) {
    char len[4];
    const uint32_t n = (uint32_t)msg.size();
    len[0] = (char)(n >> 24);
    len[1] = (char)(n >> 16);
    len[2] = (char)(n >> 8);
    len[3] = (char)n;
    out->append(len, 4);
    out->append(msg);
}

struct ThriftCall {
    Controller cntl;
    ThriftFramedMessage req, res;
    Server* server = nullptr;
    uint64_t seq = 0;
    std::shared_ptr<OrderedResponseWriter> writer;
    int64_t received_us = 0;
    bool added_concurrency = false;
    bool oneway = false;
};

void SendThriftResponse(ThriftCall* c) {
    std::unique_ptr<ThriftCall> guard(c);
    ThriftService* svc = c->server->options().thrift_service;
    ConcurrencyRemover remover(svc ? svc->status() : nullptr, &c->cntl, c->received_us,
                               c->added_concurrency ? c->server : nullptr);
    SocketUniquePtr sock;
    if (Socket::Address(c->cntl._server_socket_id, &sock) != 0) return;
    if (c->cntl.IsCloseConnection()) {
        sock->SetFailed(ECLOSE, "close connection by thrift service");
        return;
    }
    Buf packet;
    if (!c->oneway) {
        thrift::MessageHeader h;
        h.name = c->req.method_name;
        h.seqid = c->req.seq_id;
        std::string msg;
        if (c->cntl.Failed()) {
            h.type = thrift::T_EXCEPTION;
            thrift::Value ex = thrift::Value::Struct();
            ex.field(1) = thrift::Value::String(c->cntl.ErrorText());
            ex.field(2) = thrift::Value::I32(c->cntl.ErrorCode() == ENOMETHOD ? thrift::TAPP_UNKNOWN_METHOD
                                                                              : thrift::TAPP_INTERNAL_ERROR);
            thrift::WriteMessage(&msg, h, ex);
        } else {
            h.type = thrift::T_REPLY;
            thrift::WriteMessage(&msg, h, c->res.body);
        }
        PackFrame(&packet, msg);
    }
    c->writer->Deliver(c->seq, &packet, sock.get());
}

}  // namespace

ParseResult ParseThriftFramedMessage(Buf* source, Socket* socket, bool, const void* arg) {
    const bool client = is_client_socket(socket);
    PipelinedInfo pi;
    ThriftServerContext* ctx = nullptr;
    if (client) {
        if (!socket->PeekPipelinedInfo(&pi) || pi.protocol != PROTOCOL_THRIFT) {
            return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        }
    } else {
        const Server* server = static_cast<const Server*>(arg);
        if (!server || !server->options().thrift_service) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        ParsingContext* pc = socket->parsing_context();
        if (pc && pc->protocol_tag() != ThriftServerContext::kTag) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        ctx = static_cast<ThriftServerContext*>(pc);
    }
    char h[6];
    const size_t n = source->copy_to(h, sizeof(h));
    if (n < sizeof(h)) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    // strict binary protocol version 0x8001 right after the frame length
    if ((uint8_t)h[4] != 0x80 || (uint8_t)h[5] != 0x01) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    const uint32_t len = ((uint32_t)(uint8_t)h[0] << 24) | ((uint32_t)(uint8_t)h[1] << 16) |
                         ((uint32_t)(uint8_t)h[2] << 8) | (uint32_t)(uint8_t)h[3];
    if (len > FLAGS_max_body_size) return MakeParseError(PARSE_ERROR_TOO_BIG_DATA);
    if (source->size() < 4 + (size_t)len) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    ThriftInputMessage* m = new ThriftInputMessage;
    if (client) {
        if (!socket->PopPipelinedInfo(&m->pi)) {
            delete m;
            return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
        }
    } else {
        if (!ctx) {
            ctx = new ThriftServerContext;
            if (!socket->InstallParsingContext(ctx)) {
                delete ctx;
                delete m;
                return MakeParseError(PARSE_ERROR_TRY_OTHERS);
            }
        }
        m->seq = ctx->seq->NextSeq();
        m->writer = ctx->seq;
    }
    source->pop_front(4);
    source->cutn(&m->frame, len);
    return MakeMessage(m);
}

void ProcessThriftFramedRequest(InputMessageBase* base) {
    std::unique_ptr<ThriftInputMessage> m(static_cast<ThriftInputMessage*>(base));
    Socket* socket = m->socket();
    Server* server = const_cast<Server*>(static_cast<const Server*>(m->arg()));
    ThriftService* svc = server->options().thrift_service;
    ThriftCall* c = new ThriftCall;
    c->server = server;
    c->seq = m->seq;
    c->writer = m->writer;
    c->received_us = m->received_us();
    Controller* cntl = &c->cntl;
    cntl->_server = server;
    cntl->_server_socket_id = socket->id();
    cntl->_remote_side = socket->remote_side();
    cntl->_local_side = socket->local_side();
    cntl->_received_us = m->received_us();
    cntl->_begin_us = m->received_us();
    cntl->_protocol_type = PROTOCOL_THRIFT;
    thrift::MessageHeader h;
    if (!thrift::ReadMessage(m->frame.data(), m->frame.size(), &h, &c->req.body)) {
        // Nothing sensible to answer: drop the connection.
        socket->SetFailed(EREQUEST, "malformed thrift message");
        c->writer.reset();
        delete c;
        return;
    }
    m.reset();
    c->req.method_name = h.name;
    c->req.seq_id = h.seqid;
    c->res.method_name = h.name;
    c->res.seq_id = h.seqid;
    c->oneway = h.type == thrift::T_ONEWAY;
    if (svc) svc->status()->OnRequested(nullptr, cntl);
    if (h.type != thrift::T_CALL && h.type != thrift::T_ONEWAY) {
        cntl->SetFailed(EREQUEST, "unexpected thrift message type %d", (int)h.type);
    } else if (!server->IsRunning()) {
        cntl->SetFailed(ELOGOFF, "Server is stopping");
    } else if (!server->AddConcurrency(cntl)) {
        cntl->SetFailed(ELIMIT, "Reached server's max_concurrency=%d", server->max_concurrency());
    } else {
        c->added_concurrency = true;
    }
    if (cntl->Failed() || !svc) {
        SendThriftResponse(c);
        return;
    }
    svc->ProcessThriftFramedRequest(cntl, &c->req, &c->res, NewCallback([c] { SendThriftResponse(c); }));
}

void SerializeThriftRequest(Buf* buf, Controller* cntl, const pb::Message* request) {
    const ThriftFramedMessage* req = dynamic_cast<const ThriftFramedMessage*>(request);
    if (!req) return cntl->SetFailed(EREQUEST, "request of thrift must be ThriftFramedMessage");
    std::string name = req->method_name;
    if (name.empty() && cntl->_method) name = cntl->_method->name;
    if (name.empty()) return cntl->SetFailed(EREQUEST, "thrift request has no method_name");
    thrift::MessageHeader h;
    h.name = name;
    h.type = thrift::T_CALL;
    h.seqid = 0;  // patched in pack
    std::string msg;
    thrift::WriteMessage(&msg, h, req->body);
    buf->append(msg);
}

void PackThriftRequest(Buf* packet, uint64_t correlation_id, const pb::MethodDescriptor*, Controller* cntl,
                       const Buf& request_buf, const Authenticator*) {
    std::string msg = request_buf.to_string();
    // seqid follows version(4) + name length(4) + name
    const uint32_t nlen = ((uint32_t)(uint8_t)msg[4] << 24) | ((uint32_t)(uint8_t)msg[5] << 16) |
                          ((uint32_t)(uint8_t)msg[6] << 8) | (uint32_t)(uint8_t)msg[7];
    const size_t at = 8 + nlen;
    const uint32_t seqid = (uint32_t)correlation_id;
    msg[at] = (char)(seqid >> 24);
    msg[at + 1] = (char)(seqid >> 16);
    msg[at + 2] = (char)(seqid >> 8);
    msg[at + 3] = (char)seqid;
    PackFrame(packet, msg);
    cntl->_pipelined_count = 1;
    cntl->_pipelined_tag = seqid;
}

void ProcessThriftFramedResponse(InputMessageBase* base) {
    std::unique_ptr<ThriftInputMessage> m(static_cast<ThriftInputMessage*>(base));
    CompleteClientCallWith(m->pi.id_wait, m->socket(), [&](Controller* cntl) -> int {
        thrift::MessageHeader h;
        thrift::Value body;
        if (!thrift::ReadMessage(m->frame.data(), m->frame.size(), &h, &body)) {
            cntl->SetFailed(ERESPONSE, "malformed thrift reply");
            return ERESPONSE;
        }
        if ((uint32_t)h.seqid != m->pi.tag) {
            cntl->SetFailed(ERESPONSE, "thrift seqid mismatch: got %d", h.seqid);
            return ERESPONSE;
        }
        if (h.type == thrift::T_EXCEPTION) {
            const thrift::Value* msg = body.find(1);
            cntl->SetFailed(EINTERNAL, "thrift exception: %s", msg ? msg->as_string().c_str() : "");
            return EINTERNAL;
        }
        ThriftFramedMessage* res = dynamic_cast<ThriftFramedMessage*>(cntl->_response);
        if (res) {
            res->method_name = h.name;
            res->seq_id = h.seqid;
            res->body = std::move(body);
        }
        return 0;
    });
}

void RegisterThriftProtocol() {
    Protocol p;
    p.parse = ParseThriftFramedMessage;
    p.serialize_request = SerializeThriftRequest;
    p.pack_request = PackThriftRequest;
    p.process_request = ProcessThriftFramedRequest;
    p.process_response = ProcessThriftFramedResponse;
    p.supported_connection_type = CONNECTION_TYPE_SINGLE | CONNECTION_TYPE_POOLED | CONNECTION_TYPE_SHORT;
    p.name = "thrift";
    RegisterProtocol(PROTOCOL_THRIFT, p);
}

}  // namespace policy
}  // namespace mrpc
