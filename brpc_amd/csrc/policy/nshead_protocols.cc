// The nshead protocol family (roles of the reference's
// src/brpc/policy/nshead_protocol.cpp, nova_pbrpc_protocol.cpp,
// public_pbrpc_protocol.cpp, nshead_mcpack_protocol.cpp and
// ubrpc2pb_protocol.cpp). All share the 36-byte nshead framing:
//   server side: one "nshead" protocol hands requests to
//                ServerOptions.nshead_service (raw, or a pb adaptor);
//   client side: nshead (raw NsheadMessage), nova_pbrpc, public_pbrpc,
//                nshead_mcpack, ubrpc_compack, ubrpc_mcpack2.
// nshead has no correlation id. Where the reference can only use one call
// per connection (Socket::correlation_id), here every client write records
// its call id in the socket's pipelined-info queue tagged with the
// protocol, so single connections can carry pipelined nshead calls and
// the parser of each client protocol only claims responses to its own
// requests.
#include <ctime>
#include <unistd.h>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "mcpack/mcpack.h"
#include "mrpc/proto/legacy_meta.pb.h"
#include "net/input_messenger.h"
#include "policy/pbrpc_common.h"
#include "policy/policies.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/nshead.h"
#include "rpc/protocol.h"
#include "rpc/server.h"
#include "rpc/span.h"

DECLARE_uint64(max_body_size);

namespace mrpc {
namespace policy {

namespace {

enum NsheadClientTag : uint32_t {
    TAG_NSHEAD = 0x4e530001,
    TAG_NOVA,
    TAG_PUBLIC_PBRPC,
    TAG_NSHEAD_MCPACK,
    TAG_UBRPC_COMPACK,
    TAG_UBRPC_MCPACK2,
};

class NsheadClientMessage : public InputMessageBase {
public:
    nshead_t head;
    Buf body;
    PipelinedInfo pi;
};

bool is_client_socket(Socket* s) { return s->user() == get_client_side_messenger(); }

// Server connection state: the response sequencer of the connection.
class NsheadServerContext : public ParsingContext {
public:
    static const int kTag = 0x4e534856;  // "NSHV"
    int protocol_tag() const override { return kTag; }
    std::shared_ptr<OrderedResponseWriter> seq = std::make_shared<OrderedResponseWriter>();
};

class NsheadServerMessage : public InputMessageBase {
public:
    Buf meta;  // the 36-byte head
    Buf payload;
    uint64_t seq = 0;
    std::shared_ptr<OrderedResponseWriter> sequencer;
};

// 0: complete frame available, else the parse error.
ParseError CheckNshead(Buf* source, Socket* socket, nshead_t* head) {
    const size_t n = source->copy_to(head, sizeof(nshead_t));
    if (n < sizeof(nshead_t)) return PARSE_ERROR_NOT_ENOUGH_DATA;
    if (head->magic_num != NSHEAD_MAGICNUM) return PARSE_ERROR_TRY_OTHERS;
    if (head->body_len > FLAGS_max_body_size) {
        LOG(ERROR) << "nshead body_len=" << head->body_len << " from " << socket->remote_side() << " is too large";
        return PARSE_ERROR_TOO_BIG_DATA;
    }
    if (source->size() < sizeof(nshead_t) + head->body_len) return PARSE_ERROR_NOT_ENOUGH_DATA;
    return PARSE_OK;
}

template <uint32_t TAG>
ParseResult ParseNsheadClient(Buf* source, Socket* socket) {
    PipelinedInfo pi;
    if (!socket->PeekPipelinedInfo(&pi) || pi.tag != TAG) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    nshead_t head;
    const ParseError e = CheckNshead(source, socket, &head);
    if (e != PARSE_OK) return MakeParseError(e);
    NsheadClientMessage* m = new NsheadClientMessage;
    if (!socket->PopPipelinedInfo(&m->pi)) {
        delete m;
        return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
    }
    m->head = head;
    source->pop_front(sizeof(nshead_t));
    source->cutn(&m->body, head.body_len);
    return MakeMessage(m);
}

template <uint32_t TAG>
ParseResult ParseClientOnly(Buf* source, Socket* socket, bool, const void*) {
    if (!is_client_socket(socket)) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    return ParseNsheadClient<TAG>(source, socket);
}

// Requests to a server, or responses of raw nshead calls.
ParseResult ParseNsheadMessage(Buf* source, Socket* socket, bool read_eof, const void* arg) {
    if (is_client_socket(socket)) return ParseNsheadClient<TAG_NSHEAD>(source, socket);
    const Server* server = static_cast<const Server*>(arg);
    if (!server || !server->options().nshead_service) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    ParsingContext* pc = socket->parsing_context();
    if (pc && pc->protocol_tag() != NsheadServerContext::kTag) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    nshead_t head;
    const ParseError e = CheckNshead(source, socket, &head);
    if (e != PARSE_OK) return MakeParseError(e);
    NsheadServerContext* ctx = static_cast<NsheadServerContext*>(pc);
    if (!ctx) {
        ctx = new NsheadServerContext;
        if (!socket->InstallParsingContext(ctx)) {
            delete ctx;
            return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        }
    }
    NsheadServerMessage* msg = new NsheadServerMessage;
    msg->seq = ctx->seq->NextSeq();
    msg->sequencer = ctx->seq;
    source->cutn(&msg->meta, sizeof(nshead_t));
    source->cutn(&msg->payload, head.body_len);
    return MakeMessage(msg);
}

void ProcessNsheadRequest(InputMessageBase* base) {
    NsheadServerMessage* msg = static_cast<NsheadServerMessage*>(base);
    Socket* socket = msg->socket();
    Server* server = const_cast<Server*>(static_cast<const Server*>(msg->arg()));
    NsheadService* svc = server->options().nshead_service;
    if (!svc) {
        socket->SetFailed(EREQUEST, "nshead request but ServerOptions.nshead_service is unset");
        msg->Destroy();
        return;
    }
    NsheadClosure* done = new NsheadClosure;
    done->_server = server;
    done->_received_us = msg->received_us();
    done->_seq = msg->seq;
    done->_sequencer = msg->sequencer;
    Controller* cntl = done->_cntl.get();
    cntl->_server = server;
    cntl->_server_socket_id = socket->id();
    cntl->_remote_side = socket->remote_side();
    cntl->_local_side = socket->local_side();
    cntl->_received_us = msg->received_us();
    cntl->_begin_us = msg->received_us();
    cntl->_protocol_type = PROTOCOL_NSHEAD;
    msg->meta.copy_to(&done->_request.head, sizeof(nshead_t));
    done->_request.body.swap(msg->payload);
    msg->Destroy();
    cntl->set_log_id(done->_request.head.log_id);
    if (IsRpczEnabled()) {
        cntl->_span = Span::CreateServerSpan(0, 0, 0, "nshead", realtime_us());
        if (cntl->_span) {
            cntl->_span->protocol = PROTOCOL_NSHEAD;
            cntl->_span->remote_side = socket->remote_side();
            cntl->_span->request_size = (int64_t)(sizeof(nshead_t) + done->_request.body.size());
            cntl->_span->log_id = done->_request.head.log_id;
        }
    }
    svc->status()->OnRequested(nullptr, nullptr);
    if (!server->IsRunning()) {
        cntl->SetFailed(ELOGOFF, "Server is stopping");
    } else if (!server->AddConcurrency(cntl)) {
        cntl->SetFailed(ELIMIT, "Reached server's max_concurrency=%d", server->max_concurrency());
    } else {
        done->_added_concurrency = true;
    }
    if (cntl->Failed() && !dynamic_cast<NsheadPbServiceAdaptor*>(svc)) {
        cntl->CloseConnection("nshead request rejected");
        done->Run();
        return;
    }
    if (cntl->_span) cntl->_span->start_callback_real_us = realtime_us();
    svc->ProcessNsheadRequest(*server, cntl, done->_request, &done->_response, done);
}

// ---- client helpers

// nshead + body, pipelined under TAG.
void PackPipelined(Buf* packet, Controller* cntl, const nshead_t& head, const Buf& body, uint32_t tag) {
    PackNsheadFrame(packet, head, body);
    cntl->_pipelined_count = 1;
    cntl->_pipelined_tag = tag;
}

nshead_t DefaultHead(Controller* cntl) {
    nshead_t h;
    memset(&h, 0, sizeof(h));
    h.log_id = (uint32_t)cntl->log_id();
    return h;
}

// ---- raw nshead client: request/response are NsheadMessage

void SerializeNsheadRequest(Buf* buf, Controller* cntl, const pb::Message* request) {
    const NsheadMessage* req = dynamic_cast<const NsheadMessage*>(request);
    if (!req) {
        cntl->SetFailed(EREQUEST, "request of nshead must be NsheadMessage");
        return;
    }
    nshead_t h = req->head;
    if (!h.log_id && cntl->log_id()) h.log_id = (uint32_t)cntl->log_id();
    PackNsheadFrame(buf, h, req->body);
}

void PackNsheadRequest(Buf* packet, uint64_t, const pb::MethodDescriptor*, Controller* cntl, const Buf& request_buf,
                       const Authenticator*) {
    packet->append(request_buf);
    cntl->_pipelined_count = 1;
    cntl->_pipelined_tag = TAG_NSHEAD;
}

void ProcessNsheadResponse(InputMessageBase* base) {
    std::unique_ptr<NsheadClientMessage> m(static_cast<NsheadClientMessage*>(base));
    CompleteClientCallWith(m->pi.id_wait, m->socket(), [&](Controller* cntl) -> int {
        NsheadMessage* res = dynamic_cast<NsheadMessage*>(cntl->_response);
        if (!res) {
            if (!cntl->_response) return 0;
            cntl->SetFailed(ERESPONSE, "response of nshead must be NsheadMessage");
            return ERESPONSE;
        }
        res->head = m->head;
        res->body.swap(m->body);
        return 0;
    });
}

// ---- nova_pbrpc client

void SerializeNovaRequest(Buf* buf, Controller* cntl, const pb::Message* request) {
    const CompressType ct = cntl->request_compress_type();
    if (ct != COMPRESS_TYPE_NONE && ct != COMPRESS_TYPE_SNAPPY) {
        cntl->SetFailed(EREQUEST, "nova_pbrpc only supports snappy compression");
        return;
    }
    if (!request || !SerializeAsCompressedData(*request, buf, ct)) cntl->SetFailed(EREQUEST, "Fail to serialize request");
}

void PackNovaRequest(Buf* packet, uint64_t, const pb::MethodDescriptor* method, Controller* cntl,
                     const Buf& request_buf, const Authenticator*) {
    if (!method) return cntl->SetFailed(EREQUEST, "nova_pbrpc needs a method");
    nshead_t h = DefaultHead(cntl);
    h.reserved = (uint32_t)method->index;
    if (cntl->request_compress_type() == COMPRESS_TYPE_SNAPPY) h.version = NOVA_SNAPPY_COMPRESS_FLAG;
    PackPipelined(packet, cntl, h, request_buf, TAG_NOVA);
}

void ProcessNovaResponse(InputMessageBase* base) {
    std::unique_ptr<NsheadClientMessage> m(static_cast<NsheadClientMessage*>(base));
    const CompressType ct = (m->head.version & NOVA_SNAPPY_COMPRESS_FLAG) ? COMPRESS_TYPE_SNAPPY : COMPRESS_TYPE_NONE;
    CompletePbClientCall(m->pi.id_wait, 0, std::string(), &m->body, nullptr, ct, m->socket());
}

// ---- public_pbrpc client

const uint32_t kPublicSnappy = 1;

void SerializePublicPbrpcRequest(Buf* buf, Controller* cntl, const pb::Message* request) {
    const CompressType ct = cntl->request_compress_type();
    if (ct != COMPRESS_TYPE_NONE && ct != COMPRESS_TYPE_SNAPPY) {
        cntl->SetFailed(EREQUEST, "public_pbrpc only supports snappy compression");
        return;
    }
    if (!request || !SerializeAsCompressedData(*request, buf, ct)) cntl->SetFailed(EREQUEST, "Fail to serialize request");
}

void PackPublicPbrpcRequest(Buf* packet, uint64_t correlation_id, const pb::MethodDescriptor* method,
                            Controller* cntl, const Buf& request_buf, const Authenticator*) {
    if (!method) return cntl->SetFailed(EREQUEST, "public_pbrpc needs a method");
    PublicPbrpcRequest whole;
    RequestHead* head = whole.mutable_requestHead();
    char host[256] = {0};
    gethostname(host, sizeof(host) - 1);
    head->set_from_host(host);
    head->set_content_type(1);
    head->set_connection(cntl->connection_type() == CONNECTION_TYPE_POOLED);
    head->set_charset("utf-8");
    head->set_accept_charset("utf-8");
    char ts[32];
    const time_t now = time(nullptr);
    struct tm tmv;
    localtime_r(&now, &tmv);
    strftime(ts, sizeof(ts), "%Y%m%d%H%M%S", &tmv);
    head->set_create_time(ts);
    if (cntl->log_id()) head->set_log_id(cntl->log_id());
    if (cntl->request_compress_type() == COMPRESS_TYPE_SNAPPY) head->set_compress_type(kPublicSnappy);
    RequestBody* body = whole.add_requestBody();
    body->set_version("pbrpc=1.0");
    body->set_charset("utf-8");
    body->set_service(method->service->name);
    body->set_method_id((uint32_t)method->index);
    body->set_id(correlation_id);
    body->set_serialized_request(request_buf.to_string());
    Buf b;
    whole.SerializeToBuf(&b);
    nshead_t h = DefaultHead(cntl);
    h.version = 1000;
    strncpy(h.provider, "__pbrpc__", sizeof(h.provider) - 1);
    PackPipelined(packet, cntl, h, b, TAG_PUBLIC_PBRPC);
}

void ProcessPublicPbrpcResponse(InputMessageBase* base) {
    std::unique_ptr<NsheadClientMessage> m(static_cast<NsheadClientMessage*>(base));
    PublicPbrpcResponse whole;
    int err = 0;
    std::string text;
    Buf body;
    CompressType ct = COMPRESS_TYPE_NONE;
    if (!ParsePbFromBuf(&whole, m->body) || whole.responseBody_size() == 0) {
        err = ERESPONSE;
        text = "Fail to parse PublicPbrpcResponse";
    } else if (whole.responseHead().code() != 0) {
        err = whole.responseHead().code();
        text = whole.responseHead().text();
    } else {
        body.append(whole.responseBody(0).serialized_response());
        if (whole.responseHead().compress_type() == kPublicSnappy) ct = COMPRESS_TYPE_SNAPPY;
    }
    CompletePbClientCall(m->pi.id_wait, err, text, &body, nullptr, ct, m->socket());
}

// ---- nshead_mcpack client: body is the mcpack (v2) object of the request

void SerializeNsheadMcpackRequest(Buf* buf, Controller* cntl, const pb::Message* request) {
    if (!request || !mcpack::SerializeToBuf(*request, mcpack::FORMAT_MCPACK_V2, buf)) {
        cntl->SetFailed(EREQUEST, "Fail to serialize request as mcpack");
    }
}

void PackNsheadMcpackRequest(Buf* packet, uint64_t, const pb::MethodDescriptor*, Controller* cntl,
                             const Buf& request_buf, const Authenticator*) {
    PackPipelined(packet, cntl, DefaultHead(cntl), request_buf, TAG_NSHEAD_MCPACK);
}

void ProcessNsheadMcpackResponse(InputMessageBase* base) {
    std::unique_ptr<NsheadClientMessage> m(static_cast<NsheadClientMessage*>(base));
    CompleteClientCallWith(m->pi.id_wait, m->socket(), [&](Controller* cntl) -> int {
        if (cntl->_response && !mcpack::ParseFromBuf(m->body, cntl->_response)) {
            cntl->SetFailed(ERESPONSE, "Fail to parse mcpack response");
            return ERESPONSE;
        }
        return 0;
    });
}

// ---- ubrpc (compack / mcpack2) client
//   request:  {header:{connection}, content:[{service_name, id, method, params:{<req_name>:{...}}}]}
//   response: {content:[{id, result?, result_params:{<res_name>:{...}}} | {id, error:{code,message}}]}

void SerializeUbrpcRequest(Buf* buf, Controller* cntl, const pb::Message* request, mcpack::Format fmt) {
    const pb::MethodDescriptor* method = cntl->_method;
    if (!request || !method) {
        cntl->SetFailed(EREQUEST, "ubrpc needs a method and a request");
        return;
    }
    std::string out;
    mcpack::Serializer sr(&out);
    sr.begin_object();
    sr.begin_object("header");
    sr.add_bool("connection", cntl->connection_type() == CONNECTION_TYPE_POOLED);
    sr.end_object();
    sr.begin_array("content", mcpack::FIELD_OBJECT, fmt);
    sr.begin_object();
    sr.add_string("service_name", method->service->name);
    // The correlation id is not known before pack: a placeholder of fixed
    // width is patched by PackUbrpcRequest.
    sr.add_int64("id", 0);
    sr.add_string("method", method->name);
    sr.begin_object("params");
    const char* rn = cntl->idl_names().request_name;
    if (rn && *rn) sr.begin_object(rn);
    mcpack::SerializeFields(*request, fmt, &sr);
    if (rn && *rn) sr.end_object();
    sr.end_object();
    sr.end_object();
    sr.end_array();
    sr.end_object();
    if (!sr.good()) {
        cntl->SetFailed(EREQUEST, "Fail to serialize %s", request->GetTypeName().c_str());
        return;
    }
    buf->append(out);
}

// Offset of the int64 value of content[0].id inside the serialized request.
size_t FindIdOffset(const std::string& s) {
    static const char kName[] = "id";  // fixed head: type, name_size=3, "id\0", 8 bytes
    for (size_t i = 0; i + 2 + sizeof(kName) + 8 <= s.size(); ++i) {
        if ((uint8_t)s[i] == mcpack::FIELD_INT64 && (uint8_t)s[i + 1] == sizeof(kName) &&
            memcmp(&s[i + 2], kName, sizeof(kName)) == 0) {
            return i + 2 + sizeof(kName);
        }
    }
    return std::string::npos;
}

template <uint32_t TAG>
void PackUbrpcRequest(Buf* packet, uint64_t correlation_id, const pb::MethodDescriptor*, Controller* cntl,
                      const Buf& request_buf, const Authenticator*) {
    std::string s = request_buf.to_string();
    const size_t off = FindIdOffset(s);
    if (off == std::string::npos) return cntl->SetFailed(EREQUEST, "malformed ubrpc request");
    const int64_t id = (int64_t)correlation_id;
    memcpy(&s[off], &id, 8);
    PackPipelined(packet, cntl, DefaultHead(cntl), Buf(s), TAG);
}

void ProcessUbrpcResponse(InputMessageBase* base) {
    std::unique_ptr<NsheadClientMessage> m(static_cast<NsheadClientMessage*>(base));
    const std::string raw = m->body.to_string();
    CompleteClientCallWith(m->pi.id_wait, m->socket(), [&](Controller* cntl) -> int {
        std::string name;
        mcpack::Value top;
        std::vector<mcpack::Item> items, content, fields;
        if (!mcpack::DecodeField(raw.data(), raw.size(), &name, &top) || !mcpack::ListItems(top, &items)) {
            cntl->SetFailed(ERESPONSE, "Fail to parse ubrpc response");
            return ERESPONSE;
        }
        const mcpack::Value* c0 = nullptr;
        for (auto& it : items) {
            if (it.name == "content" && mcpack::ListItems(it.value, &content) && !content.empty()) c0 = &content[0].value;
        }
        if (!c0 || !mcpack::ListItems(*c0, &fields)) {
            cntl->SetFailed(ERESPONSE, "ubrpc response has no content[0]");
            return ERESPONSE;
        }
        const mcpack::Value* params = nullptr;
        for (auto& f : fields) {
            if (f.name == "error") {
                std::vector<mcpack::Item> err;
                int64_t code = 0;
                std::string msg;
                if (mcpack::ListItems(f.value, &err)) {
                    for (auto& e : err) {
                        if (e.name == "code") e.value.to_int64(&code);
                        if (e.name == "message") e.value.to_string(&msg);
                    }
                }
                cntl->SetFailed(code ? (int)code : ERESPONSE, "%s", msg.c_str());
                return cntl->ErrorCode();
            } else if (f.name == "result") {
                int64_t r;
                if (f.value.to_int64(&r)) cntl->set_idl_result(r);
            } else if (f.name == "result_params") {
                params = &f.value;
            }
        }
        if (!cntl->_response) return 0;
        if (!params) {
            cntl->SetFailed(ERESPONSE, "ubrpc response has no result_params");
            return ERESPONSE;
        }
        mcpack::Value obj = *params;
        const char* rn = cntl->idl_names().response_name;
        if (rn && *rn) {
            std::vector<mcpack::Item> sub;
            bool found = false;
            if (mcpack::ListItems(*params, &sub)) {
                for (auto& s : sub) {
                    if (s.name == rn) {
                        obj = s.value;
                        found = true;
                    }
                }
            }
            if (!found) {
                cntl->SetFailed(ERESPONSE, "Fail to find %s in result_params", rn);
                return ERESPONSE;
            }
        }
        cntl->_response->Clear();
        if (!mcpack::ParseFromObject(obj, cntl->_response) || !cntl->_response->IsInitialized()) {
            cntl->SetFailed(ERESPONSE, "Fail to parse %s from ubrpc response", cntl->_response->GetTypeName().c_str());
            return ERESPONSE;
        }
        return 0;
    });
}

void SerializeUbrpcCompack(Buf* b, Controller* c, const pb::Message* r) { SerializeUbrpcRequest(b, c, r, mcpack::FORMAT_COMPACK); }
void SerializeUbrpcMcpack2(Buf* b, Controller* c, const pb::Message* r) { SerializeUbrpcRequest(b, c, r, mcpack::FORMAT_MCPACK_V2); }

Protocol ClientProtocol(const char* name) {
    Protocol p;
    p.supported_connection_type = CONNECTION_TYPE_SINGLE | CONNECTION_TYPE_POOLED | CONNECTION_TYPE_SHORT;
    p.name = name;
    return p;
}

}  // namespace

void RegisterNsheadProtocols() {
    Protocol ns = ClientProtocol("nshead");
    ns.parse = ParseNsheadMessage;
    ns.serialize_request = SerializeNsheadRequest;
    ns.pack_request = PackNsheadRequest;
    ns.process_request = ProcessNsheadRequest;
    ns.process_response = ProcessNsheadResponse;
    RegisterProtocol(PROTOCOL_NSHEAD, ns);

    Protocol nova = ClientProtocol("nova_pbrpc");
    nova.parse = ParseClientOnly<TAG_NOVA>;
    nova.serialize_request = SerializeNovaRequest;
    nova.pack_request = PackNovaRequest;
    nova.process_response = ProcessNovaResponse;
    RegisterProtocol(PROTOCOL_NOVA_PBRPC, nova);

    Protocol pub = ClientProtocol("public_pbrpc");
    pub.parse = ParseClientOnly<TAG_PUBLIC_PBRPC>;
    pub.serialize_request = SerializePublicPbrpcRequest;
    pub.pack_request = PackPublicPbrpcRequest;
    pub.process_response = ProcessPublicPbrpcResponse;
    RegisterProtocol(PROTOCOL_PUBLIC_PBRPC, pub);

    Protocol mc = ClientProtocol("nshead_mcpack");
    mc.parse = ParseClientOnly<TAG_NSHEAD_MCPACK>;
    mc.serialize_request = SerializeNsheadMcpackRequest;
    mc.pack_request = PackNsheadMcpackRequest;
    mc.process_response = ProcessNsheadMcpackResponse;
    RegisterProtocol(PROTOCOL_NSHEAD_MCPACK, mc);

    Protocol ubc = ClientProtocol("ubrpc_compack");
    ubc.parse = ParseClientOnly<TAG_UBRPC_COMPACK>;
    ubc.serialize_request = SerializeUbrpcCompack;
    ubc.pack_request = PackUbrpcRequest<TAG_UBRPC_COMPACK>;
    ubc.process_response = ProcessUbrpcResponse;
    RegisterProtocol(PROTOCOL_UBRPC_COMPACK, ubc);

    Protocol ubm = ClientProtocol("ubrpc_mcpack2");
    ubm.parse = ParseClientOnly<TAG_UBRPC_MCPACK2>;
    ubm.serialize_request = SerializeUbrpcMcpack2;
    ubm.pack_request = PackUbrpcRequest<TAG_UBRPC_MCPACK2>;
    ubm.process_response = ProcessUbrpcResponse;
    RegisterProtocol(PROTOCOL_UBRPC_MCPACK2, ubm);
}

}  // namespace policy
}  // namespace mrpc
