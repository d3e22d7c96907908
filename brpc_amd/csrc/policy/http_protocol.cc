// HTTP/1.1 protocol: pb services over http+json (or http+proto), plain
// HTTP calls (method == nullptr: body in the attachments), builtin pages,
// RESTful mappings and progressive bodies. Role of the reference's
// src/brpc/policy/http_rpc_protocol.cpp (ParseHttpMessage :1083,
// SerializeHttpRequest :486, PackHttpRequest :661, ProcessHttpRequest
// :1254, ProcessHttpResponse :269, VerifyHttpRequest :1210).
//
// Client calls run one request per connection at a time (pooled or short
// connections), so in-order responses always map to the right call through
// the socket's pipelined-info queue.
#include <cerrno>
#include <cstring>
#include <memory>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"
#include "fiber/call_id.h"
#include "http/http_header.h"
#include "http/http_message.h"
#include "json/json2pb.h"
#include "policy/policies.h"
#include "rpc/authenticator.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/method_status.h"
#include "rpc/progressive.h"
#include "rpc/protocol.h"
#include "rpc/server.h"
#include "rpc/span.h"
#include "rpc/usercode_backup_pool.h"

DECLARE_uint64(max_body_size);
DEFINE_bool(http_verbose, false, "print http request/response heads to stderr");
DEFINE_string(http_header_of_user_ip, "", "header carrying the real client ip behind a proxy");

namespace mrpc {
namespace policy {

enum : uint32_t { kTagHead = 1, kTagProgressive = 2 };

static const char* kJson = "application/json";
static const char* kProto = "application/proto";

static bool is_proto_content(const std::string& ct) {
    return starts_with(ct, "application/proto") || starts_with(ct, "application/x-protobuf");
}

static bool has_fields(const pb::Message* m) { return m && m->GetDescriptor()->field_count() > 0; }

// ------------------------------------------------------------------ parse
static void OnHead(HttpParser* p, HttpMessage* m, void* arg) {
    if (!m->is_response) return;
    Socket* s = static_cast<Socket*>(arg);
    PipelinedInfo pi;
    if (!s->PopPipelinedInfo(&pi)) return;  // unsolicited response: dropped later
    m->pi = pi;
    if (pi.tag & kTagHead) p->set_no_body();
    if (pi.tag & kTagProgressive) p->set_progressive(std::make_shared<ProgressiveSink>());
}

ParseResult ParseHttpMessage(Buf* source, Socket* socket, bool read_eof, const void* arg) {
    ParsingContext* ctx = socket->parsing_context();
    HttpParser* p = nullptr;
    if (ctx) {
        if (ctx->protocol_tag() != HttpParser::kTag) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        p = static_cast<HttpParser*>(ctx);
    } else {
        if (source->empty()) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
        char head[8];
        const size_t n = source->copy_to(head, sizeof(head));
        const int r = HttpParser::LooksLikeHttp(head, n);
        if (r == 0) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        if (r < 0) return MakeParseError(read_eof ? PARSE_ERROR_TRY_OTHERS : PARSE_ERROR_NOT_ENOUGH_DATA);
        p = new HttpParser((int64_t)FLAGS_max_body_size);
        p->on_head = OnHead;
        p->on_head_arg = socket;
        socket->reset_parsing_context(p);
    }
    std::string err;
    const HttpParser::Result r = p->Consume(source, read_eof, &err);
    if (r == HttpParser::NEED_MORE) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    if (r == HttpParser::FAILED) {
        LOG_EVERY_SECOND(WARNING) << "Bad http message from " << socket->remote_side() << ": " << err;
        return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
    }
    HttpMessage* msg = p->release();
    if (!msg->is_response) {
        if (!p->order) p->order = std::make_shared<HttpResponseOrder>();
        msg->order = p->order;
        msg->order_seq = p->order->next_req++;
    }
    if (FLAGS_http_verbose) {
        fprintf(stderr, "[http %s] %s %s\n", msg->is_response ? "response" : "request",
                msg->is_response ? std::to_string(msg->header.status_code()).c_str()
                                 : HttpMethod2Str(msg->header.method()),
                msg->header.uri().path().c_str());
    }
    return MakeMessage(msg);
}

// ------------------------------------------------------------------ client
void SerializeHttpRequest(Buf* buf, Controller* cntl, const pb::Message* request) {
    HttpHeader& h = cntl->http_request();
    if (cntl->_method && has_fields(request)) {
        if (!request->IsInitialized()) {
            cntl->SetFailed(EREQUEST, "Missing required fields in request: %s",
                            request->InitializationErrorString().c_str());
            return;
        }
        if (is_proto_content(h.content_type())) {
            std::string bytes;
            if (!request->SerializeToString(&bytes)) {
                cntl->SetFailed(EREQUEST, "Fail to serialize %s", request->GetDescriptor()->full_name.c_str());
                return;
            }
            buf->append(bytes);
        } else {
            std::string json, err;
            json2pb::Pb2JsonOptions opt;
            if (!json2pb::ProtoMessageToJson(*request, &json, opt, &err)) {
                cntl->SetFailed(EREQUEST, "Fail to convert request to json: %s", err.c_str());
                return;
            }
            if (h.content_type().empty()) h.set_content_type(kJson);
            buf->append(json);
        }
        if (h.method() == HTTP_METHOD_GET) h.set_method(HTTP_METHOD_POST);
        if (!cntl->request_attachment().empty()) {
            cntl->SetFailed(EREQUEST, "request_attachment must be empty when the http request carries a pb body");
        }
        return;
    }
    // plain http: the attachment is the body
    buf->append(cntl->request_attachment());
}

void PackHttpRequest(Buf* packet, uint64_t correlation_id, const pb::MethodDescriptor* method, Controller* cntl,
                     const Buf& request_buf, const Authenticator* auth) {
    (void)correlation_id;
    HttpHeader& h = cntl->http_request();
    if (method && (h.uri().path().empty() || h.uri().path() == "/")) {
        h.uri().set_path("/" + method->service->full_name + "/" + method->name);
    }
    if (auth) {
        std::string cred;
        if (auth->GenerateCredential(&cred) != 0) {
            cntl->SetFailed(ERPCAUTH, "Fail to generate credential");
            return;
        }
        h.SetHeader("Authorization", cred);
    }
    if (cntl->log_id()) h.SetHeader("log-id", std::to_string(cntl->log_id()));
    if (cntl->trace_id()) {
        h.SetHeader("x-mrpc-trace-id", std::to_string(cntl->trace_id()));
        h.SetHeader("x-mrpc-span-id", std::to_string(cntl->span_id()));
    }
    std::string host = h.uri().host();
    if (host.empty()) host = cntl->remote_side().to_string();
    else if (h.uri().port() > 0) host += ":" + std::to_string(h.uri().port());
    SerializeHttpRequestHead(packet, h, host, (int64_t)request_buf.size(), false);
    packet->append(request_buf);
    cntl->_pipelined_count = 1;
    cntl->_pipelined_tag = (h.method() == HTTP_METHOD_HEAD ? kTagHead : 0) |
                           (cntl->is_response_read_progressively() ? kTagProgressive : 0);
}

void ProcessHttpResponse(InputMessageBase* msg_base) {
    std::unique_ptr<HttpMessage> msg(static_cast<HttpMessage*>(msg_base));
    const fiber::CallId cid = msg->pi.id_wait;
    if (cid == fiber::INVALID_CALL_ID) return;  // unsolicited
    Controller* cntl = nullptr;
    if (fiber::call_id_lock(cid, (void**)&cntl) != 0) {
        if (msg->progressive) msg->progressive->End(ECANCELED, "rpc already ended");
        return;
    }
    if (cid != cntl->current_id() && cid != cntl->_unfinished_call.id) {
        fiber::call_id_unlock(cid);
        return;
    }
    HttpHeader& rh = cntl->http_response();
    rh = msg->header;
    int saved_error = 0;
    const int status = msg->header.status_code();
    if (status < 200 || status >= 300) {
        std::string body = msg->body.to_string();
        if (body.size() > 512) body.resize(512);
        const std::string* ec = msg->header.GetHeader("x-mrpc-error-code");
        saved_error = ec ? atoi(ec->c_str()) : EHTTP;
        if (saved_error == 0) saved_error = EHTTP;
        cntl->SetFailed(saved_error, "[HTTP %d %s] %s", status, HttpReasonPhrase(status), body.c_str());
        cntl->response_attachment().swap(msg->body);
    } else if (msg->progressive) {
        cntl->_progressive_sink = msg->progressive;
    } else if (cntl->_response && has_fields(cntl->_response)) {
        const std::string& ct = msg->header.content_type();
        if (is_proto_content(ct)) {
            if (!ParsePbFromBuf(cntl->_response, msg->body)) {
                cntl->SetFailed(ERESPONSE, "Fail to parse proto body of %s",
                                cntl->_response->GetDescriptor()->full_name.c_str());
                saved_error = ERESPONSE;
            }
        } else {
            std::string err;
            json2pb::Json2PbOptions opt;
            if (!json2pb::JsonToProtoMessage(msg->body, cntl->_response, opt, &err)) {
                cntl->SetFailed(ERESPONSE, "Fail to parse json body: %s", err.c_str());
                saved_error = ERESPONSE;
            }
        }
    } else {
        cntl->response_attachment().swap(msg->body);
    }
    cntl->_local_side = msg->socket()->local_side();
    if (!msg->keep_alive) msg->socket()->SetFailed(ECLOSE, "server closed the http connection");
    msg.reset();
    cntl->OnVersionedRPCReturned(cid, saved_error);
}

// ------------------------------------------------------------------ server
// Writes `packet` once every earlier response of the connection was written
// (pipelined requests finish in any order; their responses may not).
static void WriteInOrder(HttpResponseOrder* order, uint64_t seq, Socket* sock, Buf* packet, bool shutdown_after) {
    auto write = [sock](Buf* b, bool shut) {
        WriteOptions wopt;
        wopt.ignore_eovercrowded = true;
        wopt.shutdown_write_after = shut;  // "Connection: close" / HTTP/1.0
        sock->Write(b, &wopt);
    };
    if (!order) {
        write(packet, shutdown_after);
        return;
    }
    std::lock_guard<std::mutex> g(order->mu);
    if (seq != order->next_resp) {
        order->ready.emplace(seq, std::make_pair(std::move(*packet), shutdown_after));
        return;
    }
    write(packet, shutdown_after);
    ++order->next_resp;
    for (auto it = order->ready.begin(); it != order->ready.end() && it->first == order->next_resp;
         it = order->ready.erase(it)) {
        write(&it->second.first, it->second.second);
        ++order->next_resp;
    }
}

static void SendHttpResponse(Controller* cntl, pb::Message* req, pb::Message* res, Server* server,
                             MethodStatus* ms, int64_t received_us, bool keep_alive, bool http10,
                             std::shared_ptr<HttpResponseOrder> order, uint64_t order_seq) {
    std::unique_ptr<Controller> cntl_guard(cntl);
    std::unique_ptr<pb::Message> req_guard(req);
    std::unique_ptr<pb::Message> res_guard(res);
    ConcurrencyRemover remover(ms, cntl, received_us, server);
    SocketUniquePtr sock;
    if (Socket::Address(cntl->_server_socket_id, &sock) != 0) {
        if (cntl->_progressive_attachment) cntl->_progressive_attachment->MarkRPCAsDone(true);
        return;
    }
    // a progressive body continues after this response: the connection
    // cannot carry another response in order, so later pipelined requests
    // of it are answered after the head (HTTP/1.x clients do not pipeline
    // behind a streamed response in practice)
    HttpHeader& rh = cntl->http_response();
    rh.set_version(1, http10 ? 0 : 1);
    Buf body;
    bool chunked = false;
    if (cntl->Failed()) {
        rh.set_status_code(ErrorCodeToStatusCode(cntl->ErrorCode()));
        rh.SetHeader("x-mrpc-error-code", std::to_string(cntl->ErrorCode()));
        rh.set_content_type("text/plain");
        body.append(cntl->ErrorText());
        body.append("\n");
    } else if (has_fields(res)) {
        if (!res->IsInitialized()) {
            rh.set_status_code(HTTP_STATUS_INTERNAL_SERVER_ERROR);
            rh.set_content_type("text/plain");
            body.append("Missing required fields in response: " + res->InitializationErrorString() + "\n");
        } else {
            const bool proto = cntl->has_http_request() && is_proto_content(cntl->http_request().content_type());
            if (proto) {
                std::string bytes;
                res->SerializeToString(&bytes);
                body.append(bytes);
                rh.set_content_type(kProto);
            } else {
                std::string json, err;
                json2pb::Pb2JsonOptions opt;
                const std::string* pretty = cntl->http_request().uri().GetQuery("pretty");
                opt.pretty_json = pretty != nullptr;
                json2pb::ProtoMessageToJson(*res, &json, opt, &err);
                body.append(json);
                if (opt.pretty_json) body.append("\n");
                rh.set_content_type(kJson);
            }
        }
    } else if (cntl->_progressive_attachment) {
        chunked = !http10;
        if (http10) keep_alive = false;
    } else {
        body.swap(cntl->response_attachment());
        if (rh.content_type().empty()) rh.set_content_type("text/plain");
    }
    Buf packet;
    SerializeHttpResponseHead(&packet, rh, chunked || (http10 && cntl->_progressive_attachment) ? -1 : (int64_t)body.size(),
                              chunked, keep_alive);
    if (cntl->http_request().method() != HTTP_METHOD_HEAD) packet.append(std::move(body));
    // a progressive body ends the connection itself (its last chunk, or the
    // close that delimits an HTTP/1.0 body), not with this head
    const bool progressive = cntl->_progressive_attachment != nullptr && !cntl->Failed();
    WriteInOrder(order.get(), order_seq, sock.get(), &packet, !keep_alive && !progressive);
    if (cntl->_progressive_attachment) {
        if (!keep_alive) cntl->_progressive_attachment->set_shutdown_after_end();
        cntl->_progressive_attachment->MarkRPCAsDone(cntl->Failed());
        cntl->_progressive_attachment.reset();
    }
    if (cntl->_span) {
        cntl->_span->sent_real_us = realtime_us();
        cntl->_span->error_code = cntl->ErrorCode();
    }
}

void ProcessHttpRequest(InputMessageBase* msg_base) {
    const int64_t start_us = monotonic_us();
    std::unique_ptr<HttpMessage> msg(static_cast<HttpMessage*>(msg_base));
    Socket* socket = msg->socket();
    Server* server = const_cast<Server*>(static_cast<const Server*>(msg->arg()));
    Controller* cntl = new Controller;
    cntl->_server = server;
    cntl->_server_socket_id = socket->id();
    cntl->_remote_side = socket->remote_side();
    cntl->_local_side = socket->local_side();
    cntl->_received_us = msg->received_us();
    cntl->_begin_us = msg->received_us();
    HttpHeader& req_h = cntl->http_request();
    req_h = msg->header;
    const bool http10 = req_h.major_version() == 1 && req_h.minor_version() == 0;
    const bool keep_alive = msg->keep_alive;
    std::shared_ptr<HttpResponseOrder> order = msg->order;
    const uint64_t order_seq = msg->order_seq;
    if (const std::string* lid = req_h.GetHeader("log-id")) cntl->set_log_id(strtoull(lid->c_str(), nullptr, 10));
    if (!FLAGS_http_header_of_user_ip.empty()) {
        if (const std::string* ip = req_h.GetHeader(FLAGS_http_header_of_user_ip)) {
            EndPoint ep;
            if (str2endpoint(ip->c_str(), 0, &ep) == 0) cntl->_remote_side = ep;
        }
    }
    MethodStatus* ms = nullptr;
    pb::Message* req = nullptr;
    pb::Message* res = nullptr;
    bool concurrency_added = false;
    const Server::MethodProperty* mp = nullptr;
    do {
        if (!server->IsRunning()) {
            cntl->SetFailed(ELOGOFF, "Server is stopping");
            break;
        }
        std::string path;
        for (char ch : req_h.uri().path()) {  // collapse "//"
            if (ch == '/' && !path.empty() && path.back() == '/') continue;
            path.push_back(ch);
        }
        if (path.empty() || path == "/") path = "/index";
        std::string unresolved;
        mp = server->FindMethodPropertyByURI(path, &unresolved);
        if (!mp && (mp = server->master_method_property()) != nullptr) unresolved = path.substr(1);
        if (!mp) {
            cntl->SetFailed(ENOMETHOD, "Fail to find method on `%s'", req_h.uri().path().c_str());
            break;
        }
        req_h.set_unresolved_path(unresolved);
        if (server->options().internal_port > 0 && mp->is_builtin_service &&
            socket->local_side().port != server->options().internal_port) {
            cntl->SetFailed(EPERM, "builtin services are only on internal_port=%d", server->options().internal_port);
            break;
        }
        if (!mp->is_builtin_service) {
            if (!server->AddConcurrency(cntl)) {
                cntl->SetFailed(ELIMIT, "Reached server's max_concurrency=%d", server->max_concurrency());
                break;
            }
            concurrency_added = true;
            int rejected = 0;
            if (!mp->status->OnRequested(&rejected, cntl)) {
                mp->status->OnResponded(ELIMIT, 0);
                cntl->SetFailed(ELIMIT, "Reached method's max_concurrency=%d", rejected - 1);
                break;
            }
            ms = mp->status.get();
        }
        const pb::Message& req_proto = mp->service->GetRequestPrototype(mp->method);
        req = req_proto.New();
        res = mp->service->GetResponsePrototype(mp->method).New();
        if (has_fields(req)) {
            if (is_proto_content(req_h.content_type())) {
                if (!ParsePbFromBuf(req, msg->body)) {
                    cntl->SetFailed(EREQUEST, "Fail to parse proto body as %s", req->GetDescriptor()->full_name.c_str());
                    break;
                }
            } else if (!msg->body.empty()) {
                std::string err;
                json2pb::Json2PbOptions opt;
                if (!json2pb::JsonToProtoMessage(msg->body, req, opt, &err)) {
                    cntl->SetFailed(EREQUEST, "Fail to parse json body: %s", err.c_str());
                    break;
                }
            } else if (!req->IsInitialized()) {
                cntl->SetFailed(EREQUEST, "Missing required fields in request: %s",
                                req->InitializationErrorString().c_str());
                break;
            }
        } else {
            cntl->request_attachment().swap(msg->body);
        }
    } while (false);
    msg.reset();
    if (!concurrency_added) server = nullptr;
    if (cntl->Failed()) {
        SendHttpResponse(cntl, req, res, server, ms, start_us, keep_alive, http10, order, order_seq);
        return;
    }
    Closure* done = NewCallback([cntl, req, res, server, ms, start_us, keep_alive, http10, order, order_seq] {
        SendHttpResponse(cntl, req, res, server, ms, start_us, keep_alive, http10, order, order_seq);
    });
    CallServiceMethod(mp->service, mp->method, cntl, req, res, done);
}

bool VerifyHttpRequest(const InputMessageBase* msg_base) {
    const HttpMessage* msg = static_cast<const HttpMessage*>(msg_base);
    const Server* server = static_cast<const Server*>(msg->arg());
    const Authenticator* auth = server->options().auth;
    if (!auth) return true;
    const std::string* cred = msg->header.GetHeader("Authorization");
    if (!cred) {
        // builtin pages stay reachable without credentials on the internal port
        return false;
    }
    AuthContext ctx;
    return auth->VerifyCredential(*cred, msg->socket()->remote_side(), &ctx) == 0;
}

static const std::string& GetHttpMethodName(const pb::MethodDescriptor* method, const Controller* cntl) {
    static const std::string kCommon = "common_http_request";
    return method ? method->full_name : kCommon;
}

void RegisterHttpProtocol() {
    Protocol p;
    p.parse = ParseHttpMessage;
    p.serialize_request = SerializeHttpRequest;
    p.pack_request = PackHttpRequest;
    p.process_request = ProcessHttpRequest;
    p.process_response = ProcessHttpResponse;
    p.verify = VerifyHttpRequest;
    p.get_method_name = GetHttpMethodName;
    p.supported_connection_type = CONNECTION_TYPE_POOLED | CONNECTION_TYPE_SHORT;
    p.name = "http";
    RegisterProtocol(PROTOCOL_HTTP, p);
}

}  // namespace policy
}  // namespace mrpc
