#include "policy/pbrpc_common.h"

#include <memory>

#include "base/logging.h"
#include "base/time.h"
#include "net/socket.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/protocol.h"
#include "rpc/rpc_dump.h"
#include "rpc/span.h"
#include "rpc/usercode_backup_pool.h"

namespace mrpc {
namespace policy {

const Server::MethodProperty* FindMethodByIndex(const Server* server, const std::string& service_name,
                                                int method_index, int* error_code, std::string* error_text) {
    Service* svc = server->FindServiceByName(service_name);
    if (!svc) svc = server->FindServiceByFullName(service_name);
    if (!svc) {
        *error_code = ENOSERVICE;
        *error_text = "Fail to find service=" + service_name;
        return nullptr;
    }
    const pb::ServiceDescriptor* sd = svc->GetDescriptor();
    if (method_index < 0 || method_index >= (int)sd->methods.size()) {
        *error_code = ENOMETHOD;
        *error_text = "Fail to find method_index=" + std::to_string(method_index) + " of service=" + service_name;
        return nullptr;
    }
    const Server::MethodProperty* mp = server->FindMethodPropertyByFullName(sd->full_name, sd->method(method_index)->name);
    if (!mp) {
        *error_code = ENOMETHOD;
        *error_text = "method " + sd->method(method_index)->name + " is not registered";
    }
    return mp;
}

const Server::MethodProperty* FindMethodByFullName(const Server* server, const std::string& full_method_name,
                                                   int* error_code, std::string* error_text) {
    const Server::MethodProperty* mp = server->FindMethodPropertyByFullName(full_method_name);
    if (mp) return mp;
    const size_t dot = full_method_name.rfind('.');
    if (dot == std::string::npos) {
        *error_code = ENOMETHOD;
        *error_text = "Invalid full method name=" + full_method_name;
        return nullptr;
    }
    const std::string svc = full_method_name.substr(0, dot);
    if (!server->FindServiceByFullName(svc) && !server->FindServiceByName(svc)) {
        *error_code = ENOSERVICE;
        *error_text = "Fail to find service=" + svc;
    } else {
        *error_code = ENOMETHOD;
        *error_text = "Fail to find method=" + full_method_name.substr(dot + 1) + " of service=" + svc;
    }
    return nullptr;
}

namespace {
struct ServerCallState {
    Controller* cntl = nullptr;
    pb::Message* req = nullptr;
    pb::Message* res = nullptr;
    Server* server = nullptr;  // non-null when server concurrency was added
    MethodStatus* ms = nullptr;
    int64_t start_us = 0;
    PbResponsePacker packer;
};

void SendPbResponse(ServerCallState* st) {
    std::unique_ptr<ServerCallState> guard(st);
    std::unique_ptr<Controller> cntl(st->cntl);
    std::unique_ptr<pb::Message> req(st->req);
    std::unique_ptr<pb::Message> res(st->res);
    ConcurrencyRemover remover(st->ms, cntl.get(), st->start_us, st->server);
    SocketUniquePtr sock;
    if (Socket::Address(cntl->_server_socket_id, &sock) != 0) return;
    if (cntl->IsCloseConnection()) {
        sock->SetFailed(ECLOSE, "close connection by user");
        return;
    }
    Span* span = cntl->_span;
    if (span) span->start_send_real_us = realtime_us();
    Buf body;
    if (!cntl->Failed() && res) {
        if (!res->IsInitialized()) {
            cntl->SetFailed(ERESPONSE, "Missing required fields in response: %s", res->InitializationErrorString().c_str());
        } else if (!SerializeAsCompressedData(*res, &body, cntl->response_compress_type())) {
            cntl->SetFailed(ERESPONSE, "Fail to serialize response");
        }
    }
    Buf attachment;
    if (cntl->Failed()) {
        body.clear();
    } else {
        attachment.swap(cntl->response_attachment());
    }
    Buf packet;
    st->packer(cntl.get(), &body, &attachment, &packet);
    if (span) span->response_size = (int64_t)packet.size();
    if (!packet.empty()) {
        WriteOptions wopt;
        wopt.ignore_eovercrowded = true;
        if (sock->Write(&packet, &wopt) != 0) {
            LOG_EVERY_SECOND(WARNING) << "Fail to write response into " << sock->description();
        }
    }
    if (span) {
        span->sent_real_us = realtime_us();
        span->error_code = cntl->ErrorCode();
        Span::Submit(span, monotonic_us());
        cntl->_span = nullptr;
    }
}
}  // namespace

void RunPbServerCall(PbServerRequest* r, PbResponsePacker packer) {
    const int64_t start_us = monotonic_us();
    Socket* socket = r->socket;
    Server* server = r->server;
    Controller* cntl = new Controller;
    cntl->_server = server;
    cntl->_server_socket_id = socket->id();
    cntl->_remote_side = socket->remote_side();
    cntl->_local_side = socket->local_side();
    cntl->_received_us = r->received_us;
    cntl->_begin_us = r->received_us;
    cntl->_protocol_type = r->protocol;
    if (r->has_log_id) cntl->set_log_id(r->log_id);
    cntl->set_request_compress_type(r->compress_type);
    // Legacy protocols answer with the request's compression.
    cntl->set_response_compress_type(r->response_compress >= 0 ? (CompressType)r->response_compress : r->compress_type);
    if (r->timeout_ms > 0) cntl->_deadline_us = r->received_us + r->timeout_ms * 1000;
    const std::string span_name = r->mp ? r->mp->service->GetDescriptor()->full_name + "." + r->mp->method->name
                                        : r->span_method_name;
    if (IsRpczEnabled()) {
        cntl->_span = Span::CreateServerSpan(r->trace_id, r->span_id, r->parent_span_id, span_name, realtime_us());
        if (cntl->_span) {
            cntl->_span->protocol = r->protocol;
            cntl->_span->remote_side = socket->remote_side();
            cntl->_span->start_parse_real_us = realtime_us();
            cntl->_span->request_size = (int64_t)(r->body.size() + r->attachment.size());
            cntl->_span->log_id = r->log_id;
            cntl->_trace_id = cntl->_span->trace_id;
            cntl->_span_id = cntl->_span->span_id;
        }
    }
    if (r->mp) {
        if (SampledRequest* sample = AskToBeSampled()) {
            sample->meta.set_service_name(r->mp->service->GetDescriptor()->full_name);
            sample->meta.set_method_name(r->mp->method->name);
            sample->meta.set_method_index(r->mp->method->index);
            sample->meta.set_compress_type(r->compress_type);
            sample->meta.set_protocol_type(r->protocol);
            sample->meta.set_attachment_size((int32_t)r->attachment.size());
            sample->request = r->body;
            sample->request.append(r->attachment);
            sample->submit();
        }
    }
    ServerCallState* st = new ServerCallState;
    st->cntl = cntl;
    st->start_us = start_us;
    st->packer = std::move(packer);
    const Server::MethodProperty* mp = r->mp;
    do {
        if (!server->IsRunning()) {
            cntl->SetFailed(ELOGOFF, "Server is stopping");
            break;
        }
        if (server->options().auth && !r->auth_data.empty()) {
            AuthContext ctx;
            if (server->options().auth->VerifyCredential(r->auth_data, socket->remote_side(), &ctx) != 0) {
                cntl->SetFailed(ERPCAUTH, "Fail to authenticate");
                break;
            }
        }
        if (!server->AddConcurrency(cntl)) {
            cntl->SetFailed(ELIMIT, "Reached server's max_concurrency=%d", server->max_concurrency());
            break;
        }
        st->server = server;
        if (!mp) {
            cntl->SetFailed(r->error_code ? r->error_code : ENOMETHOD, "%s", r->error_text.c_str());
            break;
        }
        int rejected = 0;
        if (!mp->status->OnRequested(&rejected, cntl)) {
            mp->status->OnResponded(ELIMIT, 0);
            cntl->SetFailed(ELIMIT, "Reached method's max_concurrency=%d", rejected - 1);
            break;
        }
        st->ms = mp->status.get();
        cntl->request_attachment().swap(r->attachment);
        st->req = mp->service->GetRequestPrototype(mp->method).New();
        if (!ParseFromCompressedData(r->body, st->req, r->compress_type)) {
            cntl->SetFailed(EREQUEST, "Fail to parse request message, CompressType=%d, size=%zu", (int)r->compress_type,
                            r->body.size());
            break;
        }
        st->res = mp->service->GetResponsePrototype(mp->method).New();
    } while (false);
    r->body.clear();
    if (cntl->Failed()) {
        SendPbResponse(st);
        return;
    }
    if (cntl->_span) cntl->_span->start_callback_real_us = realtime_us();
    Span::set_tls_parent(cntl->_span);
    Closure* done = NewCallback([st] { SendPbResponse(st); });
    CallServiceMethod(mp->service, mp->method, cntl, st->req, st->res, done);
}

void CompleteClientCallWith(fiber::CallId cid, Socket* sock, const std::function<int(Controller*)>& fill) {
    Controller* cntl = nullptr;
    if (fiber::call_id_lock(cid, (void**)&cntl) != 0) return;  // timed out / canceled / duplicated
    if (cid != cntl->current_id() && cid != cntl->_unfinished_call.id) {
        fiber::call_id_unlock(cid);  // response of an obsolete attempt
        return;
    }
    const int saved_error = fill(cntl);
    if (sock) cntl->_local_side = sock->local_side();
    cntl->OnVersionedRPCReturned(cid, saved_error);
}

void CompletePbClientCall(fiber::CallId cid, int error_code, const std::string& error_text, Buf* body,
                          Buf* attachment, CompressType ct, Socket* sock) {
    CompleteClientCallWith(cid, sock, [&](Controller* cntl) -> int {
        if (error_code != 0) {
            cntl->_error_code = 0;
            cntl->_error_text.clear();
            cntl->SetFailed(error_code, "%s", error_text.c_str());
            return error_code;
        }
        cntl->response_attachment().clear();
        if (attachment) cntl->response_attachment().swap(*attachment);
        if (cntl->_response && !ParseFromCompressedData(*body, cntl->_response, ct)) {
            cntl->SetFailed(ERESPONSE, "Fail to parse response message, CompressType=%d, size=%zu", (int)ct, body->size());
            return ERESPONSE;
        }
        cntl->set_response_compress_type(ct);
        return 0;
    });
}

}  // namespace policy
}  // namespace mrpc
