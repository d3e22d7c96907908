#include "rpc/nshead.h"

#include <unistd.h>

#include "base/logging.h"
#include "base/snappy.h"
#include "base/time.h"
#include "mcpack/mcpack.h"
#include "mrpc/proto/legacy_meta.pb.h"
#include "net/socket.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/method_status.h"
#include "rpc/protocol.h"
#include "rpc/server.h"
#include "rpc/span.h"
#include "rpc/usercode_backup_pool.h"

namespace mrpc {

using policy::NsheadMeta;

const pb::Descriptor* NsheadMessage::GetDescriptor() const { return OpaqueDescriptor("mrpc.NsheadMessage"); }

void PackNsheadFrame(Buf* out, const nshead_t& head, const Buf& body) {
    nshead_t h = head;
    h.magic_num = NSHEAD_MAGICNUM;
    h.body_len = (uint32_t)body.size();
    out->append(&h, sizeof(h));
    out->append(body);
}

// ------------------------------------------------------------ NsheadClosure

NsheadClosure::NsheadClosure() : _cntl(new Controller) {}
NsheadClosure::~NsheadClosure() {}

void NsheadClosure::Run() {
    std::unique_ptr<NsheadClosure> self(this);
    Controller* cntl = _cntl.get();
    NsheadService* svc = _server->options().nshead_service;
    ConcurrencyRemover remover(svc ? svc->status() : nullptr, cntl, _received_us,
                               _added_concurrency ? _server : nullptr);
    SocketUniquePtr sock;
    if (Socket::Address(cntl->_server_socket_id, &sock) != 0) return;
    if (cntl->IsCloseConnection()) {
        sock->SetFailed(ECLOSE, "close connection by nshead service");
        return;
    }
    Span* span = cntl->_span;
    if (span) span->start_send_real_us = realtime_us();
    if (_sequencer) {
        Buf packet;
        if (_do_respond) {
            nshead_t h = _request.head;
            const nshead_t& rh = _response.head;
            if (rh.version) h.version = rh.version;
            if (rh.reserved) h.reserved = rh.reserved;
            if (rh.id) h.id = rh.id;
            if (rh.provider[0]) memcpy(h.provider, rh.provider, sizeof(h.provider));
            PackNsheadFrame(&packet, h, _response.body);
            if (span) span->response_size = (int64_t)packet.size();
        }
        _sequencer->Deliver(_seq, &packet, sock.get());
    } else if (_do_respond) {
        // The response head defaults to the request's (log_id, id, provider).
        nshead_t h = _request.head;
        const nshead_t& rh = _response.head;
        if (rh.version) h.version = rh.version;
        if (rh.reserved) h.reserved = rh.reserved;
        if (rh.id) h.id = rh.id;
        if (rh.provider[0]) memcpy(h.provider, rh.provider, sizeof(h.provider));
        Buf packet;
        PackNsheadFrame(&packet, h, _response.body);
        if (span) span->response_size = (int64_t)packet.size();
        WriteOptions wopt;
        wopt.ignore_eovercrowded = true;
        if (sock->Write(&packet, &wopt) != 0) {
            LOG_EVERY_SECOND(WARNING) << "Fail to write nshead response into " << sock->description();
        }
    }
    if (span) {
        span->sent_real_us = realtime_us();
        span->error_code = cntl->ErrorCode();
        Span::Submit(span, monotonic_us());
        cntl->_span = nullptr;
    }
}

// ------------------------------------------------------------ NsheadService

NsheadService::NsheadService() : _status(new MethodStatus) {}
NsheadService::~NsheadService() {}
void NsheadService::Expose(const std::string& prefix) { _status->Expose(prefix); }

void NsheadPbServiceAdaptor::ProcessNsheadRequest(const Server& server, Controller* cntl, const NsheadMessage& request,
                                                  NsheadMessage* response, NsheadClosure* done) {
    std::shared_ptr<NsheadMeta> meta(new NsheadMeta);
    const Server::MethodProperty* mp = nullptr;
    do {
        if (cntl->Failed()) break;
        ParseNsheadMeta(server, request, cntl, meta.get());
        if (cntl->Failed()) break;
        if (meta->has_log_id()) cntl->set_log_id((uint64_t)meta->log_id());
        mp = server.FindMethodPropertyByFullName(meta->full_method_name());
        if (!mp) {
            cntl->SetFailed(ENOMETHOD, "Fail to find method=%s", meta->full_method_name().c_str());
            break;
        }
        if (cntl->_span) cntl->_span->full_method_name = meta->full_method_name();
        int rejected = 0;
        if (!mp->status->OnRequested(&rejected, cntl)) {
            mp->status->OnResponded(ELIMIT, 0);
            mp = nullptr;
            cntl->SetFailed(ELIMIT, "Reached method's max_concurrency=%d", rejected - 1);
            break;
        }
    } while (false);
    if (cntl->Failed()) {
        SerializeResponseToBuf(*meta, cntl, nullptr, response);
        done->Run();
        return;
    }
    pb::Message* req = mp->service->GetRequestPrototype(mp->method).New();
    pb::Message* res = mp->service->GetResponsePrototype(mp->method).New();
    MethodStatus* ms = mp->status.get();
    const int64_t received_us = done->received_us();
    Closure* pb_done = NewCallback([this, meta, cntl, req, res, response, done, ms, received_us] {
        std::unique_ptr<pb::Message> rq(req), rs(res);
        if (!cntl->IsCloseConnection()) SerializeResponseToBuf(*meta, cntl, cntl->Failed() ? nullptr : res, response);
        { ConcurrencyRemover remover(ms, cntl, received_us); }
        done->Run();
    });
    ParseRequestFromBuf(*meta, request, cntl, req);
    if (cntl->Failed()) {
        pb_done->Run();
        return;
    }
    CallServiceMethod(mp->service, mp->method, cntl, req, res, pb_done);
}

// ------------------------------------------------------------ nova_pbrpc

void NovaServiceAdaptor::ParseNsheadMeta(const Server& server, const NsheadMessage& request, Controller* cntl,
                                         NsheadMeta* out) const {
    Service* svc = server.first_service();
    if (!svc) {
        cntl->SetFailed(ENOSERVICE, "No service in server");
        return;
    }
    const pb::ServiceDescriptor* sd = svc->GetDescriptor();
    const int idx = (int)request.head.reserved;
    if (idx < 0 || idx >= sd->method_count()) {
        cntl->SetFailed(ENOMETHOD, "Fail to find method by index=%d", idx);
        return;
    }
    out->set_full_method_name(sd->full_name + "." + sd->method(idx)->name);
    if (request.head.version & NOVA_SNAPPY_COMPRESS_FLAG) out->set_compress_type(COMPRESS_TYPE_SNAPPY);
    if (request.head.log_id) out->set_log_id(request.head.log_id);
}

void NovaServiceAdaptor::ParseRequestFromBuf(const NsheadMeta& meta, const NsheadMessage& raw_req, Controller* cntl,
                                             pb::Message* pb_req) const {
    const CompressType ct = meta.compress_type();
    if (!ParseFromCompressedData(raw_req.body, pb_req, ct)) {
        cntl->SetFailed(EREQUEST, "Fail to parse nova request, CompressType=%d", (int)ct);
        return;
    }
    cntl->set_request_compress_type(ct);
}

void NovaServiceAdaptor::SerializeResponseToBuf(const NsheadMeta& meta, Controller* cntl, const pb::Message* pb_res,
                                                NsheadMessage* raw_res) const {
    if (cntl->Failed()) {
        // nova carries no error field: the connection is the only signal.
        cntl->CloseConnection("nova request failed");
        return;
    }
    const CompressType ct = meta.compress_type();
    if (!SerializeAsCompressedData(*pb_res, &raw_res->body, ct)) {
        cntl->CloseConnection("Fail to serialize nova response");
        return;
    }
    if (ct == COMPRESS_TYPE_SNAPPY) raw_res->head.version = NOVA_SNAPPY_COMPRESS_FLAG;
}

// ------------------------------------------------------------ public_pbrpc

static const uint32_t kPublicSnappy = 1;

void PublicPbrpcServiceAdaptor::ParseNsheadMeta(const Server& server, const NsheadMessage& request, Controller* cntl,
                                                NsheadMeta* out) const {
    policy::PublicPbrpcRequest whole;
    if (!ParsePbFromBuf(&whole, request.body)) {
        cntl->CloseConnection("Fail to parse PublicPbrpcRequest");
        return;
    }
    if (whole.requestBody_size() == 0) {
        cntl->CloseConnection("PublicPbrpcRequest has no body");
        return;
    }
    const policy::RequestHead& head = whole.requestHead();
    const policy::RequestBody& body = whole.requestBody(0);
    Service* svc = server.FindServiceByName(body.service());
    if (!svc) svc = server.FindServiceByFullName(body.service());
    if (!svc || (int)body.method_id() >= svc->GetDescriptor()->method_count()) {
        cntl->SetFailed(ENOMETHOD, "Fail to find method by service=%s method_id=%u", body.service().c_str(),
                        body.method_id());
        return;
    }
    const pb::ServiceDescriptor* sd = svc->GetDescriptor();
    out->set_full_method_name(sd->full_name + "." + sd->method((int)body.method_id())->name);
    out->set_correlation_id((int64_t)body.id());
    if (head.has_log_id()) out->set_log_id((int64_t)head.log_id());
    if (head.compress_type() == kPublicSnappy) out->set_compress_type(COMPRESS_TYPE_SNAPPY);
    out->set_user_string(body.version());
    // Leave only the serialized request in the body for ParseRequestFromBuf.
    NsheadMessage& mut = const_cast<NsheadMessage&>(request);
    mut.body.clear();
    mut.body.append(body.serialized_request());
}

void PublicPbrpcServiceAdaptor::ParseRequestFromBuf(const NsheadMeta& meta, const NsheadMessage& raw_req,
                                                    Controller* cntl, pb::Message* pb_req) const {
    if (!ParseFromCompressedData(raw_req.body, pb_req, meta.compress_type())) {
        cntl->SetFailed(EREQUEST, "Fail to parse public_pbrpc request");
        return;
    }
    cntl->set_request_compress_type(meta.compress_type());
}

void PublicPbrpcServiceAdaptor::SerializeResponseToBuf(const NsheadMeta& meta, Controller* cntl,
                                                       const pb::Message* pb_res, NsheadMessage* raw_res) const {
    policy::PublicPbrpcResponse whole;
    policy::ResponseHead* head = whole.mutable_responseHead();
    policy::ResponseBody* body = whole.add_responseBody();
    char host[256] = {0};
    gethostname(host, sizeof(host) - 1);
    head->set_from_host(host);
    body->set_version(meta.user_string());
    body->set_id((uint64_t)meta.correlation_id());
    if (cntl->Failed() || !pb_res) {
        head->set_code(cntl->ErrorCode() ? cntl->ErrorCode() : EINTERNAL);
        head->set_text(cntl->ErrorText());
    } else {
        head->set_code(0);
        head->set_text("success");
        Buf res;
        if (!SerializeAsCompressedData(*pb_res, &res, meta.compress_type())) {
            cntl->CloseConnection("Fail to serialize public_pbrpc response");
            return;
        }
        body->set_serialized_response(res.to_string());
        if (meta.compress_type() == COMPRESS_TYPE_SNAPPY) head->set_compress_type(kPublicSnappy);
    }
    whole.SerializeToBuf(&raw_res->body);
}

// ------------------------------------------------------------ nshead_mcpack

void NsheadMcpackAdaptor::ParseNsheadMeta(const Server& server, const NsheadMessage& request, Controller* cntl,
                                          NsheadMeta* out) const {
    if (!_method.empty()) {
        out->set_full_method_name(_method);
    } else {
        Service* svc = server.first_service();
        if (!svc || svc->GetDescriptor()->method_count() == 0) {
            cntl->SetFailed(ENOSERVICE, "No service for nshead_mcpack");
            return;
        }
        out->set_full_method_name(svc->GetDescriptor()->full_name + "." + svc->GetDescriptor()->method(0)->name);
    }
    if (request.head.log_id) out->set_log_id(request.head.log_id);
}

void NsheadMcpackAdaptor::ParseRequestFromBuf(const NsheadMeta&, const NsheadMessage& raw_req, Controller* cntl,
                                              pb::Message* pb_req) const {
    if (!mcpack::ParseFromBuf(raw_req.body, pb_req)) {
        cntl->SetFailed(EREQUEST, "Fail to parse mcpack request of %s", pb_req->GetTypeName().c_str());
    }
}

void NsheadMcpackAdaptor::SerializeResponseToBuf(const NsheadMeta&, Controller* cntl, const pb::Message* pb_res,
                                                 NsheadMessage* raw_res) const {
    if (cntl->Failed() || !pb_res) {
        cntl->CloseConnection("nshead_mcpack request failed");
        return;
    }
    if (!mcpack::SerializeToBuf(*pb_res, mcpack::FORMAT_MCPACK_V2, &raw_res->body)) {
        cntl->CloseConnection("Fail to serialize mcpack response");
    }
}

}  // namespace mrpc
