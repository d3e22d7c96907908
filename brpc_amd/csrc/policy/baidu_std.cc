// baidu_std protocol (role of src/brpc/policy/baidu_rpc_protocol.cpp:57-767):
//   "PRPC" | body_size (u32 BE) | meta_size (u32 BE) | RpcMeta | payload | attachment
// MI355X-native: attachment blocks that live in HBM are moved by the
// socket's device transport and described in RpcMeta.device_payload
// (policy/device_payload.h); everything else is byte-identical to baidu_std.
#include <cerrno>
#include <memory>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"
#include "fiber/call_id.h"
#include "gpu/rccl_plane.h"
#include "gpu/xgmi.h"
#include "mrpc/proto/rpc_meta.pb.h"
#include "policy/device_payload.h"
#include "policy/policies.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/protocol.h"
#include "rpc/server.h"
#include "rpc/span.h"
#include "rpc/rpc_dump.h"
#include "rpc/stream_internal.h"
#include "rpc/usercode_backup_pool.h"

DECLARE_uint64(max_body_size);
DEFINE_bool(baidu_protocol_use_fullname, true, "put the full service name in requests");
DEFINE_bool(baidu_std_protocol_deliver_timeout_ms, false, "put timeout_ms in request meta");

namespace mrpc {
namespace policy {

static inline void PackRpcHeader(char* h, uint32_t meta_size, uint32_t payload_size) {
    memcpy(h, "PRPC", 4);
    pack_be32(h + 4, meta_size + payload_size);
    pack_be32(h + 8, meta_size);
}

void SerializeRpcHeaderAndMeta(Buf* out, const RpcMeta& meta, size_t payload_size) {
    const uint32_t meta_size = (uint32_t)meta.ByteSizeLong();
    char* p = out->append_contiguous(12 + meta_size);
    PackRpcHeader(p, meta_size, (uint32_t)payload_size);
    meta.SerializeWithCachedSizesToArray((uint8_t*)p + 12);
}

ParseResult ParseRpcMessage(Buf* source, Socket* socket, bool, const void*) {
    char header[12];
    const size_t n = source->copy_to(header, sizeof(header));
    if (n >= 4) {
        if (memcmp(header, "PRPC", 4) != 0) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
    } else {
        if (memcmp(header, "PRPC", n) != 0) return MakeParseError(PARSE_ERROR_TRY_OTHERS);
        return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    }
    if (n < sizeof(header)) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    const uint32_t body_size = unpack_be32(header + 4);
    const uint32_t meta_size = unpack_be32(header + 8);
    if (body_size > FLAGS_max_body_size) {
        LOG(ERROR) << "body_size=" << body_size << " from " << socket->remote_side() << " is too large";
        return MakeParseError(PARSE_ERROR_TOO_BIG_DATA);
    }
    if (source->size() < sizeof(header) + body_size) return MakeParseError(PARSE_ERROR_NOT_ENOUGH_DATA);
    if (meta_size > body_size) {
        LOG(ERROR) << "meta_size=" << meta_size << " is bigger than body_size=" << body_size;
        source->pop_front(sizeof(header) + body_size);
        return MakeParseError(PARSE_ERROR_ABSOLUTELY_WRONG);
    }
    source->pop_front(sizeof(header));
    MostCommonMessage* msg = MostCommonMessage::Get();
    source->cutn(&msg->meta, meta_size);
    source->cutn(&msg->payload, body_size - meta_size);
    return MakeMessage(msg);
}

void SerializeRpcRequest(Buf* buf, Controller* cntl, const pb::Message* request) {
    if (!request) {
        cntl->SetFailed(EREQUEST, "request is NULL");
        return;
    }
    if (!request->IsInitialized()) {
        cntl->SetFailed(EREQUEST, "Missing required fields in request: %s", request->InitializationErrorString().c_str());
        return;
    }
    if (!SerializeAsCompressedData(*request, buf, cntl->request_compress_type())) {
        cntl->SetFailed(EREQUEST, "Fail to compress request");
    }
}

void PackRpcRequest(Buf* packet, uint64_t correlation_id, const pb::MethodDescriptor* method, Controller* cntl,
                    const Buf& request_buf, const Authenticator* auth) {
    RpcMeta meta;
    RpcRequestMeta* rm = meta.mutable_request();
    if (method) {
        rm->set_service_name(FLAGS_baidu_protocol_use_fullname ? method->service->full_name : method->service->name);
        rm->set_method_name(method->name);
    } else {
        cntl->SetFailed(EREQUEST, "method is NULL");
        return;
    }
    meta.set_compress_type(cntl->request_compress_type());
    meta.set_correlation_id((int64_t)correlation_id);
    if (cntl->log_id()) rm->set_log_id((int64_t)cntl->log_id());
    if (cntl->trace_id()) {
        rm->set_trace_id((int64_t)cntl->trace_id());
        rm->set_span_id((int64_t)cntl->span_id());
        if (cntl->_parent_span_id) rm->set_parent_span_id((int64_t)cntl->_parent_span_id);
    }
    if (!cntl->request_id().empty()) rm->set_request_id(cntl->request_id());
    if (FLAGS_baidu_std_protocol_deliver_timeout_ms && cntl->timeout_ms() > 0) rm->set_timeout_ms((int32_t)cntl->timeout_ms());
    if (auth) {
        std::string cred;
        if (auth->GenerateCredential(&cred) != 0) {
            cntl->SetFailed(ERPCAUTH, "Fail to generate credential");
            return;
        }
        meta.set_authentication_data(cred);
    }
    StreamId sid = cntl->_request_stream;
    if (sid) FillStreamSettings(sid, meta.mutable_stream_settings());
    // xGMI hello: offered on every request until the connection has a
    // device transport, so each response that could carry device payloads
    // also carries the server's arena description.
    if (cntl->_use_device_transport && cntl->_pack_socket && !cntl->_pack_socket->transport()) {
        gpu::FillXgmiHello(meta.mutable_xgmi_hello());
    }
    // RCCL plane hello: offered until a response told us whether the
    // server is a rank of our plane
    if (cntl->_pack_socket && cntl->_pack_socket->plane_rank() == Socket::kPlaneUnknown) {
        gpu::rccl::FillHello(meta.mutable_plane_hello());
    }
    Buf host_attachment;
    if (!SplitDevicePayload(cntl, /*request=*/true, cntl->request_attachment(), &host_attachment, &meta)) return;
    if (host_attachment.size()) meta.set_attachment_size((int32_t)host_attachment.size());
    SerializeRpcHeaderAndMeta(packet, meta, request_buf.size() + host_attachment.size());
    packet->append(request_buf);
    packet->append(std::move(host_attachment));
}

static void SendRpcResponse(int64_t correlation_id, Controller* cntl, pb::Message* req, pb::Message* res,
                            Server* server, MethodStatus* method_status, int64_t received_us) {
    std::unique_ptr<Controller> cntl_guard(cntl);
    std::unique_ptr<pb::Message> req_guard(req);
    std::unique_ptr<pb::Message> res_guard(res);
    ConcurrencyRemover remover(method_status, cntl, received_us, server);
    SocketUniquePtr sock;
    if (Socket::Address(cntl->_server_socket_id, &sock) != 0) return;  // client gone
    if (cntl->IsCloseConnection()) {
        sock->SetFailed(ECLOSE, "close connection by user");
        return;
    }
    Span* span = cntl->_span;
    if (span) span->start_send_real_us = realtime_us();
    RpcMeta meta;
    Buf res_body;
    if (!cntl->Failed() && res) {
        if (!res->IsInitialized()) {
            cntl->SetFailed(ERESPONSE, "Missing required fields in response: %s", res->InitializationErrorString().c_str());
        } else if (!SerializeAsCompressedData(*res, &res_body, cntl->response_compress_type())) {
            cntl->SetFailed(ERESPONSE, "Fail to serialize response");
        }
    }
    Buf host_attachment;
    if (cntl->Failed()) {
        meta.mutable_response()->set_error_code(cntl->ErrorCode());
        meta.mutable_response()->set_error_text(cntl->ErrorText());
        res_body.clear();
    } else {
        meta.set_compress_type(cntl->response_compress_type());
        if (!SplitDevicePayload(cntl, /*request=*/false, cntl->response_attachment(), &host_attachment, &meta, sock.get())) {
            res_body.clear();
            meta.Clear();
            meta.mutable_response()->set_error_code(cntl->ErrorCode());
            meta.mutable_response()->set_error_text(cntl->ErrorText());
        } else if (host_attachment.size()) {
            meta.set_attachment_size((int32_t)host_attachment.size());
        }
    }
    meta.set_correlation_id(correlation_id);
    if (cntl->_reply_xgmi_hello) gpu::FillXgmiHello(meta.mutable_xgmi_hello());
    if (cntl->_reply_plane_hello) gpu::rccl::FillHello(meta.mutable_plane_hello());
    if (cntl->_response_stream) FillStreamSettings(cntl->_response_stream, meta.mutable_stream_settings());
    Buf packet;
    SerializeRpcHeaderAndMeta(&packet, meta, res_body.size() + host_attachment.size());
    packet.append(std::move(res_body));
    packet.append(std::move(host_attachment));
    if (span) span->response_size = (int64_t)packet.size();
    WriteOptions wopt;
    wopt.ignore_eovercrowded = true;
    if (sock->Write(&packet, &wopt) != 0) {
        LOG_EVERY_SECOND(WARNING) << "Fail to write response into " << sock->description();
    }
    if (cntl->_response_stream) OnServerStreamCreated(cntl->_response_stream, sock->id());
    if (span) {
        span->sent_real_us = realtime_us();
        span->error_code = cntl->ErrorCode();
        Span::Submit(span, monotonic_us());
        cntl->_span = nullptr;
    }
}

void ProcessRpcRequest(InputMessageBase* msg_base) {
    const int64_t start_parse_us = monotonic_us();
    MostCommonMessage* msg = static_cast<MostCommonMessage*>(msg_base);
    struct Destroyer {
        MostCommonMessage* m;
        ~Destroyer() { if (m) m->Destroy(); }
    } destroyer{msg};
    Socket* socket = msg->socket();
    Server* server = const_cast<Server*>(static_cast<const Server*>(msg->arg()));
    RpcMeta meta;
    if (!ParsePbFromBuf(&meta, msg->meta)) {
        LOG(WARNING) << "Fail to parse RpcMeta from " << socket->remote_side();
        socket->SetFailed(EREQUEST, "fail to parse RpcMeta");
        return;
    }
    const RpcRequestMeta& rm = meta.request();
    Controller* cntl = new Controller;
    cntl->_server = server;
    cntl->_server_socket_id = socket->id();
    cntl->_remote_side = socket->remote_side();
    cntl->_local_side = socket->local_side();
    cntl->_server_correlation_id = meta.correlation_id();
    cntl->_received_us = msg->received_us();
    cntl->_begin_us = msg->received_us();
    if (rm.has_log_id()) cntl->set_log_id((uint64_t)rm.log_id());
    cntl->set_request_compress_type((CompressType)meta.compress_type());
    if (rm.has_request_id()) cntl->set_request_id(rm.request_id());
    if (rm.has_timeout_ms() && rm.timeout_ms() > 0) cntl->_deadline_us = msg->received_us() + (int64_t)rm.timeout_ms() * 1000;
    if (IsRpczEnabled()) {
        cntl->_span = Span::CreateServerSpan((uint64_t)rm.trace_id(), (uint64_t)rm.span_id(), (uint64_t)rm.parent_span_id(),
                                             rm.service_name() + "." + rm.method_name(),
                                             realtime_us() - (monotonic_us() - msg->received_us()));
        if (cntl->_span) {
            cntl->_span->remote_side = socket->remote_side();
            cntl->_span->start_parse_real_us = realtime_us();
            cntl->_span->request_size = (int64_t)(msg->meta.size() + msg->payload.size() + 12);
            cntl->_span->log_id = (uint64_t)rm.log_id();
            cntl->_trace_id = cntl->_span->trace_id;
            cntl->_span_id = cntl->_span->span_id;
        }
    }
    if (meta.has_xgmi_hello() && gpu::XgmiEnabled()) {
        std::string err;
        if (gpu::AttachXgmiPeer(socket, meta.xgmi_hello(), &err) == 0) {
            cntl->_reply_xgmi_hello = true;
        } else {
            LOG_EVERY_SECOND(WARNING) << "xGMI peer " << socket->remote_side() << " not attached: " << err;
        }
    }
    if (meta.has_plane_hello()) {
        socket->set_plane_rank(gpu::rccl::PeerRank(meta.plane_hello()));
        cntl->_reply_plane_hello = true;
    }
    if (SampledRequest* sample = AskToBeSampled()) {
        sample->meta.set_service_name(rm.service_name());
        sample->meta.set_method_name(rm.method_name());
        sample->meta.set_compress_type((CompressType)meta.compress_type());
        sample->meta.set_protocol_type(PROTOCOL_BAIDU_STD);
        sample->meta.set_attachment_size(meta.attachment_size());
        if (meta.has_authentication_data()) sample->meta.set_authentication_data(meta.authentication_data());
        sample->request = msg->payload;  // shares the blocks
        sample->submit();
    }
    const int64_t corr = meta.correlation_id();
    MethodStatus* ms = nullptr;
    pb::Message* req = nullptr;
    pb::Message* res = nullptr;
    bool concurrency_added = false;
    bool device_payload_taken = false;  // pulled, or released by the merge on failure
    const Server::MethodProperty* mp = nullptr;
    do {
        if (!server->IsRunning()) {
            cntl->SetFailed(ELOGOFF, "Server is stopping");
            break;
        }
        if (!server->AddConcurrency(cntl)) {
            cntl->SetFailed(ELIMIT, "Reached server's max_concurrency=%d", server->max_concurrency());
            break;
        }
        concurrency_added = true;
        if (!meta.has_request()) {
            cntl->SetFailed(EREQUEST, "RpcMeta has no request meta");
            break;
        }
        mp = server->FindMethodPropertyByFullName(rm.service_name(), rm.method_name());
        if (!mp) {
            if (!server->FindServiceByFullName(rm.service_name()) && !server->FindServiceByName(rm.service_name())) {
                cntl->SetFailed(ENOSERVICE, "Fail to find service=%s", rm.service_name().c_str());
            } else {
                cntl->SetFailed(ENOMETHOD, "Fail to find method=%s of service=%s", rm.method_name().c_str(),
                                rm.service_name().c_str());
            }
            break;
        }
        int rejected = 0;
        if (!mp->status->OnRequested(&rejected, cntl)) {
            ms = nullptr;
            mp->status->OnResponded(ELIMIT, 0);
            cntl->SetFailed(ELIMIT, "Reached method's max_concurrency=%d", rejected - 1);
            break;
        }
        ms = mp->status.get();
        Buf req_buf;
        const int attach_size = meta.attachment_size();
        if (attach_size > 0) {
            if ((size_t)attach_size > msg->payload.size()) {
                cntl->SetFailed(EREQUEST, "attachment_size=%d is larger than payload=%zu", attach_size, msg->payload.size());
                break;
            }
            msg->payload.cutn(&req_buf, msg->payload.size() - attach_size);
            cntl->request_attachment().swap(msg->payload);
        } else {
            req_buf.swap(msg->payload);
        }
        device_payload_taken = true;
        if (meta.device_payload_size() > 0) {
            Span::set_tls_parent(cntl->_span);  // rpcz: annotate the xGMI pull
            if (!MergeDevicePayload(cntl, socket, meta, /*request=*/true, &cntl->request_attachment())) break;
        }
        if (meta.has_stream_settings()) OnRequestStreamSettings(cntl, socket, meta.stream_settings());
        req = mp->service->GetRequestPrototype(mp->method).New();
        if (!ParseFromCompressedData(req_buf, req, (CompressType)meta.compress_type())) {
            cntl->SetFailed(EREQUEST, "Fail to parse request message, CompressType=%d, size=%zu", meta.compress_type(),
                            req_buf.size());
            break;
        }
        res = mp->service->GetResponsePrototype(mp->method).New();
    } while (false);
    // rejected before the attachment was looked at: the sender's lent HBM
    // blocks must still be given back, or they stay pinned on its side
    if (!device_payload_taken) ReleaseDevicePayload(socket, meta);
    msg->Destroy();
    destroyer.m = nullptr;
    if (!concurrency_added) server = nullptr;  // nothing to remove
    if (cntl->Failed()) {
        SendRpcResponse(corr, cntl, req, res, server, ms, start_parse_us);
        return;
    }
    if (cntl->_span) cntl->_span->start_callback_real_us = realtime_us();
    Span::set_tls_parent(cntl->_span);
    Closure* done = NewCallback([corr, cntl, req, res, server, ms, start_parse_us] {
        SendRpcResponse(corr, cntl, req, res, server, ms, start_parse_us);
    });
    CallServiceMethod(mp->service, mp->method, cntl, req, res, done);
}

bool VerifyRpcRequest(const InputMessageBase* msg_base) {
    const MostCommonMessage* msg = static_cast<const MostCommonMessage*>(msg_base);
    const Server* server = static_cast<const Server*>(msg->arg());
    const Authenticator* auth = server->options().auth;
    if (!auth) return true;
    RpcMeta meta;
    if (!ParsePbFromBuf(&meta, msg->meta)) return false;
    AuthContext ctx;
    return auth->VerifyCredential(meta.authentication_data(), msg->socket()->remote_side(), &ctx) == 0;
}

void ProcessRpcResponse(InputMessageBase* msg_base) {
    MostCommonMessage* msg = static_cast<MostCommonMessage*>(msg_base);
    RpcMeta meta;
    if (!ParsePbFromBuf(&meta, msg->meta)) {
        LOG(WARNING) << "Fail to parse RpcMeta from " << msg->socket()->remote_side();
        msg->Destroy();
        return;
    }
    if (meta.has_stream_settings() && !meta.has_correlation_id()) {
        ReleaseDevicePayload(msg->socket(), meta);
        msg->Destroy();
        return;
    }
    const fiber::CallId cid{(uint64_t)meta.correlation_id()};
    Controller* cntl = nullptr;
    if (fiber::call_id_lock(cid, (void**)&cntl) != 0) {
        ReleaseDevicePayload(msg->socket(), meta);
        msg->Destroy();  // timed out / canceled / duplicated response
        return;
    }
    if (cid != cntl->current_id() && cid != cntl->_unfinished_call.id) {
        fiber::call_id_unlock(cid);  // response of an obsolete attempt
        ReleaseDevicePayload(msg->socket(), meta);
        msg->Destroy();
        return;
    }
    if (cntl->_span) {
        const int64_t now = realtime_us();
        cntl->_span->start_parse_real_us = now;
        cntl->_span->cut_real_us = now - (monotonic_us() - msg->received_us());
    }
    if (meta.has_xgmi_hello() && gpu::XgmiEnabled()) {
        std::string err;
        if (gpu::AttachXgmiPeer(msg->socket(), meta.xgmi_hello(), &err) != 0) {
            LOG_EVERY_SECOND(WARNING) << "xGMI peer " << msg->socket()->remote_side() << " not attached: " << err;
        }
    }
    if (msg->socket()->plane_rank() == Socket::kPlaneUnknown) {
        msg->socket()->set_plane_rank(meta.has_plane_hello() ? gpu::rccl::PeerRank(meta.plane_hello()) : -1);
    }
    msg->socket()->DeviceHelloAnswered();  // requests waiting to learn the transports go ahead
    int saved_error = 0;
    bool device_payload_taken = false;
    const RpcResponseMeta& rm = meta.response();
    if (rm.error_code() != 0) {
        cntl->_error_code = 0;
        cntl->_error_text.clear();
        cntl->SetFailed(rm.error_code(), "%s", rm.error_text().c_str());
        saved_error = rm.error_code();
    } else {
        Buf res_buf;
        const int attach_size = meta.attachment_size();
        cntl->response_attachment().clear();
        if (attach_size > 0) {
            if ((size_t)attach_size > msg->payload.size()) {
                cntl->SetFailed(ERESPONSE, "attachment_size=%d > payload", attach_size);
                saved_error = ERESPONSE;
            } else {
                msg->payload.cutn(&res_buf, msg->payload.size() - attach_size);
                cntl->response_attachment().swap(msg->payload);
            }
        } else {
            res_buf.swap(msg->payload);
        }
        if (!saved_error && meta.device_payload_size() > 0) {
            device_payload_taken = true;
            Span* const prev_span = Span::tls_parent();
            Span::set_tls_parent(cntl->_span);  // rpcz: annotate the xGMI pull
            if (!MergeDevicePayload(cntl, msg->socket(), meta, /*request=*/false, &cntl->response_attachment())) {
                saved_error = cntl->ErrorCode();
            }
            Span::set_tls_parent(prev_span);
        }
        if (!saved_error && meta.has_stream_settings()) OnResponseStreamSettings(cntl, msg->socket(), meta.stream_settings());
        if (!saved_error && cntl->_response &&
            !ParseFromCompressedData(res_buf, cntl->_response, (CompressType)meta.compress_type())) {
            cntl->SetFailed(ERESPONSE, "Fail to parse response message, CompressType=%d, size=%zu", meta.compress_type(),
                            res_buf.size());
            saved_error = ERESPONSE;
        }
        if (!saved_error) cntl->set_response_compress_type((CompressType)meta.compress_type());
    }
    if (!device_payload_taken) ReleaseDevicePayload(msg->socket(), meta);
    cntl->_local_side = msg->socket()->local_side();
    msg->Destroy();
    cntl->OnVersionedRPCReturned(cid, saved_error);
}

void RegisterBaiduStdProtocol() {
    Protocol p;
    p.parse = ParseRpcMessage;
    p.serialize_request = SerializeRpcRequest;
    p.pack_request = PackRpcRequest;
    p.process_request = ProcessRpcRequest;
    p.process_response = ProcessRpcResponse;
    p.verify = VerifyRpcRequest;
    p.supported_connection_type = CONNECTION_TYPE_SINGLE | CONNECTION_TYPE_POOLED | CONNECTION_TYPE_SHORT;
    p.name = "baidu_std";
    RegisterProtocol(PROTOCOL_BAIDU_STD, p);
}

}  // namespace policy
}  // namespace mrpc
