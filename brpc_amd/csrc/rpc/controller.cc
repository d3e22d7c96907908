#include "rpc/controller.h"
#include "rpc/stream_internal.h"

#include <cerrno>
#include <cstdarg>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"
#include "cluster/circuit_breaker.h"
#include "cluster/load_balancer.h"
#include "fiber/fiber.h"
#include "http/http_header.h"
#include "http/http_message.h"
#include "rpc/progressive.h"
#include "rpc/errno.h"
#include "rpc/protocol.h"
#include "rpc/retry_policy.h"
#include "rpc/server.h"
#include "rpc/span.h"
#include "policy/device_payload.h"

DEFINE_int32(device_hello_wait_ms, 200,
             "requests with device payloads wait at most this long for the connection's transport negotiation "
             "(another request's hello round trip) before staging their payloads inline");

namespace mrpc {

const IdlNames idl_single_req_single_res = {"req", "res"};
const IdlNames idl_single_req_multi_res = {"req", ""};
const IdlNames idl_multi_req_single_res = {"", "res"};
const IdlNames idl_multi_req_multi_res = {"", ""};

Controller::Controller() {}

Controller::~Controller() {
    ResetNonPods();
}

void Controller::ResetNonPods() {
    if (_correlation_id.value) {
        // A finished RPC already destroyed the id; an unused one must be cancelled.
        fiber::call_id_cancel(_correlation_id);
    }
    if (_timeout_id) fiber::timer_del(_timeout_id);
    if (_backup_id) fiber::timer_del(_backup_id);
    delete _accessed;
    _accessed = nullptr;
    delete _http_request;
    _http_request = nullptr;
    delete _http_response;
    _http_response = nullptr;
    if (_session_local_data && _server) _server->ReturnSessionLocalData(_session_local_data);
    _session_local_data = nullptr;
    if (_span) {
        Span::Submit(_span, _end_us ? _end_us : monotonic_us());
        _span = nullptr;
    }
}

void Controller::Reset() {
    ResetNonPods();
    _method = nullptr;
    _response = nullptr;
    _done = nullptr;
    _protocol = nullptr;
    _single_server_id = INVALID_SOCKET_ID;
    _lb = nullptr;
    _lb_holder.reset();
    _auth = nullptr;
    _request_buf.clear();
    _request_attachment.clear();
    _response_attachment.clear();
    _error_code = 0;
    _error_text.clear();
    _timeout_ms = UNSET_MAGIC;
    _backup_request_ms = UNSET_MAGIC;
    _max_retry = UNSET_MAGIC;
    _nretry = 0;
    _has_backup = false;
    _retry_policy = nullptr;
    _connection_type = CONNECTION_TYPE_SINGLE;
    _request_compress_type = COMPRESS_TYPE_NONE;
    _response_compress_type = COMPRESS_TYPE_NONE;
    _log_id = 0;
    _has_log_id = false;
    _request_code = 0;
    _has_request_code = false;
    _request_id.clear();
    _correlation_id = fiber::CallId{0};
    _ended_id = fiber::CallId{0};
    _timeout_id = 0;
    _backup_id = 0;
    _begin_us = _begin_real_us = _end_us = 0;
    _deadline_us = -1;
    _current_call.Reset();
    _unfinished_call.Reset();
    _remote_side = EndPoint();
    _local_side = EndPoint();
    _canceled = false;
    _cancel_callback = nullptr;
    _span_enabled = false;
    _trace_id = _span_id = _parent_span_id = 0;
    _verify_device_payload = false;
    _device_payload_compress = COMPRESS_TYPE_NONE;
    _device_payload_scan = false;
    _received_device_compress = COMPRESS_TYPE_NONE;
    _device_payload_index.nfields = -1;
    _device_payload_index.fields.clear();
    _read_progressively = false;
    _progressive_reader = nullptr;
    _progressive_attachment.reset();
    _progressive_sink.reset();
    _pipelined_count = 0;
    _auth_replies = 0;
    _auth_winner = false;
    _pipelined_tag = 0;
    _idl_names = idl_single_req_single_res;
    _idl_result = IDL_VOID_RESULT;
    _use_device_transport = false;
    _reply_xgmi_hello = false;
    _reply_plane_hello = false;
    _session_kv.clear();
    _request_stream = _response_stream = 0;
    _stream_creator.reset();
    _server = nullptr;
    _method_status = nullptr;
    _server_socket_id = INVALID_SOCKET_ID;
    _server_correlation_id = 0;
    _close_connection = false;
    _on_end = nullptr;
    _received_us = 0;
}

void Controller::SetFailed(const std::string& reason) {
    if (_error_code == 0) _error_code = EINTERNAL;
    if (!_error_text.empty()) _error_text += "; ";
    _error_text += reason;
}

void Controller::SetFailed(int error_code, const char* fmt, ...) {
    if (error_code == 0) error_code = EINTERNAL;
    _error_code = error_code;
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (!_error_text.empty()) _error_text += "; ";
    string_appendf(&_error_text, "[E%d]%s", error_code, buf);
}

fiber::CallId Controller::call_id() {
    // after the call ended, the same (now destroyed) id: StartCancel on it
    // does nothing, as in the reference, instead of failing a finished call
    if (_correlation_id.value == 0 && _ended_id.value != 0) return _ended_id;
    if (_correlation_id.value == 0) {
        if (fiber::call_id_create(&_correlation_id, this, HandleError) != 0) {
            LOG(FATAL) << "Fail to create call id";
        }
    }
    return _correlation_id;
}

void Controller::Join() {
    // EndRPC may clear the id concurrently (async calls joined by the user)
    const fiber::CallId cid{__atomic_load_n(&_correlation_id.value, __ATOMIC_ACQUIRE)};
    if (cid.value) fiber::call_id_join(cid);
}

void Controller::CloseConnection(const char* reason) {
    _close_connection = true;
    (void)reason;
}

bool Controller::IsAskedToQuit() const {
    if (_server_socket_id == INVALID_SOCKET_ID) return false;
    SocketUniquePtr s;
    return Socket::Address(_server_socket_id, &s) != 0;
}

HttpHeader& Controller::http_request() {
    if (!_http_request) _http_request = new HttpHeader;
    return *_http_request;
}

HttpHeader& Controller::http_response() {
    if (!_http_response) _http_response = new HttpHeader;
    return *_http_response;
}

std::shared_ptr<ProgressiveAttachment> Controller::CreateProgressiveAttachment() {
    if (!_progressive_attachment) {
        const bool http10 = _http_request && _http_request->major_version() == 1 && _http_request->minor_version() == 0;
        _progressive_attachment = std::make_shared<ProgressiveAttachment>(_server_socket_id, http10);
    }
    return _progressive_attachment;
}

void Controller::ReadProgressiveAttachmentBy(ProgressiveReader* r) {
    if (!r) return;
    if (!_progressive_sink) {
        r->OnEndOfMessage(Status(EINVAL, _read_progressively ? "response has no progressive body"
                                                             : "call response_will_be_read_progressively() first"));
        return;
    }
    _progressive_sink->SetReader(r);
}

void Controller::StartCancel() {
    if (_canceled.exchange(true)) return;
    const fiber::CallId cid{__atomic_load_n(&_correlation_id.value, __ATOMIC_ACQUIRE)};
    if (cid.value) fiber::call_id_error(cid, ECANCELED, "canceled");
    Closure* cb = _cancel_callback;
    _cancel_callback = nullptr;
    if (cb) cb->Run();
}

void StartCancel(fiber::CallId id) { fiber::call_id_error(id, ECANCELED, "canceled"); }

void Controller::NotifyOnCancel(Closure* callback) {
    if (_canceled.load()) {
        callback->Run();
        return;
    }
    _cancel_callback = callback;
}

// ----------------------------------------------------------------- engine

int Controller::HandleError(fiber::CallId id, void* data, int error_code, const std::string& error_text) {
    Controller* c = static_cast<Controller*>(data);
    if (error_code == ERPCTIMEDOUT) {
        c->SetFailed(ERPCTIMEDOUT, "reached timeout=%lldms @%s", (long long)c->_timeout_ms,
                     c->_remote_side.to_string().c_str());
        c->EndRPC(c->_current_call.id);
        return 0;
    }
    if (error_code == ECANCELED) {
        c->SetFailed(ECANCELED, "RPC canceled");
        c->EndRPC(c->_current_call.id);
        return 0;
    }
    if (error_code == EBACKUPREQUEST) {
        c->_backup_id = 0;
        if (c->_nretry >= c->_max_retry || c->_unfinished_call.id.value != 0) {
            fiber::call_id_unlock(id);
            return 0;
        }
        // Keep the in-flight attempt as "unfinished" and send a duplicate to
        // another server; the first response wins.
        c->_unfinished_call.id = c->_current_call.id;
        c->_unfinished_call.peer_id = c->_current_call.peer_id;
        c->_unfinished_call.sending_sock = std::move(c->_current_call.sending_sock);
        c->_unfinished_call.begin_us = c->_current_call.begin_us;
        c->_unfinished_call.need_feedback = c->_current_call.need_feedback;
        if (!c->_accessed) c->_accessed = new ExcludedServers;
        c->_accessed->Add(c->_current_call.peer_id);
        ++c->_nretry;
        c->_has_backup = true;
        c->IssueRPC(monotonic_us());
        return 0;
    }
    if (id != c->_current_call.id && id != c->_unfinished_call.id) {
        fiber::call_id_unlock(id);  // error of an obsolete attempt
        return 0;
    }
    if (id == c->_current_call.id) {
        c->_error_code = 0;  // replace the error of the attempt
        c->_error_text.clear();
        c->SetFailed(error_code, "%s", error_text.c_str());
    }
    c->OnVersionedRPCReturned(id, error_code);
    return 0;
}

void Controller::OnVersionedRPCReturned(fiber::CallId id, int error_code) {
    if (id != _current_call.id && id != _unfinished_call.id) {
        fiber::call_id_unlock(_correlation_id);
        return;
    }
    if (error_code == 0) {
        EndRPC(id);
        return;
    }
    if (id != _current_call.id) {
        // The original attempt of a backup request failed; keep waiting.
        OnCallComplete(&_unfinished_call, error_code, false);
        _unfinished_call.Reset();
        fiber::call_id_unlock(_correlation_id);
        return;
    }
    const RetryPolicy* rp = _retry_policy ? _retry_policy : DefaultRetryPolicy();
    if (_nretry < _max_retry && !_canceled.load() && rp->DoRetry(this)) {
        OnCallComplete(&_current_call, error_code, false);
        if (!_accessed) _accessed = new ExcludedServers;
        _accessed->Add(_current_call.peer_id);
        ++_nretry;
        _error_code = 0;
        _error_text.clear();
        IssueRPC(monotonic_us());
        return;
    }
    EndRPC(id);
}

void Controller::OnCallComplete(Call* c, int error_code, bool responded) {
    if (c->id.value == 0) return;
    if (_enable_circuit_breaker && c->peer_id != INVALID_SOCKET_ID && error_code != ECANCELED) {
        FeedCircuitBreaker(c->peer_id, error_code, monotonic_us() - c->begin_us);
    }
    if (c->need_feedback && _lb) {
        LoadBalancer::CallInfo info;
        info.begin_time_us = c->begin_us;
        info.server_id = c->peer_id;
        info.error_code = error_code;
        info.controller = this;
        _lb->Feedback(info);
    }
    if (c->sending_sock) {
        if (_connection_type == CONNECTION_TYPE_POOLED && responded && error_code == 0 && _progressive_sink &&
            !_progressive_sink->body_done()) {
            // the body still streams over this connection: it rejoins the
            // pool when the body is done, not with the response head
            const SocketId sid = c->sending_sock->id();
            _progressive_sink->SetOnBodyDone([sid] {
                SocketUniquePtr s;
                if (Socket::Address(sid, &s) == 0) s->ReturnToPool();
            });
        } else if (_connection_type == CONNECTION_TYPE_POOLED && responded && error_code == 0) {
            c->sending_sock->ReturnToPool();
        } else if (_connection_type == CONNECTION_TYPE_POOLED || _connection_type == CONNECTION_TYPE_SHORT) {
            c->sending_sock->SetFailed(EUNUSED, "short/pooled connection done");
        }
        c->sending_sock.reset();
    }
}

void Controller::EndRPC(fiber::CallId id) {
    if (_timeout_id) {
        fiber::timer_del(_timeout_id);
        _timeout_id = 0;
    }
    if (_backup_id) {
        fiber::timer_del(_backup_id);
        _backup_id = 0;
    }
    const bool responded = (_error_code == 0);
    if (id == _current_call.id) {
        OnCallComplete(&_current_call, _error_code, responded);
        OnCallComplete(&_unfinished_call, ECANCELED, false);
    } else {
        OnCallComplete(&_unfinished_call, _error_code, responded);
        OnCallComplete(&_current_call, ECANCELED, false);
    }
    _end_us = monotonic_us();
    if (_request_stream != INVALID_STREAM_ID) OnRequestStreamCallEnded(_request_stream);
    if (_span) Span::EndClientSpan(_span, this);
    if (_on_end) _on_end(this);
    Closure* done = _done;
    _done = nullptr;
    const fiber::CallId cid = _correlation_id;
    _ended_id = cid;
    __atomic_store_n(&_correlation_id.value, 0, __ATOMIC_RELEASE);  // pairs with Join()
    // After this, a sync caller may destroy *this.
    fiber::call_id_unlock_and_destroy(cid);
    if (done) done->Run();
}

void Controller::IssueRPC(int64_t begin_us) {
    const fiber::CallId cid = fiber::call_id_with_version(_correlation_id, 1 + _nretry);
    _current_call.Reset();
    _current_call.id = cid;
    _current_call.begin_us = begin_us;
    SocketUniquePtr tmp;
    if (_single_server_id != INVALID_SOCKET_ID) {
        if (Socket::Address(_single_server_id, &tmp) != 0) {
            fiber::call_id_unlock(_correlation_id);
            fiber::call_id_error(cid, EHOSTDOWN, "server " + _remote_side.to_string() + " is down");
            return;
        }
        _current_call.peer_id = _single_server_id;
    } else if (_lb) {
        LoadBalancer::SelectIn in;
        in.begin_time_us = _current_call.begin_us;
        in.has_request_code = _has_request_code;
        in.request_code = _request_code;
        in.excluded = _accessed;
        LoadBalancer::SelectOut out;
        out.ptr = &tmp;
        const int rc = _lb->SelectServer(in, &out);
        if (rc != 0 || !tmp) {
            fiber::call_id_unlock(_correlation_id);
            if (rc == EREJECT) {
                fiber::call_id_error(cid, EREJECT, "rejected by the cluster recover policy");
            } else {
                fiber::call_id_error(cid, EHOSTDOWN, "no server available");
            }
            return;
        }
        _current_call.need_feedback = out.need_feedback;
        _current_call.peer_id = tmp->id();
    } else {
        fiber::call_id_unlock(_correlation_id);
        fiber::call_id_error(cid, EINTERNAL, "channel has no server");
        return;
    }
    _remote_side = tmp->remote_side();
    Socket* sock = tmp.get();
    if (_connection_type == CONNECTION_TYPE_POOLED) {
        if (tmp->GetPooledSocket(&_current_call.sending_sock) != 0) {
            fiber::call_id_unlock(_correlation_id);
            fiber::call_id_error(cid, EFAILEDSOCKET, "fail to get pooled connection");
            return;
        }
        sock = _current_call.sending_sock.get();
    } else if (_connection_type == CONNECTION_TYPE_SHORT) {
        if (tmp->GetShortSocket(&_current_call.sending_sock) != 0) {
            fiber::call_id_unlock(_correlation_id);
            fiber::call_id_error(cid, EFAILEDSOCKET, "fail to create short connection");
            return;
        }
        sock = _current_call.sending_sock.get();
    }
    Buf packet;
    _pack_socket = sock;
    _auth_replies = 0;
    _auth_winner = false;
    // Credentials ride on the FIRST request of a connection only: the
    // first writer wins the socket's authentication fight and packs them;
    // the others wait until its write is queued, so the credentials are
    // first on the wire (reference: controller.cpp IssueRPC +
    // socket.cpp:1999-2035).
    const Authenticator* auth = nullptr;
    if (_auth) {
        int auth_error = 0;
        if (sock->FightAuthentication(&auth_error)) {
            auth = _auth;
            _auth_winner = true;
        } else if (auth_error != 0) {
            fiber::call_id_unlock(_correlation_id);
            fiber::call_id_error(cid, ERPCAUTH, "fail to authenticate the connection: " +
                                                    std::string(::mrpc::ErrorText(auth_error)));
            return;
        }
    }
    // Device payloads on a connection whose transports are not negotiated
    // yet: one request negotiates, the others wait for its answer.
    bool hello_negotiator = false;
    if (_use_device_transport && !sock->transport() && sock->plane_rank() == Socket::kPlaneUnknown &&
        !_request_attachment.all_host_accessible()) {
        hello_negotiator = sock->FightDeviceHello((int64_t)FLAGS_device_hello_wait_ms * 1000);
    }
    _protocol->pack_request(&packet, cid.value, _method, this, _request_buf, auth);
    _pack_socket = nullptr;
    if (_error_code != 0) {
        if (_auth_winner) sock->ResetAuthentication();
        if (hello_negotiator) sock->DeviceHelloAbandoned();
        const int ec = _error_code;
        const std::string et = _error_text;
        fiber::call_id_unlock(_correlation_id);
        fiber::call_id_error(cid, ec, et);
        return;
    }
    WriteOptions wopt;
    wopt.id_wait = cid;
    wopt.pipelined_count = _pipelined_count;
    wopt.pipelined_tag = _pipelined_tag;
    wopt.pipelined_protocol = (int)_protocol_type;
    wopt.auth_replies = _auth_replies;
    wopt.auth_winner = _auth_winner;
    // Errors of Write() are delivered through call_id_error(cid), which is
    // queued while we hold the lock and handled at unlock.
    if (sock->Write(&packet, &wopt) != 0) {
        // refused (overcrowded / failed socket): the peer never sees the
        // meta, so give back the lent blocks and withdraw plane payloads
        if (_packed_payloads && _packed_payloads->descs.size() > 0) policy::CancelDeviceBlocks(_packed_payloads->descs);
        if (hello_negotiator) sock->DeviceHelloAbandoned();
    }
    if (_packed_payloads) _packed_payloads->descs.Clear();
    if (_span) _span->sent_real_us = realtime_us();
    fiber::call_id_unlock(cid);
}

}  // namespace mrpc
