#include "rpc/channel.h"

#include "policy/authenticators.h"

#include <cerrno>

#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"
#include "cluster/lb_with_naming.h"
#include "fiber/fiber.h"
#include "gpu/xgmi.h"
#include "rdma/rdma.h"
#include "net/socket_map.h"
#include "rpc/errno.h"
#include "rpc/protocol.h"
#include "rpc/span.h"

namespace mrpc {

ConnectionType StringToConnectionType(const std::string& s) {
    std::string l = to_lower(s);
    if (l == "single") return CONNECTION_TYPE_SINGLE;
    if (l == "pooled") return CONNECTION_TYPE_POOLED;
    if (l == "short") return CONNECTION_TYPE_SHORT;
    return CONNECTION_TYPE_UNKNOWN;
}

const char* ConnectionTypeToString(ConnectionType t) {
    switch (t) {
    case CONNECTION_TYPE_SINGLE: return "single";
    case CONNECTION_TYPE_POOLED: return "pooled";
    case CONNECTION_TYPE_SHORT: return "short";
    default: return "unknown";
    }
}

Channel::Channel() {}

Channel::~Channel() {
    if (_server_id != INVALID_SOCKET_ID && !_lb) {
        SocketMapKey key{_server_address, _map_signature};
        SocketMapRemove(key);
    }
}

int Channel::InitChannelOptions(const ChannelOptions* options) {
    GlobalInitializeOrDie();
    if (options) _options = *options;
    size_t colon = _options.protocol.find(':');
    if (colon != std::string::npos) _protocol_param = _options.protocol.substr(colon + 1);
    _protocol_type = StringToProtocolType(_options.protocol);
    _protocol = FindProtocol(_protocol_type);
    if (!_protocol || !_protocol->support_client()) {
        LOG(ERROR) << "Channel does not support protocol " << _options.protocol;
        return -1;
    }
    // esp connections start with the ESP preamble (reference channel.cpp:222-226)
    if (_protocol_type == PROTOCOL_ESP && !_options.auth) _options.auth = policy::global_esp_authenticator();
    if (!_options.connection_type.empty()) {
        _connection_type = StringToConnectionType(_options.connection_type);
        if (_connection_type == CONNECTION_TYPE_UNKNOWN) {
            LOG(ERROR) << "Unknown connection_type " << _options.connection_type;
            return -1;
        }
        if (!(_protocol->supported_connection_type & _connection_type)) {
            LOG(ERROR) << _protocol->name << " does not support connection type " << _options.connection_type;
            return -1;
        }
    } else {
        _connection_type = (_protocol->supported_connection_type & CONNECTION_TYPE_SINGLE) ? CONNECTION_TYPE_SINGLE
                                                                                          : CONNECTION_TYPE_POOLED;
    }
    // "ssl:<sni>" in the signature makes SocketMap create TLS client sockets.
    // Connections are shared only between channels that would talk the same
    // way: a connection authenticated by one Authenticator must never carry
    // calls of a channel with another (or none).
    _map_signature = string_printf("%s|%s|%s|%d%s|auth:%p", _protocol->name, _options.connection_group.c_str(),
                                   _options.use_ssl ? ("ssl:" + _options.ssl_sni).c_str() : "",
                                   _options.use_device_transport ? _options.gpu_device : -2,
                                   _options.use_rdma ? "|rdma" : "", (const void*)_options.auth);
    if (_options.use_rdma) {
        std::string err;
        if (_options.use_ssl) {
            LOG(ERROR) << "use_rdma and use_ssl are exclusive";
            return -1;
        }
        if (rdma::GlobalRdmaInitialize(&err) != 0) {
            LOG(ERROR) << "Fail to initialise RDMA: " << err;
            return -1;
        }
    }
    if (_options.use_device_transport) {
        std::string err;
        if (gpu::EnableXgmiTransport(_options.gpu_device, &err) != 0) {
            LOG(WARNING) << "xGMI device transport unavailable (" << err
                         << "); device attachments will be staged through host memory";
            _options.use_device_transport = false;
        }
    }
    return 0;
}

int Channel::InitSingle(const EndPoint& ep, const char* raw, const ChannelOptions* options) {
    if (InitChannelOptions(options) != 0) return -1;
    (void)raw;
    _server_address = ep;
    SocketMapKey key{ep, _map_signature};
    if (SocketMapInsert(key, &_server_id) != 0) {
        LOG(ERROR) << "Fail to insert " << ep << " into SocketMap";
        return -1;
    }
    _inited = true;
    return 0;
}

int Channel::Init(const char* server_addr_and_port, const ChannelOptions* options) {
    ChannelOptions opt = options ? *options : ChannelOptions();
    std::string addr = server_addr_and_port;
    // strip scheme for http-like protocols: http://host:port/path
    if (starts_with(addr, "http://") || starts_with(addr, "https://")) {
        bool https = starts_with(addr, "https://");
        addr = addr.substr(https ? 8 : 7);
        size_t slash = addr.find('/');
        if (slash != std::string::npos) addr = addr.substr(0, slash);
        if (addr.find(':') == std::string::npos) addr += https ? ":443" : ":80";
        if (https) opt.use_ssl = true;
    }
    EndPoint ep;
    if (str2endpoint(addr.c_str(), &ep) != 0 && hostname2endpoint(addr.c_str(), &ep) != 0) {
        LOG(ERROR) << "Invalid address `" << server_addr_and_port << "'";
        return -1;
    }
    return InitSingle(ep, server_addr_and_port, &opt);
}

int Channel::Init(const char* server_addr, int port, const ChannelOptions* options) {
    EndPoint ep;
    if (str2endpoint(server_addr, port, &ep) != 0 &&
        hostname2endpoint((std::string(server_addr) + ":" + std::to_string(port)).c_str(), &ep) != 0) {
        LOG(ERROR) << "Invalid address " << server_addr;
        return -1;
    }
    return InitSingle(ep, server_addr, options);
}

int Channel::Init(const EndPoint& server, const ChannelOptions* options) { return InitSingle(server, nullptr, options); }

int Channel::Init(const char* ns_url, const char* lb_name, const ChannelOptions* options) {
    if (!lb_name || !*lb_name) return Init(ns_url, options);
    if (InitChannelOptions(options) != 0) return -1;
    _lb = std::make_shared<LoadBalancerWithNaming>();
    LoadBalancerWithNaming::Options lo;
    lo.socket_signature = _map_signature;
    lo.ns_filter = _options.ns_filter;
    lo.enable_circuit_breaker = _options.enable_circuit_breaker;
    if (_lb->Init(ns_url, lb_name, lo) != 0) {
        LOG(ERROR) << "Fail to init load balancer `" << lb_name << "' with naming service `" << ns_url << "'";
        _lb.reset();
        return -1;
    }
    if (!_options.succeed_without_server && _lb->ServerCount() == 0) {
        LOG(ERROR) << "No server in " << ns_url;
        _lb.reset();
        return -1;
    }
    _inited = true;
    return 0;
}

static void* RunTimeoutError(void* arg) {
    fiber::call_id_error(fiber::CallId{(uint64_t)(uintptr_t)arg}, ERPCTIMEDOUT, "timeout");
    return nullptr;
}
static void HandleTimeout(void* arg) {
    // Never run RPC completion (and user callbacks) in the timer pthread.
    fiber::fiber_t th;
    if (fiber::start_background(&th, nullptr, RunTimeoutError, arg) != 0) RunTimeoutError(arg);
}
static void* RunBackupError(void* arg) {
    fiber::call_id_error(fiber::CallId{(uint64_t)(uintptr_t)arg}, EBACKUPREQUEST, "backup");
    return nullptr;
}
static void HandleBackupRequest(void* arg) {
    fiber::fiber_t th;
    if (fiber::start_background(&th, nullptr, RunBackupError, arg) != 0) RunBackupError(arg);
}

void Channel::CallMethod(const pb::MethodDescriptor* method, RpcController* controller_base,
                         const pb::Message* request, pb::Message* response, Closure* done) {
    Controller* cntl = static_cast<Controller*>(controller_base);
    const int64_t start_real_us = realtime_us();
    cntl->_begin_us = monotonic_us();
    cntl->_begin_real_us = start_real_us;
    if (!_inited) {
        cntl->SetFailed(EINVAL, "Channel is not initialized");
        if (done) done->Run();
        return;
    }
    // canceled before the call (StartCancel on its call_id()): nothing is
    // sent, the call ends with ECANCELED
    if (cntl->Failed() && cntl->ErrorCode() == ECANCELED) {
        if (done) done->Run();
        return;
    }
    // Controller-level settings override the channel's only if set.
    if (cntl->_timeout_ms == Controller::UNSET_MAGIC) cntl->_timeout_ms = _options.timeout_ms;
    if (cntl->_backup_request_ms == Controller::UNSET_MAGIC) cntl->_backup_request_ms = _options.backup_request_ms;
    if (cntl->_max_retry == Controller::UNSET_MAGIC) cntl->_max_retry = _options.max_retry;
    if (cntl->_max_retry < 0) cntl->_max_retry = 0;
    const fiber::CallId cid = cntl->call_id();
    const int rc = fiber::call_id_lock_and_reset_range(cid, nullptr, 2 + cntl->_max_retry);
    if (rc != 0) {
        LOG(ERROR) << "Fail to lock call id (controller reused while in use?)";
        cntl->SetFailed(EINVAL, "controller is in use");
        if (done) done->Run();
        return;
    }
    cntl->_method = method;
    cntl->_response = response;
    cntl->_done = done;
    cntl->_protocol = _protocol;
    cntl->_protocol_type = _protocol_type;
    if (!_protocol_param.empty()) cntl->_protocol_param = _protocol_param;
    cntl->_use_device_transport = _options.use_device_transport;
    cntl->_auth = _options.auth;
    if (cntl->_connection_type == CONNECTION_TYPE_SINGLE) cntl->_connection_type = _connection_type;
    if (!cntl->_retry_policy) cntl->_retry_policy = _options.retry_policy;
    cntl->_enable_circuit_breaker = _options.enable_circuit_breaker;
    if (_lb) {
        cntl->_lb = _lb->lb();
        cntl->_lb_holder = _lb;
        cntl->_single_server_id = INVALID_SOCKET_ID;
    } else {
        cntl->_single_server_id = _server_id;
        cntl->_remote_side = _server_address;
    }
    if (IsRpczEnabled() && !cntl->_span && method) {
        cntl->_span = Span::CreateClientSpan(method->full_name, start_real_us);
        if (cntl->_span) {
            cntl->_trace_id = cntl->_span->trace_id;
            cntl->_span_id = cntl->_span->span_id;
            cntl->_parent_span_id = cntl->_span->parent_span_id;
        }
    }
    cntl->_request_buf.clear();
    _protocol->serialize_request(&cntl->_request_buf, cntl, request);
    if (cntl->Failed()) {
        cntl->HandleSendFailed();
        return;
    }
    if (cntl->_span) cntl->_span->request_size = (int64_t)cntl->_request_buf.size();
    if (cntl->_timeout_ms >= 0) {
        fiber::timer_add_us(&cntl->_timeout_id, cntl->_timeout_ms * 1000, HandleTimeout, (void*)(uintptr_t)cid.value);
        cntl->_deadline_us = cntl->_begin_us + cntl->_timeout_ms * 1000;
    }
    if (cntl->_backup_request_ms >= 0 && (cntl->_timeout_ms < 0 || cntl->_backup_request_ms < cntl->_timeout_ms)) {
        fiber::timer_add_us(&cntl->_backup_id, cntl->_backup_request_ms * 1000, HandleBackupRequest,
                            (void*)(uintptr_t)cid.value);
    }
    cntl->IssueRPC(cntl->_begin_us);  // the first try starts with the call
    if (!done) fiber::call_id_join(cid);
}

int Channel::CheckHealth() {
    if (_lb) return _lb->ServerCount() > 0 ? 0 : -1;
    SocketUniquePtr s;
    return Socket::Address(_server_id, &s) == 0 ? 0 : -1;
}

std::string Channel::Describe() const {
    if (_lb) return string_printf("Channel{lb=%s protocol=%s}", _lb->Describe().c_str(), _protocol ? _protocol->name : "");
    return string_printf("Channel{%s protocol=%s conn=%s}", _server_address.to_string().c_str(),
                         _protocol ? _protocol->name : "", ConnectionTypeToString(_connection_type));
}

}  // namespace mrpc
