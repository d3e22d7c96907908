// Channel: the client endpoint (role of src/brpc/channel.h:41-140,
// channel.cpp:317-587). Single-server mode shares the connection through
// SocketMap; naming-service mode resolves "scheme://name" into servers fed
// to a load balancer.
#pragma once

#include <memory>
#include <string>

#include "base/endpoint.h"
#include "mrpc/proto/options.pb.h"
#include "pb/service.h"
#include "rpc/authenticator.h"
#include "rpc/controller.h"
#include "rpc/retry_policy.h"

namespace mrpc {

class LoadBalancerWithNaming;
class NamingServiceFilter;

struct ChannelOptions {
    int32_t connect_timeout_ms = 200;
    int32_t timeout_ms = 500;       // -1: no timeout
    int32_t backup_request_ms = -1;
    int max_retry = 3;
    // "baidu_std", "http", "h2", "h2:grpc", "streaming_rpc", "redis", "memcache", ...
    std::string protocol = "baidu_std";
    // "single", "pooled", "short" (empty = protocol default)
    std::string connection_type;
    bool succeed_without_server = true;
    const Authenticator* auth = nullptr;
    const RetryPolicy* retry_policy = nullptr;
    const NamingServiceFilter* ns_filter = nullptr;
    std::string connection_group;  // separates connection pools
    bool enable_circuit_breaker = false;
    // MI355X: move DEVICE attachment blocks over the xGMI transport.
    bool use_device_transport = false;
    int gpu_device = -1;  // local GPU for device transport (-1 = current)
    // SSL: verify nothing, just encrypt when true (ChannelSSLOptions analog)
    bool use_ssl = false;
    std::string ssl_sni;
    // Move every byte of the connection over RDMA verbs after a TCP hello
    // exchange (rdma/rdma.h); the server must enable ServerOptions.use_rdma.
    bool use_rdma = false;
};

class ChannelBase : public RpcChannel {
public:
    virtual int Weight() { return 0; }
    virtual int CheckHealth() = 0;
};

class Channel : public ChannelBase {
public:
    Channel();
    ~Channel() override;
    // "ip:port", "host:port", "unix:/path", or protocol-specific ("http://h:p")
    int Init(const char* server_addr_and_port, const ChannelOptions* options);
    int Init(const char* server_addr, int port, const ChannelOptions* options);
    int Init(const EndPoint& server, const ChannelOptions* options);
    // "list://a:1,b:2", "file://path", "http://domain:port" (dns), ... + lb name
    int Init(const char* naming_service_url, const char* load_balancer_name, const ChannelOptions* options);

    void CallMethod(const pb::MethodDescriptor* method, RpcController* controller, const pb::Message* request,
                    pb::Message* response, Closure* done) override;
    int CheckHealth() override;
    const ChannelOptions& options() const { return _options; }
    ProtocolType protocol_type() const { return _protocol_type; }
    bool SingleServer() const { return _lb == nullptr; }
    SocketId server_id() const { return _server_id; }
    const EndPoint& server_address() const { return _server_address; }
    std::string Describe() const;

protected:
    int InitChannelOptions(const ChannelOptions* options);
    int InitSingle(const EndPoint& ep, const char* raw_address, const ChannelOptions* options);

    ChannelOptions _options;
    ProtocolType _protocol_type = PROTOCOL_BAIDU_STD;
    std::string _protocol_param;
    const struct Protocol* _protocol = nullptr;
    ConnectionType _connection_type = CONNECTION_TYPE_SINGLE;
    EndPoint _server_address;
    SocketId _server_id = INVALID_SOCKET_ID;
    std::string _map_signature;
    std::shared_ptr<LoadBalancerWithNaming> _lb;
    bool _inited = false;
};

// Parse "single"/"pooled"/"short".
ConnectionType StringToConnectionType(const std::string& s);
const char* ConnectionTypeToString(ConnectionType t);

}  // namespace mrpc
