// Controller: per-RPC state for client and server (role of
// src/brpc/controller.h / controller.cpp:555-1003).
//
// Client engine: one CallId per RPC with a range of versions, one version
// per attempt (first try, retries, backup request). Responses, socket
// failures, timeouts and backup timers all arrive as "errors"/unlocks on
// that id; OnVersionedRPCReturned() decides retry / backup / end, and stale
// versions are dropped, which is how retries and backups de-duplicate.
#pragma once

#include <atomic>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <string>

#include "base/buf.h"
#include "base/endpoint.h"
#include "fiber/call_id.h"
#include "mrpc/proto/options.pb.h"
#include "net/socket.h"
#include "pb/service.h"
#include "policy/device_payload.h"

namespace mrpc {

class Server;
class Channel;
class LoadBalancer;
class RetryPolicy;
class Authenticator;
class ExcludedServers;
class MethodStatus;
class Span;
class HttpHeader;
class ProgressiveAttachment;
class ProgressiveReader;
class ProgressiveSink;
class StreamCreator;
class MongoContext;
struct Protocol;
namespace policy {
struct PackedPayloads;
}  // namespace policy
typedef uint64_t StreamId;

// Server-side per-connection / per-call user data factory hooks.
class DataFactory {
public:
    virtual ~DataFactory() {}
    virtual void* CreateData() const = 0;
    virtual void DestroyData(void* d) const = 0;
};

// Names wrapping the request/response inside ubrpc's params/result_params
// objects (reference controller.h:86-94).
struct IdlNames {
    const char* request_name;   // must be a string constant
    const char* response_name;
};
extern const IdlNames idl_single_req_single_res;  // {"req", "res"} (default)
extern const IdlNames idl_single_req_multi_res;   // {"req", ""}
extern const IdlNames idl_multi_req_single_res;   // {"", "res"}
extern const IdlNames idl_multi_req_multi_res;    // {"", ""}
static const int64_t IDL_VOID_RESULT = 12345678987654321LL;

class Controller : public RpcController {
public:
    Controller();
    ~Controller() override;
    Controller(const Controller&) = delete;
    Controller& operator=(const Controller&) = delete;

    // ---------------- client-side settings
    void set_timeout_ms(int64_t ms) { _timeout_ms = ms; }
    int64_t timeout_ms() const { return _timeout_ms; }
    void set_backup_request_ms(int64_t ms) { _backup_request_ms = ms; }
    int64_t backup_request_ms() const { return _backup_request_ms; }
    void set_max_retry(int n) { _max_retry = n; }
    int max_retry() const { return _max_retry; }
    void set_log_id(uint64_t id) { _log_id = id; _has_log_id = true; }
    uint64_t log_id() const { return _log_id; }
    void set_request_code(uint64_t c) { _request_code = c; _has_request_code = true; }
    bool has_request_code() const { return _has_request_code; }
    uint64_t request_code() const { return _request_code; }
    void set_request_compress_type(CompressType t) { _request_compress_type = t; }
    CompressType request_compress_type() const { return _request_compress_type; }
    void set_response_compress_type(CompressType t) { _response_compress_type = t; }
    CompressType response_compress_type() const { return _response_compress_type; }
    void set_connection_type(ConnectionType t) { _connection_type = t; }
    ConnectionType connection_type() const { return _connection_type; }
    void set_request_id(const std::string& s) { _request_id = s; }
    const std::string& request_id() const { return _request_id; }
    void set_retry_policy(const RetryPolicy* p) { _retry_policy = p; }
    // Called by the channel on the caller's fiber/thread before issuing.
    void set_span_enabled(bool on) { _span_enabled = on; }

    Buf& request_attachment() { return _request_attachment; }
    Buf& response_attachment() { return _response_attachment; }
    const Buf& request_attachment() const { return _request_attachment; }
    const Buf& response_attachment() const { return _response_attachment; }

    // ---------------- results
    bool Failed() const override { return _error_code != 0; }
    // Server side: the request carries a stream the handler may StreamAccept.
    bool has_remote_stream() const { return _request_stream != 0; }
    int ErrorCode() const { return _error_code; }
    std::string ErrorText() const override { return _error_text; }
    void SetFailed(const std::string& reason) override;
    void SetFailed(int error_code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
    int64_t latency_us() const { return _end_us > _begin_us ? _end_us - _begin_us : 0; }
    const EndPoint& remote_side() const { return _remote_side; }
    const EndPoint& local_side() const { return _local_side; }
    int retried_count() const { return _nretry; }
    bool has_backup_request() const { return _has_backup; }
    bool is_server_side() const { return _server != nullptr; }
    void Reset() override;
    fiber::CallId call_id();  // correlation id (creates it on first use)
    // the id of the call in flight, 0 once it ended; safe to read while the
    // call ends on another thread (no id is created)
    fiber::CallId inflight_call_id() const {
        return fiber::CallId{__atomic_load_n(&_correlation_id.value, __ATOMIC_ACQUIRE)};
    }
    void Join();              // wait for an async RPC to finish

    // ---------------- cancellation
    void StartCancel() override;
    bool IsCanceled() const override { return _canceled.load(); }
    void NotifyOnCancel(Closure* callback) override;

    // ---------------- server side
    const Server* server() const { return _server; }
    bool IsCloseConnection() const { return _close_connection; }
    void CloseConnection(const char* reason);
    void* session_local_data();
    // true when the client asked the call to stop (socket failed)
    bool IsAskedToQuit() const;
    int64_t server_deadline_us() const { return _deadline_us; }

    // ---------------- http (filled by http/h2 protocols)
    HttpHeader& http_request();
    HttpHeader& http_response();
    bool has_http_request() const { return _http_request != nullptr; }
    // Progressive (chunked) response for server push: keep the returned
    // object and Write() body pieces after done->Run(); dropping the last
    // reference ends the body.
    std::shared_ptr<ProgressiveAttachment> CreateProgressiveAttachment();
    bool has_progressive_attachment() const { return (bool)_progressive_attachment; }
    void ReadProgressiveAttachmentBy(ProgressiveReader* r);
    void response_will_be_read_progressively() { _read_progressively = true; }
    bool is_response_read_progressively() const { return _read_progressively; }

    // ---------------- ubrpc (mcpack/compack idl) naming and result
    void set_idl_names(const IdlNames& n) { _idl_names = n; }
    IdlNames idl_names() const { return _idl_names; }
    void set_idl_result(int64_t r) { _idl_result = r; }
    int64_t idl_result() const { return _idl_result; }

    // ---------------- mongo: per-connection context of a mongo server call
    MongoContext* mongo_session_data() const { return _mongo_session_data.get(); }
    std::shared_ptr<MongoContext> _mongo_session_data;

    // ---------------- kv log for server logging (SessionKV)
    Controller& LogKV(const std::string& k, const std::string& v) {
        _session_kv[k] = v;
        return *this;
    }
    const std::map<std::string, std::string>& session_kv() const { return _session_kv; }

    // ---------------- tracing
    uint64_t trace_id() const { return _trace_id; }
    uint64_t span_id() const { return _span_id; }
    Span* span() const { return _span; }

    // ---------------- GPU payloads (MI355X): device-resident attachments
    // A request/response attachment whose blocks are DEVICE memory travels
    // over the socket's xGMI transport (RpcMeta.device_payload) instead of
    // the TCP byte stream. The receiver sees DEVICE/PEER blocks in its
    // attachment. device_payload_crc: set by the sender to request on-device
    // checksum verification.
    void set_verify_device_payload(bool on) { _verify_device_payload = on; }
    bool verify_device_payload() const { return _verify_device_payload; }
    // Device-side compression of the device blocks this side sends (request
    // attachment on a client, response attachment on a server): with
    // COMPRESS_TYPE_SNAPPY each lent block of at least
    // -device_payload_compress_min_bytes is snappy-encoded in HBM by the
    // batched codec kernels and the receiver decodes it straight out of the
    // lent region into its own HBM — the bytes never reach the host
    // (reference analog: the body codec of src/brpc/compress.cpp:79-92,
    // moved onto the device payload). Incompressible blocks are lent raw.
    void set_device_payload_compress_type(CompressType t) { _device_payload_compress = t; }
    CompressType device_payload_compress_type() const { return _device_payload_compress; }
    // The device attachment this side sends is ONE serialized protobuf
    // message: the receiver indexes its top-level fields on the device
    // (pb_scan) and finds the table in device_payload_index().
    void set_device_payload_scan(bool on) { _device_payload_scan = on; }
    bool device_payload_scan() const { return _device_payload_scan; }
    // What arrived: the field table of a received pb_scan payload, and the
    // device compression the peer used (COMPRESS_TYPE_NONE: lent raw). The
    // table exists only for payloads that came over the device transport: a
    // payload staged inline over TCP (no transport yet, or a busy lender)
    // arrives as host bytes with nfields = -1, for the host parser.
    const DevicePayloadIndex& device_payload_index() const { return _device_payload_index; }
    CompressType received_device_payload_compress_type() const { return _received_device_compress; }

    // ================= internal (protocols / channels) =================
    struct Call {
        fiber::CallId id{0};          // attempt id (base + version)
        SocketId peer_id = INVALID_SOCKET_ID;
        SocketUniquePtr sending_sock;  // pooled/short socket if any
        int64_t begin_us = 0;
        bool need_feedback = false;
        bool touched_by_stream_creator = false;
        void Reset() {
            id = fiber::CallId{0};
            peer_id = INVALID_SOCKET_ID;
            sending_sock.reset();
            begin_us = 0;
            need_feedback = false;
        }
    };
    // set by Channel::CallMethod
    const pb::MethodDescriptor* _method = nullptr;
    pb::Message* _response = nullptr;
    Closure* _done = nullptr;
    const Protocol* _protocol = nullptr;
    ProtocolType _protocol_type = PROTOCOL_BAIDU_STD;
    SocketId _single_server_id = INVALID_SOCKET_ID;
    LoadBalancer* _lb = nullptr;  // not owned
    std::shared_ptr<void> _lb_holder;  // keeps the LB alive during the call
    const Authenticator* _auth = nullptr;
    Buf _request_buf;  // serialized request
    Buf _request_attachment;
    Buf _response_attachment;
    static const int UNSET_MAGIC = -123456789;
    int _error_code = 0;
    std::string _error_text;
    int64_t _timeout_ms = UNSET_MAGIC;
    int64_t _backup_request_ms = UNSET_MAGIC;
    int64_t _connect_timeout_ms = 200;
    int _max_retry = UNSET_MAGIC;
    int _nretry = 0;
    bool _has_backup = false;
    const RetryPolicy* _retry_policy = nullptr;
    ConnectionType _connection_type = CONNECTION_TYPE_SINGLE;
    CompressType _request_compress_type = COMPRESS_TYPE_NONE;
    CompressType _response_compress_type = COMPRESS_TYPE_NONE;
    uint64_t _log_id = 0;
    bool _has_log_id = false;
    uint64_t _request_code = 0;
    bool _has_request_code = false;
    std::string _request_id;
    fiber::CallId _correlation_id{0};
    fiber::CallId _ended_id{0};  // the id of the finished call: call_id() keeps naming it (cancels are no-ops)
    fiber::TimerId _timeout_id = 0;
    fiber::TimerId _backup_id = 0;
    int64_t _begin_us = 0;
    int64_t _begin_real_us = 0;
    int64_t _end_us = 0;
    int64_t _deadline_us = -1;
    Call _current_call;
    Call _unfinished_call;
    ExcludedServers* _accessed = nullptr;
    Socket* _pack_socket = nullptr;  // socket being packed for (valid during pack_request)
    bool _enable_circuit_breaker = false;
    EndPoint _remote_side;
    EndPoint _local_side;
    std::atomic<bool> _canceled{false};
    Closure* _cancel_callback = nullptr;
    bool _span_enabled = false;
    Span* _span = nullptr;
    uint64_t _trace_id = 0, _span_id = 0, _parent_span_id = 0;
    bool _verify_device_payload = false;
    CompressType _device_payload_compress = COMPRESS_TYPE_NONE;
    bool _device_payload_scan = false;
    CompressType _received_device_compress = COMPRESS_TYPE_NONE;
    DevicePayloadIndex _device_payload_index;
    // device payloads described in the request being written (lent blocks,
    // RCCL plane sequences): cancelled when the write is refused, since the
    // receiver will never see their meta
    std::unique_ptr<policy::PackedPayloads> _packed_payloads;
    bool _read_progressively = false;
    ProgressiveReader* _progressive_reader = nullptr;
    std::shared_ptr<ProgressiveAttachment> _progressive_attachment;
    std::shared_ptr<ProgressiveSink> _progressive_sink;  // client: streamed response body
    // set by pack_request of in-order protocols (http/1.1, redis, memcache)
    int _pipelined_count = 0;
    int _auth_replies = 0;       // replies to credentials packed in front (redis AUTH/SELECT)
    bool _auth_winner = false;   // this write carries the connection's credentials
    uint32_t _pipelined_tag = 0;
    std::string _protocol_param;  // "grpc" for channels of protocol "h2:grpc"
    IdlNames _idl_names = {"req", "res"};
    int64_t _idl_result = IDL_VOID_RESULT;
    bool _use_device_transport = false;  // client: offer the xGMI hello on this call
    bool _reply_xgmi_hello = false;      // server: answer the peer's xGMI hello
    bool _reply_plane_hello = false;     // server: answer the peer's RCCL plane hello
    HttpHeader* _http_request = nullptr;
    HttpHeader* _http_response = nullptr;
    std::map<std::string, std::string> _session_kv;
    // streaming
    StreamId _request_stream = 0;
    StreamId _response_stream = 0;
    std::shared_ptr<void> _stream_creator;
    // server side
    Server* _server = nullptr;
    MethodStatus* _method_status = nullptr;
    SocketId _server_socket_id = INVALID_SOCKET_ID;
    int64_t _server_correlation_id = 0;
    bool _close_connection = false;
    void* _session_local_data = nullptr;
    const DataFactory* _session_data_factory = nullptr;
    // callback when the response arrives (used by ParallelChannel etc.)
    std::function<void(Controller*)> _on_end;

    // Engine
    void IssueRPC(int64_t begin_us);  // begin_us: monotonic start of this try
    // Called with the correlation id locked. error_code==0 means a response
    // for attempt `id` has been parsed into _response.
    void OnVersionedRPCReturned(fiber::CallId id, int error_code);
    static int HandleError(fiber::CallId id, void* data, int error_code, const std::string& error_text);
    fiber::CallId current_id() const { return _current_call.id; }
    // latency bookkeeping for server side
    int64_t _received_us = 0;
    // End an RPC that failed before any attempt was issued (id locked).
    void HandleSendFailed() { EndRPC(_current_call.id); }

private:
    void EndRPC(fiber::CallId id);
    void OnCallComplete(Call* c, int error_code, bool responded);
    void ResetNonPods();
};

// Sync helper: starts `fn` if a done closure is provided else runs it and joins.
void StartCancel(fiber::CallId id);

}  // namespace mrpc
