// Server: service registry + acceptor + lifecycle (role of
// src/brpc/server.h:399-450, server.cpp:741-1128,1168-1237,1768-1823,2116).
#pragma once

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "base/endpoint.h"
#include "net/acceptor.h"
#include "net/ssl.h"
#include "pb/service.h"
#include "rpc/authenticator.h"
#include "rpc/concurrency_limiter.h"
#include "rpc/controller.h"
#include "rpc/method_status.h"

namespace mrpc {

class HealthReporter;
class RedisService;
class NsheadService;
class ThriftService;
class MongoServiceAdaptor;
class RtmpService;

enum ServiceOwnership { SERVER_OWNS_SERVICE, SERVER_DOESNT_OWN_SERVICE };

struct ServerOptions {
    int idle_timeout_sec = -1;
    // Worker pthreads of the fiber runtime (bthread_concurrency analog).
    int num_threads = -1;
    AdaptiveMaxConcurrency max_concurrency;  // server-wide ("unlimited" default)
    bool has_builtin_services = true;
    // comma separated protocol names, empty = all
    std::string enabled_protocols;
    const Authenticator* auth = nullptr;
    int internal_port = -1;  // builtin services only on this port if > 0
    bool reuse_port = false;
    const DataFactory* session_local_data_factory = nullptr;
    const DataFactory* thread_local_data_factory = nullptr;
    Service* http_master_service = nullptr;
    RedisService* redis_service = nullptr;
    NsheadService* nshead_service = nullptr;
    ThriftService* thrift_service = nullptr;
    MongoServiceAdaptor* mongo_service_adaptor = nullptr;
    RtmpService* rtmp_service = nullptr;
    HealthReporter* health_reporter = nullptr;
    std::string pid_file;
    // SSL: certificate + private key (PEM paths); enabled when both set.
    std::string ssl_cert_file;
    std::string ssl_key_file;
    std::string ssl_ciphers;  // OpenSSL cipher list (empty: library default)
    std::string ssl_alpns;    // e.g. "h2,http/1.1"
    // More certificates chosen by the client's SNI name, and whether a name
    // no certificate serves (or no name) is refused (net/ssl.h CertInfo;
    // reference: src/brpc/ssl_options.h:97-110)
    std::vector<CertInfo> ssl_certs;
    bool ssl_strict_sni = false;
    // Accept RDMA clients (hello detected per connection; TCP clients keep
    // working on the same port). Exclusive with TLS.
    bool use_rdma = false;
    // MI355X: device ordinal the server's GPU services run on (-1 = none).
    int gpu_device = -1;
};

class Server {
public:
    enum Status { UNINITIALIZED = 0, READY = 1, RUNNING = 2, STOPPING = 3 };
    struct MethodProperty {
        bool is_builtin_service = false;
        bool own_method_status = true;
        Service* service = nullptr;
        const pb::MethodDescriptor* method = nullptr;
        std::shared_ptr<MethodStatus> status;
        std::string http_url;  // restful mapping
    };
    struct ServiceProperty {
        bool is_builtin_service = false;
        ServiceOwnership ownership = SERVER_DOESNT_OWN_SERVICE;
        Service* service = nullptr;
        std::string restful_mappings;
    };

    Server();
    ~Server();
    Server(const Server&) = delete;
    Server& operator=(const Server&) = delete;

    // restful_mappings: "/path/a => Method1, /b/* => Method2"
    int AddService(Service* service, ServiceOwnership ownership, const std::string& restful_mappings = "");
    int AddBuiltinService(Service* service);
    int RemoveService(Service* service);
    void ClearServices();
    Service* FindServiceByFullName(const std::string& full_name) const;
    Service* FindServiceByName(const std::string& name) const;            // short name: "EchoService"
    const MethodProperty* FindMethodPropertyByFullName(const std::string& service_full_name,
                                                       const std::string& method_name) const;
    const MethodProperty* FindMethodPropertyByFullName(const std::string& full_method_name) const;
    // ServerOptions.http_master_service's method (nullptr when unset).
    const MethodProperty* master_method_property() const { return _master_mp; }
    // restful lookup: returns property and fills unresolved path
    const MethodProperty* FindMethodPropertyByURI(const std::string& path, std::string* unresolved) const;
    size_t service_count() const;
    // The first non-builtin service added (nova_pbrpc / nshead adaptors).
    Service* first_service() const { return _first_service; }
    void ListServices(std::vector<Service*>* out) const;
    void ListMethodProperties(std::vector<const MethodProperty*>* out) const;

    int Start(int port, const ServerOptions* opt);
    int Start(const char* ip_port_str, const ServerOptions* opt);
    int Start(const EndPoint& ep, const ServerOptions* opt);
    // first free port in [start,end]
    int Start(int port_start, int port_end, const ServerOptions* opt);
    int Stop(int closewait_ms);
    // Certificates chosen by SNI, changeable while the server runs
    // (reference: src/brpc/server.h:450-465). The server must have been
    // started with a default certificate. 0 on success.
    int AddCertificate(const CertInfo& cert);
    int RemoveCertificate(const CertInfo& cert);
    int ResetCertificates(const std::vector<CertInfo>& certs);
    int Join();
    void RunUntilAskedToQuit();
    static bool IsAskedToQuit();

    bool IsRunning() const { return _status.load() == RUNNING; }
    Status status() const { return _status.load(); }
    EndPoint listen_address() const { return _listen_addr; }
    int listen_port() const { return _listen_addr.port; }
    const ServerOptions& options() const { return _options; }
    int ResetMaxConcurrency(const AdaptiveMaxConcurrency& amc);
    // Per-method admission (reference Server::MaxConcurrencyOf): "N",
    // "auto", "timeout" or "unlimited" for "pkg.Service.Method" (or
    // "Service.Method"). 0 on success, -1 if no such method.
    int SetMaxConcurrencyOf(const std::string& full_method_name, const AdaptiveMaxConcurrency& amc);
    AdaptiveMaxConcurrency MaxConcurrencyOf(const std::string& full_method_name) const;
    int max_concurrency() const;
    // server-wide concurrency (AddConcurrency/RemoveConcurrency)
    bool AddConcurrency(Controller* c);
    void RemoveConcurrency();
    int concurrency() const { return _concurrency.load(std::memory_order_relaxed); }
    Acceptor* acceptor() const { return _am.get(); }
    Acceptor* internal_acceptor() const { return _internal_am.get(); }
    int64_t start_time_us() const { return _start_us; }
    const std::string& version() const { return _version; }
    void set_version(const std::string& v) { _version = v; }
    fiber::KeyTablePool* keytable_pool() const { return _keytable_pool; }
    // Per-connection user data (Controller::session_local_data).
    void* BorrowSessionLocalData();
    void ReturnSessionLocalData(void* d);
    // thread-local data (DataFactory per worker thread)
    void* thread_local_data();

private:
    int StartInternal(const EndPoint& ep, const ServerOptions* opt);
    std::unique_ptr<Acceptor> BuildAcceptor(bool builtin_only);
    int AddServiceInternal(Service* s, bool is_builtin, ServiceOwnership ownership, const std::string& restful);

    mutable std::mutex _mu;
    std::atomic<Status> _status;
    ServerOptions _options;
    EndPoint _listen_addr;
    std::unique_ptr<Acceptor> _am;
    std::unique_ptr<Acceptor> _internal_am;
    std::shared_ptr<SslContext> _ssl_ctx;  // TLS contexts of the listening port (SNI)
    std::map<std::string, ServiceProperty> _services;           // full name
    std::map<std::string, Service*> _services_by_short_name;
    Service* _first_service = nullptr;
    std::unordered_map<std::string, MethodProperty> _methods;  // "svc.Method"
    std::vector<std::pair<std::string, std::string>> _restful;  // prefix -> full method name
    const MethodProperty* _master_mp = nullptr;
    std::atomic<int> _concurrency{0};
    std::unique_ptr<ConcurrencyLimiter> _cl;
    AdaptiveMaxConcurrency _amc;
    int64_t _start_us = 0;
    std::string _version;
    fiber::KeyTablePool* _keytable_pool = nullptr;
    std::mutex _session_mu;
    std::vector<void*> _session_pool;
    fiber::FiberKey _tls_key = 0;
    bool _tls_key_created = false;
};

// Builtin services are installed by this hook (set by builtin/).
typedef int (*AddBuiltinServicesFn)(Server* server);
void SetAddBuiltinServicesHook(AddBuiltinServicesFn fn);

// Start a server hosting only builtin services (tools, dummy server).
int StartDummyServerAt(int port);
bool IsDummyServerRunning();
// Servers of this process that are running (var `rpc_server_count`).
int RunningServerCount();
// The housekeeping task every process with a channel or server runs (role of
// the reference's GlobalUpdate, src/brpc/global.cpp:223-260): once a second,
// while no server runs, a new or changed -dummy_server_port_file starts a
// builtin-only server on the port it holds. Started by GlobalInitializeOrDie.
void StartGlobalUpdate();

}  // namespace mrpc
