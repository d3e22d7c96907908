#include "rpc/server.h"

#include <sys/stat.h>

#include <signal.h>
#include <unistd.h>

#include <cerrno>
#include <fstream>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"
#include "fiber/fiber.h"
#include "gpu/xgmi.h"
#include "rpc/errno.h"
#include "rpc/protocol.h"
#include "rdma/rdma.h"
#include "rpc/trackme.h"
#include "var/var.h"

DEFINE_bool(reuse_addr, true, "SO_REUSEADDR on listening sockets");

namespace mrpc {

namespace {
AddBuiltinServicesFn g_builtin_hook = nullptr;
std::atomic<bool> g_asked_to_quit{false};
void quit_handler(int) { g_asked_to_quit.store(true); }
std::atomic<int> g_running_servers{0};
var::PassiveStatus<int>* g_server_count_var = nullptr;
}  // namespace

void SetAddBuiltinServicesHook(AddBuiltinServicesFn fn) { g_builtin_hook = fn; }

Server::Server() : _status(UNINITIALIZED) {}

Server::~Server() {
    Stop(0);
    Join();
    ClearServices();
    if (!_options.pid_file.empty()) unlink(_options.pid_file.c_str());
    if (_keytable_pool) fiber::keytable_pool_destroy(_keytable_pool);
    if (_options.session_local_data_factory) {
        for (void* d : _session_pool) _options.session_local_data_factory->DestroyData(d);
    }
}

static void parse_restful(const std::string& mappings, std::vector<std::pair<std::string, std::string>>* out) {
    for (const std::string& item : split_string(mappings, ',')) {
        size_t arrow = item.find("=>");
        if (arrow == std::string::npos) continue;
        out->emplace_back(trim(item.substr(0, arrow)), trim(item.substr(arrow + 2)));
    }
}

int Server::AddServiceInternal(Service* s, bool is_builtin, ServiceOwnership ownership, const std::string& restful) {
    if (!s) return -1;
    const pb::ServiceDescriptor* sd = s->GetDescriptor();
    if (!sd) return -1;
    std::lock_guard<std::mutex> g(_mu);
    if (_status.load() == RUNNING && !is_builtin) {
        LOG(ERROR) << "Can't add service " << sd->full_name << " to a running server";
        return -1;
    }
    if (_services.count(sd->full_name)) {
        LOG(ERROR) << "Service " << sd->full_name << " already added";
        return -1;
    }
    // the restful mappings are checked before anything is registered, so a
    // bad mapping leaves no trace of the service (reference
    // Server::AddServiceInternal + RestfulMap::AddMethod)
    std::vector<std::pair<std::string, std::string>> maps;
    parse_restful(restful, &maps);
    std::vector<std::pair<std::string, std::string>> resolved;
    for (auto& m : maps) {
        std::string target = m.second;
        if (target.find('.') == std::string::npos) target = sd->full_name + "." + target;
        const pb::MethodDescriptor* found = nullptr;
        for (int i = 0; i < sd->method_count(); ++i) {
            if (sd->full_name + "." + sd->method(i)->name == target) found = sd->method(i);
        }
        if (!found) {
            LOG(ERROR) << "restful mapping to unknown method " << target;
            return -1;
        }
        if (m.first.empty() || m.first[0] != '/') {
            LOG(ERROR) << "restful path `" << m.first << "' must start with '/'";
            return -1;
        }
        for (auto& r : _restful) {
            if (r.first == m.first) {
                LOG(ERROR) << "restful path `" << m.first << "' is already mapped to " << r.second;
                return -1;
            }
        }
        for (auto& r : resolved) {
            if (r.first == m.first) {
                LOG(ERROR) << "restful path `" << m.first << "' is mapped twice";
                return -1;
            }
        }
        resolved.emplace_back(m.first, target);
    }
    ServiceProperty sp;
    sp.is_builtin_service = is_builtin;
    sp.ownership = ownership;
    sp.service = s;
    sp.restful_mappings = restful;
    _services[sd->full_name] = sp;
    _services_by_short_name[sd->name] = s;
    if (!is_builtin && !_first_service) _first_service = s;
    for (int i = 0; i < sd->method_count(); ++i) {
        const pb::MethodDescriptor* md = sd->method(i);
        MethodProperty mp;
        mp.is_builtin_service = is_builtin;
        mp.service = s;
        mp.method = md;
        mp.status = std::make_shared<MethodStatus>();
        _methods[sd->full_name + "." + md->name] = mp;
    }
    for (auto& r : resolved) {
        _methods[r.second].http_url = r.first;
        _restful.push_back(r);
    }
    return 0;
}

int Server::AddService(Service* service, ServiceOwnership ownership, const std::string& restful_mappings) {
    return AddServiceInternal(service, false, ownership, restful_mappings);
}

int Server::AddBuiltinService(Service* service) {
    return AddServiceInternal(service, true, SERVER_OWNS_SERVICE, "");
}

int Server::RemoveService(Service* service) {
    std::lock_guard<std::mutex> g(_mu);
    if (_status.load() == RUNNING) return -1;
    const pb::ServiceDescriptor* sd = service->GetDescriptor();
    auto it = _services.find(sd->full_name);
    if (it == _services.end()) return -1;
    for (int i = 0; i < sd->method_count(); ++i) _methods.erase(sd->full_name + "." + sd->method(i)->name);
    for (auto r = _restful.begin(); r != _restful.end();) {
        if (r->second.compare(0, sd->full_name.size() + 1, sd->full_name + ".") == 0) r = _restful.erase(r);
        else ++r;
    }
    _services_by_short_name.erase(sd->name);
    if (_first_service == service) _first_service = nullptr;
    if (it->second.ownership == SERVER_OWNS_SERVICE) delete it->second.service;
    _services.erase(it);
    return 0;
}

void Server::ClearServices() {
    std::lock_guard<std::mutex> g(_mu);
    for (auto& kv : _services) {
        if (kv.second.ownership == SERVER_OWNS_SERVICE) delete kv.second.service;
    }
    _services.clear();
    _services_by_short_name.clear();
    _first_service = nullptr;
    _methods.clear();
    _restful.clear();
}

Service* Server::FindServiceByFullName(const std::string& full_name) const {
    std::lock_guard<std::mutex> g(_mu);
    auto it = _services.find(full_name);
    return it == _services.end() ? nullptr : it->second.service;
}

Service* Server::FindServiceByName(const std::string& name) const {
    std::lock_guard<std::mutex> g(_mu);
    auto it = _services_by_short_name.find(name);
    return it == _services_by_short_name.end() ? nullptr : it->second;
}

const Server::MethodProperty* Server::FindMethodPropertyByFullName(const std::string& svc, const std::string& method) const {
    // The method map is immutable while running (only builtin services are
    // added before Start completes), so lookups are lock-free.
    std::string key;
    key.reserve(svc.size() + 1 + method.size());
    key.append(svc).push_back('.');
    key.append(method);
    auto it = _methods.find(key);
    if (it != _methods.end()) return &it->second;
    // allow short service names
    auto s = _services_by_short_name.find(svc);
    if (s != _services_by_short_name.end()) {
        it = _methods.find(s->second->GetDescriptor()->full_name + "." + method);
        if (it != _methods.end()) return &it->second;
    }
    return nullptr;
}

const Server::MethodProperty* Server::FindMethodPropertyByFullName(const std::string& full) const {
    size_t sep = full.find_last_of("./");
    if (sep == std::string::npos) return nullptr;
    return FindMethodPropertyByFullName(full.substr(0, sep), full.substr(sep + 1));
}

const Server::MethodProperty* Server::FindMethodPropertyByURI(const std::string& path, std::string* unresolved) const {
    // restful mappings first (longest prefix, '*' suffix wildcard)
    const std::pair<std::string, std::string>* best = nullptr;
    size_t best_len = 0;
    for (auto& r : _restful) {
        const std::string& pat = r.first;
        if (!pat.empty() && pat.back() == '*') {
            std::string prefix = pat.substr(0, pat.size() - 1);
            if (starts_with(path, prefix) && prefix.size() >= best_len) {
                best = &r;
                best_len = prefix.size();
            }
        } else if (path == pat || path == pat + "/") {
            best = &r;
            best_len = pat.size();
            break;
        }
    }
    if (best) {
        const std::string& pat = best->first;
        if (unresolved) *unresolved = pat.back() == '*' ? path.substr(best_len) : "";
        auto it = _methods.find(best->second);
        return it == _methods.end() ? nullptr : &it->second;
    }
    // default: /ServiceName/MethodName[/unresolved] or /pkg.Service/Method
    std::vector<std::string> parts = split_string(path, '/');
    if (parts.empty()) return nullptr;
    const MethodProperty* mp = nullptr;
    if (parts.size() >= 2) mp = FindMethodPropertyByFullName(parts[0], parts[1]);
    if (mp) {
        if (unresolved) {
            unresolved->clear();
            for (size_t i = 2; i < parts.size(); ++i) *unresolved += (i > 2 ? "/" : "") + parts[i];
        }
        return mp;
    }
    // [service]/default_method: /status -> status.default_method. Only
    // services that define default_method (the builtin pages) take it; an
    // unknown method of any other service is not found (404), as in the
    // reference's FindMethodPropertyByURIImpl (http_rpc_protocol.cpp:1040-1053)
    auto s = _services_by_short_name.find(parts[0]);
    if (s != _services_by_short_name.end()) {
        const pb::ServiceDescriptor* sd = s->second->GetDescriptor();
        if (sd->method_count() > 0) {
            auto it = _methods.find(sd->full_name + ".default_method");
            if (it != _methods.end()) {
                if (unresolved) {
                    unresolved->clear();
                    for (size_t i = 1; i < parts.size(); ++i) *unresolved += (i > 1 ? "/" : "") + parts[i];
                }
                return &it->second;
            }
        }
    }
    return nullptr;
}

size_t Server::service_count() const {
    std::lock_guard<std::mutex> g(_mu);
    size_t n = 0;
    for (auto& kv : _services) {
        if (!kv.second.is_builtin_service) ++n;
    }
    return n;
}

void Server::ListServices(std::vector<Service*>* out) const {
    std::lock_guard<std::mutex> g(_mu);
    out->clear();
    for (auto& kv : _services) out->push_back(kv.second.service);
}

void Server::ListMethodProperties(std::vector<const MethodProperty*>* out) const {
    std::lock_guard<std::mutex> g(_mu);
    out->clear();
    for (auto& kv : _methods) out->push_back(&kv.second);
}

std::unique_ptr<Acceptor> Server::BuildAcceptor(bool builtin_only) {
    std::unique_ptr<Acceptor> am(new Acceptor);
    std::vector<std::string> enabled;
    if (!_options.enabled_protocols.empty()) enabled = split_string_any(_options.enabled_protocols, " ,;");
    std::vector<std::pair<ProtocolType, Protocol>> protocols;
    ListProtocols(&protocols);
    // every enabled name must be a server protocol (the reference refuses to
    // start with unknown ones, server.cpp:569-612)
    for (auto& e : enabled) {
        bool known = false;
        for (auto& p : protocols) known |= p.second.support_server() && e == p.second.name;
        if (!known) {
            LOG(ERROR) << "ServerOptions.enabled_protocols has an unknown protocol `" << e << "'";
            return nullptr;
        }
    }
    for (auto& p : protocols) {
        if (!p.second.support_server()) continue;
        if (builtin_only && p.first != PROTOCOL_HTTP && p.first != PROTOCOL_H2) continue;
        if (!enabled.empty()) {
            bool ok = false;
            for (auto& e : enabled) ok |= (e == p.second.name);
            if (!ok) continue;
        }
        InputMessageHandler h;
        h.parse = p.second.parse;
        h.process = p.second.process_request;
        h.verify = _options.auth ? p.second.verify : nullptr;
        h.arg = this;
        h.name = p.second.name;
        if (am->AddHandler(h) != 0) {
            LOG(ERROR) << "Fail to add handler of protocol " << p.second.name;
            return nullptr;
        }
    }
    return am;
}

int Server::StartInternal(const EndPoint& ep, const ServerOptions* opt) {
    GlobalInitializeOrDie();
    Status expected = UNINITIALIZED;
    if (!_status.compare_exchange_strong(expected, READY)) {
        expected = READY;
        if (_status.load() == RUNNING || _status.load() == STOPPING) {
            LOG(ERROR) << "Server is already running";
            return -1;
        }
    }
    if (opt) _options = *opt;
    if (_options.num_threads > 0) fiber::set_concurrency(std::max(_options.num_threads, fiber::get_concurrency()));
    fiber::init_runtime();
    if (_options.has_builtin_services && g_builtin_hook) {
        static std::mutex once_mu;
        std::lock_guard<std::mutex> g(once_mu);
        if (!FindServiceByName("index")) g_builtin_hook(this);
    }
    if (_options.gpu_device >= 0) {
        // Serve device attachments over xGMI to same-node peers that offer it.
        std::string err;
        if (gpu::EnableXgmiTransport(_options.gpu_device, &err) != 0) {
            LOG(WARNING) << "xGMI device transport unavailable on device " << _options.gpu_device << ": " << err;
        }
    }
    _master_mp = nullptr;
    if (Service* master = _options.http_master_service) {
        // Every http request no service/restful mapping claims goes to the
        // master service's first method (tools/rpc_view proxies this way).
        const std::string& sname = master->GetDescriptor()->full_name;
        if (!FindServiceByFullName(sname) && AddService(master, SERVER_DOESNT_OWN_SERVICE) != 0) {
            LOG(ERROR) << "Fail to add http_master_service " << sname;
            _status = UNINITIALIZED;
            return -1;
        }
        if (!master->GetDescriptor()->methods.empty()) {
            _master_mp = FindMethodPropertyByFullName(sname, master->GetDescriptor()->methods[0].name);
        }
    }
    _amc = _options.max_concurrency;
    _cl.reset(CreateConcurrencyLimiter(_amc));
    if (_options.session_local_data_factory && !_keytable_pool) _keytable_pool = fiber::keytable_pool_create();
    if (_options.thread_local_data_factory && !_tls_key_created) {
        const DataFactory* f = _options.thread_local_data_factory;
        fiber::key_create2(&_tls_key, [](void* d, const void* arg) { ((const DataFactory*)arg)->DestroyData(d); }, f);
        _tls_key_created = true;
    }
    int fd = tcp_listen(ep, _options.reuse_port);
    if (fd < 0) {
        PLOG(ERROR) << "Fail to listen " << ep;
        _status = UNINITIALIZED;
        return -1;
    }
    EndPoint actual;
    if (!ep.is_unix()) {
        get_local_side(fd, &actual);
        if (!ep.v6) actual.ip = ep.ip;  // keep the asked address (0.0.0.0 stays)
    } else {
        actual = ep;
    }
    _listen_addr = actual;
    _am = BuildAcceptor(false);
    if (_am && !_options.ssl_cert_file.empty()) {
        ServerSslOptions so;
        so.cert_file = _options.ssl_cert_file;
        so.key_file = _options.ssl_key_file;
        so.ciphers = _options.ssl_ciphers;
        so.alpns = _options.ssl_alpns;
        so.certs = _options.ssl_certs;
        so.strict_sni = _options.ssl_strict_sni;
        std::string err;
        std::shared_ptr<SslContext> ctx = SslContext::NewServer(so, &err);
        if (!ctx) {
            LOG(ERROR) << "Fail to set up TLS: " << err;
            ::close(fd);
            _status = UNINITIALIZED;
            return -1;
        }
        _am->set_ssl_ctx(ctx);  // TLS and plaintext clients share the port
        _ssl_ctx = ctx;
    }
    if (_am && _options.use_rdma) {
        std::string err;
        if (!_options.ssl_cert_file.empty() || rdma::GlobalRdmaInitialize(&err) != 0) {
            LOG(ERROR) << "Fail to enable RDMA: " << (err.empty() ? "exclusive with TLS" : err);
            ::close(fd);
            _status = UNINITIALIZED;
            return -1;
        }
        _am->set_rdma(true);
    }
    if (!_am || _am->StartAccept(fd, _options.idle_timeout_sec) != 0) {
        ::close(fd);
        _status = UNINITIALIZED;
        return -1;
    }
    if (_options.internal_port > 0) {
        EndPoint iep = ep;
        iep.port = _options.internal_port;
        int ifd = tcp_listen(iep, false);
        if (ifd >= 0) {
            _internal_am = BuildAcceptor(true);
            if (_internal_am) _internal_am->StartAccept(ifd, _options.idle_timeout_sec);
        }
    }
    if (!_options.pid_file.empty()) {
        // parent directories first, like the reference's PutPidFileIfNeeded
        for (size_t pos = _options.pid_file.find('/', 1); pos != std::string::npos;
             pos = _options.pid_file.find('/', pos + 1)) {
            const std::string dir = _options.pid_file.substr(0, pos);
            if (mkdir(dir.c_str(), 0755) != 0 && errno != EEXIST) {
                LOG(WARNING) << "Fail to create " << dir << " for the pid file";
                break;
            }
        }
        std::ofstream(_options.pid_file) << getpid();
    }
    _start_us = realtime_us();
    _status = RUNNING;
    g_running_servers.fetch_add(1);
    if (!g_server_count_var) {
        g_server_count_var = new var::PassiveStatus<int>("rpc_server_count", [] { return g_running_servers.load(); });
    }
    var::start_dump_thread_if_needed();
    // expose method statuses under the real listening port
    {
        std::lock_guard<std::mutex> g(_mu);
        for (auto& kv : _methods) {
            if (kv.second.is_builtin_service) continue;
            std::string name = "rpc_server_" + std::to_string(_listen_addr.port) + "_" + kv.first;
            kv.second.status->Expose(name);
        }
    }
    LOG(INFO) << "Server is serving on " << _listen_addr;
    SetTrackMeAddress(_listen_addr);
    return 0;
}

int Server::Start(const EndPoint& ep, const ServerOptions* opt) { return StartInternal(ep, opt); }

int Server::Start(int port, const ServerOptions* opt) {
    EndPoint ep;
    str2endpoint("0.0.0.0", port, &ep);
    return StartInternal(ep, opt);
}

int Server::Start(const char* ip_port_str, const ServerOptions* opt) {
    EndPoint ep;
    if (str2endpoint(ip_port_str, &ep) != 0 && hostname2endpoint(ip_port_str, &ep) != 0) {
        // maybe just a port
        int64_t port;
        if (!parse_int64(ip_port_str, &port)) {
            LOG(ERROR) << "Invalid address `" << ip_port_str << "'";
            return -1;
        }
        str2endpoint("0.0.0.0", (int)port, &ep);
    }
    return StartInternal(ep, opt);
}

int Server::Start(int port_start, int port_end, const ServerOptions* opt) {
    for (int p = port_start; p <= port_end; ++p) {
        if (Start(p, opt) == 0) return 0;
        _status = UNINITIALIZED;
    }
    return -1;
}

int Server::Stop(int closewait_ms) {
    Status expected = RUNNING;
    if (!_status.compare_exchange_strong(expected, STOPPING)) return 0;
    if (_am) _am->StopAccept(closewait_ms);
    if (_internal_am) _internal_am->StopAccept(0);
    g_running_servers.fetch_sub(1);
    return 0;
}

int Server::AddCertificate(const CertInfo& cert) {
    std::string err;
    if (!_ssl_ctx) {
        LOG(ERROR) << "AddCertificate: the server has no default certificate";
        return -1;
    }
    if (_ssl_ctx->AddCertificate(cert, &err) != 0) {
        LOG(ERROR) << "AddCertificate: " << err;
        return -1;
    }
    return 0;
}

int Server::RemoveCertificate(const CertInfo& cert) { return _ssl_ctx ? _ssl_ctx->RemoveCertificate(cert) : -1; }

int Server::ResetCertificates(const std::vector<CertInfo>& certs) {
    std::string err;
    if (!_ssl_ctx) {
        LOG(ERROR) << "ResetCertificates: the server has no default certificate";
        return -1;
    }
    if (_ssl_ctx->ResetCertificates(certs, &err) != 0) {
        LOG(ERROR) << "ResetCertificates: " << err;
        return -1;
    }
    return 0;
}

int Server::Join() {
    if (_status.load() != STOPPING) return 0;
    // wait for in-flight requests to drain
    for (int i = 0; i < 2000 && _concurrency.load(std::memory_order_acquire) > 0; ++i) fiber::usleep(1000);
    if (_am) _am->Join();
    if (_internal_am) _internal_am->Join();
    _am.reset();
    _internal_am.reset();
    _status = READY;
    return 0;
}

void Server::RunUntilAskedToQuit() {
    signal(SIGINT, quit_handler);
    signal(SIGTERM, quit_handler);
    while (!g_asked_to_quit.load()) usleep(100000);
    Stop(0);
    Join();
}

bool Server::IsAskedToQuit() { return g_asked_to_quit.load(); }

int Server::ResetMaxConcurrency(const AdaptiveMaxConcurrency& amc) {
    std::lock_guard<std::mutex> g(_mu);
    _amc = amc;
    _cl.reset(CreateConcurrencyLimiter(amc));
    return 0;
}

int Server::max_concurrency() const { return _amc.max_concurrency(); }

int Server::SetMaxConcurrencyOf(const std::string& full_method_name, const AdaptiveMaxConcurrency& amc) {
    const size_t dot = full_method_name.rfind('.');
    if (dot == std::string::npos) return -1;
    const MethodProperty* mp =
        FindMethodPropertyByFullName(full_method_name.substr(0, dot), full_method_name.substr(dot + 1));
    if (!mp || !mp->status) return -1;
    return mp->status->SetMaxConcurrency(amc);
}

AdaptiveMaxConcurrency Server::MaxConcurrencyOf(const std::string& full_method_name) const {
    const size_t dot = full_method_name.rfind('.');
    if (dot == std::string::npos) return AdaptiveMaxConcurrency();
    const MethodProperty* mp = const_cast<Server*>(this)->FindMethodPropertyByFullName(
        full_method_name.substr(0, dot), full_method_name.substr(dot + 1));
    return mp && mp->status ? mp->status->max_concurrency() : AdaptiveMaxConcurrency();
}

bool Server::AddConcurrency(Controller* c) {
    const int cc = _concurrency.fetch_add(1, std::memory_order_relaxed) + 1;
    if (_cl && !_cl->OnRequested(cc, c)) {
        _concurrency.fetch_sub(1, std::memory_order_relaxed);
        return false;
    }
    return true;
}

void Server::RemoveConcurrency() { _concurrency.fetch_sub(1, std::memory_order_release); }

void* Server::BorrowSessionLocalData() {
    if (!_options.session_local_data_factory) return nullptr;
    {
        std::lock_guard<std::mutex> g(_session_mu);
        if (!_session_pool.empty()) {
            void* d = _session_pool.back();
            _session_pool.pop_back();
            return d;
        }
    }
    return _options.session_local_data_factory->CreateData();
}

void Server::ReturnSessionLocalData(void* d) {
    if (!d) return;
    std::lock_guard<std::mutex> g(_session_mu);
    _session_pool.push_back(d);
}

void* Server::thread_local_data() {
    if (!_tls_key_created) return nullptr;
    void* d = fiber::getspecific(_tls_key);
    if (!d) {
        d = _options.thread_local_data_factory->CreateData();
        fiber::setspecific(_tls_key, d);
    }
    return d;
}

void* Controller::session_local_data() {
    if (_session_local_data) return _session_local_data;
    if (!_server) return nullptr;
    _session_local_data = _server->BorrowSessionLocalData();
    return _session_local_data;
}

namespace {
std::mutex g_dummy_mu;
Server* g_dummy = nullptr;
}  // namespace

int StartDummyServerAt(int port) {
    std::lock_guard<std::mutex> g(g_dummy_mu);
    if (g_dummy) return -1;
    Server* s = new Server;
    ServerOptions opt;
    if (s->Start(port, &opt) != 0) {
        delete s;
        return -1;
    }
    g_dummy = s;
    return 0;
}

bool IsDummyServerRunning() {
    std::lock_guard<std::mutex> g(g_dummy_mu);
    return g_dummy != nullptr;
}

int RunningServerCount() { return g_running_servers.load(std::memory_order_relaxed); }

}  // namespace mrpc
