// Built-in naming services: list://, file://, http:// and dns:// (DNS
// resolution), remotefile:// (list fetched over HTTP), consul://,
// discovery://, nacos:// (HTTP control planes; their JSON is parsed with the
// framework's own JSON reader). Periodic services poll every
// ns_access_interval seconds (reference periodic_naming_service.cpp:28-36).
#include <netdb.h>
#include <sys/stat.h>

#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>

#include "base/flags.h"
#include "base/logging.h"
#include "base/util.h"
#include "cluster/naming_service.h"
#include "fiber/fiber.h"
#include "http/http_client.h"
#include "json/json.h"

DEFINE_int32(ns_access_interval, 5, "Wait so many seconds before next access to naming service");
DEFINE_string(consul_agent_addr, "http://127.0.0.1:8500", "address of the consul agent");
DEFINE_string(consul_service_discovery_url, "/v1/health/service/", "consul health api");
DEFINE_string(discovery_api_addr, "http://127.0.0.1:7171", "address of discovery api");
DEFINE_string(nacos_address, "http://127.0.0.1:8848", "address of nacos");

namespace mrpc {

bool ParseServerNode(const std::string& line0, ServerNode* out) {
    std::string line = trim(line0);
    if (line.empty() || line[0] == '#') return false;
    std::string addr = line, tag;
    size_t sp = line.find_first_of(" \t");
    if (sp != std::string::npos) {
        addr = line.substr(0, sp);
        tag = trim(line.substr(sp + 1));
    }
    EndPoint ep;
    if (str2endpoint(addr.c_str(), &ep) != 0 && hostname2endpoint(addr.c_str(), &ep) != 0) return false;
    out->addr = ep;
    out->tag = tag;
    return true;
}

int PeriodicNamingService::GetNamingServiceAccessIntervalMs() const {
    return std::max(FLAGS_ns_access_interval, 1) * 1000;
}

int PeriodicNamingService::RunNamingService(const char* service_name, NamingServiceActions* actions) {
    std::vector<ServerNode> servers;
    bool ever_reset = false;
    for (;;) {
        servers.clear();
        const int rc = GetServers(service_name, &servers);
        if (rc == 0) {
            actions->ResetServers(servers);
            ever_reset = true;
        } else if (!ever_reset) {
            // publish an empty list so that waiters of the first batch return
            actions->ResetServers(servers);
            ever_reset = true;
        }
        if (fiber::usleep((uint64_t)GetNamingServiceAccessIntervalMs() * 1000) < 0) {
            if (errno == fiber::ESTOP || errno == EINTR) return 0;
        }
        if (fiber::stopped(fiber::self())) return 0;
    }
}

namespace {

class ListNamingService : public NamingService {
public:
    int RunNamingService(const char* name, NamingServiceActions* actions) override {
        std::vector<ServerNode> servers;
        for (const std::string& s : split_string(name, ',')) {
            ServerNode n;
            if (ParseServerNode(s, &n)) servers.push_back(n);
            else if (!trim(s).empty()) LOG(ERROR) << "Invalid address `" << s << "' in list://";
        }
        actions->ResetServers(servers);
        return 0;
    }
    bool RunNamingServiceReturnsQuickly() override { return true; }
    NamingService* New() const override { return new ListNamingService; }
    void Describe(std::ostream& os) const override { os << "list"; }
};

class FileNamingService : public NamingService {
public:
    int RunNamingService(const char* path, NamingServiceActions* actions) override {
        time_t last_mtime = 0;
        bool first = true;
        for (;;) {
            struct stat st;
            if (stat(path, &st) == 0 && (first || st.st_mtime != last_mtime)) {
                last_mtime = st.st_mtime;
                std::ifstream in(path);
                std::vector<ServerNode> servers;
                std::string line;
                while (std::getline(in, line)) {
                    ServerNode n;
                    if (ParseServerNode(line, &n)) servers.push_back(n);
                }
                actions->ResetServers(servers);
                first = false;
            } else if (first) {
                actions->ResetServers({});
                first = false;
            }
            if (fiber::usleep(100000) < 0 && (errno == fiber::ESTOP || errno == EINTR)) return 0;
            if (fiber::stopped(fiber::self())) return 0;
        }
    }
    NamingService* New() const override { return new FileNamingService; }
    void Describe(std::ostream& os) const override { os << "file"; }
};

class DomainNamingService : public PeriodicNamingService {
public:
    explicit DomainNamingService(int default_port = 80) : _default_port(default_port) {}
    int GetServers(const char* name, std::vector<ServerNode>* servers) override {
        std::string host = name;
        int port = _default_port;
        size_t slash = host.find('/');
        if (slash != std::string::npos) host = host.substr(0, slash);
        size_t colon = host.rfind(':');
        if (colon != std::string::npos) {
            port = atoi(host.c_str() + colon + 1);
            host = host.substr(0, colon);
        }
        addrinfo hints;
        memset(&hints, 0, sizeof(hints));
        hints.ai_family = AF_INET;
        hints.ai_socktype = SOCK_STREAM;
        addrinfo* res = nullptr;
        if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0) return -1;
        for (addrinfo* p = res; p; p = p->ai_next) {
            EndPoint ep(((sockaddr_in*)p->ai_addr)->sin_addr.s_addr, port);
            ServerNode n(ep);
            if (std::find(servers->begin(), servers->end(), n) == servers->end()) servers->push_back(n);
        }
        freeaddrinfo(res);
        return 0;
    }
    NamingService* New() const override { return new DomainNamingService(_default_port); }
    void Describe(std::ostream& os) const override { os << "dns"; }

private:
    int _default_port;
};

// dlist://a.com:80,b.com:8080 — every domain of the list resolved and merged
// (reference policy/domain_naming_service.cpp DomainListNamingService).
class DomainListNamingService : public PeriodicNamingService {
public:
    int GetServers(const char* name, std::vector<ServerNode>* servers) override {
        const std::string list = name;
        size_t b = 0;
        int resolved = 0;
        while (b <= list.size()) {
            size_t e = list.find(',', b);
            if (e == std::string::npos) e = list.size();
            const std::string item = trim(list.substr(b, e - b));
            if (!item.empty()) {
                DomainNamingService one;
                if (one.GetServers(item.c_str(), servers) == 0) ++resolved;
            }
            b = e + 1;
        }
        return resolved > 0 ? 0 : -1;
    }
    NamingService* New() const override { return new DomainListNamingService; }
    void Describe(std::ostream& os) const override { os << "dlist"; }
};

class RemoteFileNamingService : public PeriodicNamingService {
public:
    int GetServers(const char* name, std::vector<ServerNode>* servers) override {
        std::string body;
        if (HttpGet(std::string("http://") + name, &body, 1000) != 0) return -1;
        std::istringstream in(body);
        std::string line;
        while (std::getline(in, line)) {
            ServerNode n;
            if (ParseServerNode(line, &n)) servers->push_back(n);
        }
        return 0;
    }
    NamingService* New() const override { return new RemoteFileNamingService; }
    void Describe(std::ostream& os) const override { os << "remotefile"; }
};

// consul health API: [{"Service":{"Address":"1.2.3.4","Port":80,"Tags":[...]}}]
class ConsulNamingService : public PeriodicNamingService {
public:
    int GetServers(const char* name, std::vector<ServerNode>* servers) override {
        std::string body;
        const std::string url = FLAGS_consul_agent_addr + FLAGS_consul_service_discovery_url + name + "?passing";
        if (HttpGet(url, &body, 1000) != 0) return -1;
        json::Value v;
        if (!json::Parse(body, &v) || !v.is_array()) return -1;
        for (const json::Value& item : v.array()) {
            const json::Value* svc = item.find("Service");
            if (!svc) continue;
            const json::Value* addr = svc->find("Address");
            const json::Value* port = svc->find("Port");
            if (!addr || !port) continue;
            EndPoint ep;
            if (str2endpoint(addr->as_string().c_str(), (int)port->as_int(), &ep) != 0) continue;
            std::string tag;
            const json::Value* tags = svc->find("Tags");
            if (tags && tags->is_array() && !tags->array().empty()) tag = tags->array()[0].as_string();
            servers->emplace_back(ep, tag);
        }
        return 0;
    }
    NamingService* New() const override { return new ConsulNamingService; }
    void Describe(std::ostream& os) const override { os << "consul"; }
};

// discovery: {"data":{"<appid>":{"instances":[{"addrs":["grpc://1.2.3.4:80"],...}]}}}
class DiscoveryNamingService : public PeriodicNamingService {
public:
    int GetServers(const char* name, std::vector<ServerNode>* servers) override {
        std::string body;
        const std::string url = FLAGS_discovery_api_addr + "/discovery/fetchs?appid=" + name + "&status=1";
        if (HttpGet(url, &body, 1000) != 0) return -1;
        json::Value v;
        if (!json::Parse(body, &v)) return -1;
        const json::Value* data = v.find("data");
        if (!data) return -1;
        const json::Value* app = data->find(name);
        if (!app) return 0;
        const json::Value* insts = app->find("instances");
        if (!insts || !insts->is_array()) return 0;
        for (const json::Value& inst : insts->array()) {
            const json::Value* addrs = inst.find("addrs");
            if (!addrs || !addrs->is_array()) continue;
            for (const json::Value& a : addrs->array()) {
                std::string s = a.as_string();
                size_t p = s.find("://");
                if (p != std::string::npos) s = s.substr(p + 3);
                ServerNode n;
                if (ParseServerNode(s, &n)) servers->push_back(n);
            }
        }
        return 0;
    }
    NamingService* New() const override { return new DiscoveryNamingService; }
    void Describe(std::ostream& os) const override { os << "discovery"; }
};

// nacos: {"hosts":[{"ip":"1.2.3.4","port":80,"weight":1.0,"healthy":true}]}
class NacosNamingService : public PeriodicNamingService {
public:
    int GetServers(const char* name, std::vector<ServerNode>* servers) override {
        std::string body;
        const std::string url = FLAGS_nacos_address + "/nacos/v1/ns/instance/list?serviceName=" + name;
        if (HttpGet(url, &body, 1000) != 0) return -1;
        json::Value v;
        if (!json::Parse(body, &v)) return -1;
        const json::Value* hosts = v.find("hosts");
        if (!hosts || !hosts->is_array()) return -1;
        for (const json::Value& h : hosts->array()) {
            const json::Value* ip = h.find("ip");
            const json::Value* port = h.find("port");
            const json::Value* healthy = h.find("healthy");
            if (!ip || !port) continue;
            if (healthy && !healthy->as_bool()) continue;
            EndPoint ep;
            if (str2endpoint(ip->as_string().c_str(), (int)port->as_int(), &ep) != 0) continue;
            std::string tag;
            const json::Value* w = h.find("weight");
            if (w) tag = std::to_string((int)w->as_double());
            servers->emplace_back(ep, tag);
        }
        return 0;
    }
    NamingService* New() const override { return new NacosNamingService; }
    void Describe(std::ostream& os) const override { os << "nacos"; }
};

struct NSRegistry {
    std::mutex mu;
    std::map<std::string, const NamingService*> m;
};
NSRegistry& ns_registry() {
    static NSRegistry* r = new NSRegistry;
    return *r;
}
}  // namespace

void RegisterNamingService(const std::string& scheme, const NamingService* prototype) {
    std::lock_guard<std::mutex> g(ns_registry().mu);
    ns_registry().m[scheme] = prototype;
}

void RegisterBuiltinNamingServices() {
    static std::once_flag once;
    std::call_once(once, [] {
        RegisterNamingService("list", new ListNamingService);
        RegisterNamingService("file", new FileNamingService);
        RegisterNamingService("http", new DomainNamingService);
        RegisterNamingService("dns", new DomainNamingService);
        RegisterNamingService("https", new DomainNamingService(443));
        RegisterNamingService("redis", new DomainNamingService(6379));
        RegisterNamingService("dlist", new DomainListNamingService);
        RegisterNamingService("remotefile", new RemoteFileNamingService);
        RegisterNamingService("consul", new ConsulNamingService);
        RegisterNamingService("discovery", new DiscoveryNamingService);
        RegisterNamingService("nacos", new NacosNamingService);
    });
}

NamingService* CreateNamingService(const std::string& scheme) {
    RegisterBuiltinNamingServices();
    std::lock_guard<std::mutex> g(ns_registry().mu);
    auto it = ns_registry().m.find(to_lower(scheme));
    return it == ns_registry().m.end() ? nullptr : it->second->New();
}

}  // namespace mrpc
