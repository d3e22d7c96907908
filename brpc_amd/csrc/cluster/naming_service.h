// Naming services (role of src/brpc/naming_service.h,
// periodic_naming_service.cpp:28-36, details/naming_service_thread.cpp,
// policy/*_naming_service.cpp): "scheme://name" -> list of ServerNodes.
// Built-in: list://, file://, http:// (DNS), dns://, remotefile://,
// consul://, discovery://, nacos:// (the HTTP-based control planes are
// spoken with this framework's own HTTP client).
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "base/endpoint.h"

namespace mrpc {

struct ServerNode {
    EndPoint addr;
    std::string tag;
    ServerNode() {}
    explicit ServerNode(const EndPoint& e) : addr(e) {}
    ServerNode(const EndPoint& e, const std::string& t) : addr(e), tag(t) {}
    bool operator<(const ServerNode& o) const { return addr != o.addr ? addr < o.addr : tag < o.tag; }
    bool operator==(const ServerNode& o) const { return addr == o.addr && tag == o.tag; }
};

class NamingServiceActions {
public:
    virtual ~NamingServiceActions() {}
    virtual void ResetServers(const std::vector<ServerNode>& servers) = 0;
};

class NamingService {
public:
    virtual ~NamingService() {}
    // Blocks (runs in a fiber) and keeps calling actions->ResetServers until
    // stopped (fiber interrupted). Returns non-zero on fatal error.
    virtual int RunNamingService(const char* service_name, NamingServiceActions* actions) = 0;
    virtual bool RunNamingServiceReturnsQuickly() { return false; }
    virtual NamingService* New() const = 0;
    virtual void Describe(std::ostream& os) const { os << "NamingService"; }
};

class PeriodicNamingService : public NamingService {
public:
    virtual int GetServers(const char* service_name, std::vector<ServerNode>* servers) = 0;
    int RunNamingService(const char* service_name, NamingServiceActions* actions) override;
    virtual int GetNamingServiceAccessIntervalMs() const;
};

class NamingServiceFilter {
public:
    virtual ~NamingServiceFilter() {}
    virtual bool Accept(const ServerNode& server) const = 0;
};

void RegisterNamingService(const std::string& scheme, const NamingService* prototype);
NamingService* CreateNamingService(const std::string& scheme);
void RegisterBuiltinNamingServices();
// Parses "host:port[ tag]" lines / comma lists.
bool ParseServerNode(const std::string& s, ServerNode* out);

}  // namespace mrpc
