// Authenticator hook (role of src/brpc/authenticator.h): the first writer
// on a client connection sends credentials; the server verifies the first
// message of each connection.
#pragma once

#include <string>

#include "base/endpoint.h"

namespace mrpc {

class AuthContext {
public:
    const std::string& user() const { return _user; }
    void set_user(const std::string& u) { _user = u; }
    const std::string& group() const { return _group; }
    void set_group(const std::string& g) { _group = g; }
    const std::string& roles() const { return _roles; }
    void set_roles(const std::string& r) { _roles = r; }
    bool is_service() const { return _is_service; }
    void set_is_service(bool s) { _is_service = s; }

private:
    std::string _user, _group, _roles;
    bool _is_service = false;
};

class Authenticator {
public:
    virtual ~Authenticator() {}
    virtual int GenerateCredential(std::string* auth_str) const = 0;
    virtual int VerifyCredential(const std::string& auth_str, const EndPoint& client_addr, AuthContext* out_ctx) const = 0;
};

}  // namespace mrpc
