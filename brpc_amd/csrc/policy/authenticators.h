// Concrete client authenticators of the reference's protocol suite:
//  * RedisAuthenticator  — "AUTH <password>" and/or "SELECT <db>" as the
//    first commands of every redis connection
//    (src/brpc/policy/redis_authenticator.{h,cpp});
//  * CouchbaseAuthenticator — memcache-binary SASL PLAIN for a bucket
//    (src/brpc/policy/couchbase_authenticator.{h,cpp});
//  * EspAuthenticator — the ESP connection preamble (magic + port), the
//    default authenticator of esp channels (src/brpc/policy/esp_authenticator.cpp,
//    src/brpc/channel.cpp:222-226).
// Credentials go out once per connection, in front of its first request
// (Controller::IssueRPC's authentication fight); the redis and memcache
// parsers consume (and check) the replies to them before the request's.
#pragma once

#include <cstdint>
#include <string>

#include "rpc/authenticator.h"

namespace mrpc {
namespace policy {

class RedisAuthenticator : public Authenticator {
public:
    explicit RedisAuthenticator(const std::string& password, int db = -1) : _password(password), _db(db) {}
    int GenerateCredential(std::string* auth_str) const override;
    int VerifyCredential(const std::string&, const EndPoint&, AuthContext*) const override { return 0; }
    // replies the server sends to the credential commands
    int auth_replies() const { return (_password.empty() ? 0 : 1) + (_db >= 0 ? 1 : 0); }
    const std::string& password() const { return _password; }
    int db() const { return _db; }

private:
    std::string _password;
    int _db;
};

class CouchbaseAuthenticator : public Authenticator {
public:
    CouchbaseAuthenticator(const std::string& bucket, const std::string& password)
        : _bucket(bucket), _password(password) {}
    int GenerateCredential(std::string* auth_str) const override;
    int VerifyCredential(const std::string&, const EndPoint&, AuthContext*) const override { return 0; }

private:
    std::string _bucket, _password;
};

class EspAuthenticator : public Authenticator {
public:
    int GenerateCredential(std::string* auth_str) const override;
    int VerifyCredential(const std::string&, const EndPoint&, AuthContext*) const override { return 0; }
};
const Authenticator* global_esp_authenticator();

// Memcache binary opcode of SASL authentication (the reply the memcache
// parser checks and drops).
const uint8_t kMemcacheSaslAuth = 0x21;

}  // namespace policy
}  // namespace mrpc
