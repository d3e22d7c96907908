#include "policy/authenticators.h"

#include <arpa/inet.h>

#include <cstring>

namespace mrpc {
namespace policy {

namespace {
// one RESP command as an array of bulk strings
void append_resp(std::string* out, std::initializer_list<std::string> args) {
    *out += "*" + std::to_string(args.size()) + "\r\n";
    for (const std::string& a : args) *out += "$" + std::to_string(a.size()) + "\r\n" + a + "\r\n";
}
}  // namespace

int RedisAuthenticator::GenerateCredential(std::string* auth_str) const {
    auth_str->clear();
    if (!_password.empty()) append_resp(auth_str, {"AUTH", _password});
    if (_db >= 0) append_resp(auth_str, {"SELECT", std::to_string(_db)});
    return 0;
}

int CouchbaseAuthenticator::GenerateCredential(std::string* auth_str) const {
    // 24-byte memcache binary request header, key "PLAIN", value
    // "<bucket>\0<bucket>\0<password>" (SASL PLAIN: authzid, authcid, passwd)
    static const char kMech[] = "PLAIN";
    const uint16_t key_len = (uint16_t)(sizeof(kMech) - 1);
    std::string value = _bucket;
    value.push_back('\0');
    value += _bucket;
    value.push_back('\0');
    value += _password;
    const uint32_t body_len = (uint32_t)(key_len + value.size());
    unsigned char h[24];
    memset(h, 0, sizeof(h));
    h[0] = 0x80;  // request magic
    h[1] = kMemcacheSaslAuth;
    const uint16_t kl = htons(key_len);
    memcpy(h + 2, &kl, 2);
    const uint32_t bl = htonl(body_len);
    memcpy(h + 8, &bl, 4);
    auth_str->assign(reinterpret_cast<const char*>(h), sizeof(h));
    auth_str->append(kMech, key_len);
    auth_str->append(value);
    return 0;
}

int EspAuthenticator::GenerateCredential(std::string* auth_str) const {
    static const char kMagic[] = {'\0', 'E', 'S', 'P', '\x01', '\x02'};
    auth_str->assign(kMagic, sizeof(kMagic));
    const uint16_t local_port = 0;
    auth_str->append(reinterpret_cast<const char*>(&local_port), sizeof(local_port));
    return 0;
}

const Authenticator* global_esp_authenticator() {
    static EspAuthenticator* a = new EspAuthenticator;
    return a;
}

}  // namespace policy
}  // namespace mrpc
