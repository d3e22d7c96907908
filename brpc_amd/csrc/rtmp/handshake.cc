#include "rtmp/handshake.h"

#include <openssl/hmac.h>

#include <cstring>

#include "base/time.h"
#include "base/util.h"

namespace mrpc {
namespace rtmp {

namespace {

// Shared 32-byte tail of both well-known keys.
const unsigned char kKeyTail[32] = {0xF0, 0xEE, 0xC2, 0x4A, 0x80, 0x68, 0xBE, 0xE8, 0x2E, 0x00, 0xD0,
                                    0xD1, 0x02, 0x9E, 0x7E, 0x57, 0x6E, 0xEC, 0x5D, 0x2D, 0x29, 0x80,
                                    0x6F, 0xAB, 0x93, 0xB8, 0xE6, 0x36, 0xCF, 0xEB, 0x31, 0xAE};
const char kPlayerText[] = "Genuine Adobe Flash Player 001";        // 30 bytes
const char kServerText[] = "Genuine Adobe Flash Media Server 001";  // 36 bytes
const size_t kPlayerTextLen = sizeof(kPlayerText) - 1;
const size_t kServerTextLen = sizeof(kServerText) - 1;
const size_t kBlock = 764;
const size_t kDigest = 32;

std::string full_key(bool server) {
    std::string k = server ? std::string(kServerText, kServerTextLen) : std::string(kPlayerText, kPlayerTextLen);
    k.append((const char*)kKeyTail, sizeof(kKeyTail));
    return k;
}

std::string hmac_sha256(const std::string& key, const char* data, size_t n) {
    unsigned char out[EVP_MAX_MD_SIZE];
    unsigned int len = 0;
    HMAC(EVP_sha256(), key.data(), (int)key.size(), (const unsigned char*)data, n, out, &len);
    return std::string((const char*)out, len);
}

// Offset of the 32-byte digest inside a C1/S1 for `schema`.
size_t digest_pos(const std::string& b, HandshakeSchema schema) {
    const size_t block = schema == kSchema0 ? 8 + kBlock : 8;  // digest block start
    const unsigned char* p = (const unsigned char*)b.data() + block;
    return block + 4 + ((size_t)p[0] + p[1] + p[2] + p[3]) % (kBlock - 4 - kDigest);
}

std::string c1s1_digest(const std::string& b, size_t pos, bool server) {
    std::string msg;
    msg.reserve(kRtmpHandshakeSize - kDigest);
    msg.append(b, 0, pos);
    msg.append(b, pos + kDigest, std::string::npos);
    const std::string key = server ? std::string(kServerText, kServerTextLen) : std::string(kPlayerText, kPlayerTextLen);
    return hmac_sha256(key, msg.data(), msg.size());
}

void make_c1s1(HandshakeSchema schema, bool server, std::string* out) {
    out->clear();
    out->reserve(kRtmpHandshakeSize);
    const uint32_t t = (uint32_t)(monotonic_us() / 1000);
    for (int s = 24; s >= 0; s -= 8) out->push_back((char)(t >> s));
    // version: a recent player / FMS build
    const unsigned char ver_c[4] = {0x80, 0x00, 0x07, 0x02}, ver_s[4] = {0x04, 0x05, 0x00, 0x01};
    out->append((const char*)(server ? ver_s : ver_c), 4);
    while (out->size() < kRtmpHandshakeSize) out->push_back((char)fast_rand());
    const size_t pos = digest_pos(*out, schema);
    const std::string d = c1s1_digest(*out, pos, server);
    out->replace(pos, kDigest, d);
}

HandshakeSchema validate_c1s1(const std::string& b, bool server, std::string* digest) {
    if (b.size() != kRtmpHandshakeSize) return kSchemaInvalid;
    for (HandshakeSchema schema : {kSchema0, kSchema1}) {
        const size_t pos = digest_pos(b, schema);
        const std::string d = c1s1_digest(b, pos, server);
        if (memcmp(d.data(), b.data() + pos, kDigest) == 0) {
            if (digest) digest->assign(b, pos, kDigest);
            return schema;
        }
    }
    return kSchemaInvalid;
}

void make_c2s2(const std::string& peer_digest, bool server, std::string* out) {
    out->clear();
    out->reserve(kRtmpHandshakeSize);
    while (out->size() < kRtmpHandshakeSize - kDigest) out->push_back((char)fast_rand());
    const std::string temp = hmac_sha256(full_key(server), peer_digest.data(), peer_digest.size());
    out->append(hmac_sha256(temp, out->data(), out->size()));
}

bool validate_c2s2(const std::string& b, const std::string& own_digest, bool server) {
    if (b.size() != kRtmpHandshakeSize || own_digest.size() != kDigest) return false;
    const std::string temp = hmac_sha256(full_key(server), own_digest.data(), own_digest.size());
    const std::string d = hmac_sha256(temp, b.data(), kRtmpHandshakeSize - kDigest);
    return memcmp(d.data(), b.data() + kRtmpHandshakeSize - kDigest, kDigest) == 0;
}

}  // namespace

void MakeComplexC1(HandshakeSchema schema, std::string* c1) { make_c1s1(schema, false, c1); }
void MakeComplexS1(HandshakeSchema schema, std::string* s1) { make_c1s1(schema, true, s1); }
HandshakeSchema ValidateComplexC1(const std::string& c1, std::string* digest) { return validate_c1s1(c1, false, digest); }
HandshakeSchema ValidateComplexS1(const std::string& s1, std::string* digest) { return validate_c1s1(s1, true, digest); }
void MakeComplexS2(const std::string& c1_digest, std::string* s2) { make_c2s2(c1_digest, true, s2); }
void MakeComplexC2(const std::string& s1_digest, std::string* c2) { make_c2s2(s1_digest, false, c2); }
bool ValidateComplexS2(const std::string& s2, const std::string& c1_digest) { return validate_c2s2(s2, c1_digest, true); }
bool ValidateComplexC2(const std::string& c2, const std::string& s1_digest) { return validate_c2s2(c2, s1_digest, false); }

bool OffersComplexHandshake(const std::string& b) {
    return b.size() >= 8 && (b[4] != 0 || b[5] != 0 || b[6] != 0 || b[7] != 0);
}

}  // namespace rtmp
}  // namespace mrpc
