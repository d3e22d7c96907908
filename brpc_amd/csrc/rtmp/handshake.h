// RTMP "complex" (digest) handshake, the form Flash players and encoders
// such as FMLE/OBS/ffmpeg use and many servers require (role of the
// reference's src/brpc/policy/rtmp_protocol.cpp handshake helpers).
//
// C1/S1 (1536 bytes) = time(4) | version(4, non-zero) | two 764-byte blocks,
// key and digest, in either order (schema 0: key first, schema 1: digest
// first). The digest block starts with 4 bytes whose sum mod 728 locates a
// 32-byte HMAC-SHA256 of the whole C1/S1 minus those 32 bytes, keyed with
// the first 30 bytes of the player key (C1) or 36 bytes of the server key
// (S1). S2 (C2) ends with HMAC-SHA256(HMAC-SHA256(full server (player) key,
// C1 (S1) digest), first 1504 bytes). No Diffie-Hellman: plain RTMP does
// not encrypt, the key block only carries random bytes.
#pragma once

#include <string>

namespace mrpc {
namespace rtmp {

static const size_t kRtmpHandshakeSize = 1536;

enum HandshakeSchema { kSchemaInvalid = -1, kSchema0 = 0, kSchema1 = 1 };

// Client: C1 with a player digest at `schema`'s position.
void MakeComplexC1(HandshakeSchema schema, std::string* c1);
// Server: S1 with a server digest at `schema`'s position.
void MakeComplexS1(HandshakeSchema schema, std::string* s1);
// Locates and verifies the digest of a peer's C1 (player key) / S1 (server
// key). Returns the schema (and the 32-byte digest) or kSchemaInvalid.
HandshakeSchema ValidateComplexC1(const std::string& c1, std::string* digest);
HandshakeSchema ValidateComplexS1(const std::string& s1, std::string* digest);
// S2 answers the client's C1 digest, C2 the server's S1 digest.
void MakeComplexS2(const std::string& c1_digest, std::string* s2);
void MakeComplexC2(const std::string& s1_digest, std::string* c2);
bool ValidateComplexS2(const std::string& s2, const std::string& c1_digest);
bool ValidateComplexC2(const std::string& c2, const std::string& s1_digest);
// True when the 4 version bytes of a C1/S1 are set (a complex handshake is
// offered); simple-handshake peers send zeros.
bool OffersComplexHandshake(const std::string& c1_or_s1);

}  // namespace rtmp
}  // namespace mrpc
