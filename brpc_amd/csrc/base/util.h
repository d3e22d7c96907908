// Small utilities: thread-local fast random numbers (role of
// butil/fast_rand.h), string helpers (string_splitter/string_printf),
// hashing (murmurhash3 + md5 for consistent hashing LBs, reference
// src/brpc/policy/hasher.cpp:20-31), base64, big-endian packing
// (butil/raw_pack.h) and a Status type.
#pragma once

#include <cstdarg>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace mrpc {

// ---- random
uint64_t fast_rand();
uint64_t fast_rand_less_than(uint64_t range);  // [0, range)
int64_t fast_rand_in(int64_t lo, int64_t hi);  // [lo, hi]
double fast_rand_double();                     // [0, 1)

// ---- strings
std::string string_printf(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void string_appendf(std::string* out, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
std::vector<std::string> split_string(const std::string& s, char sep, bool skip_empty = true);
std::vector<std::string> split_string_any(const std::string& s, const char* seps, bool skip_empty = true);
std::string trim(const std::string& s);
bool starts_with(const std::string& s, const std::string& p);
bool ends_with(const std::string& s, const std::string& p);
std::string to_lower(std::string s);
bool iequals(const std::string& a, const std::string& b);
std::string join(const std::vector<std::string>& v, const std::string& sep);
bool parse_int64(const std::string& s, int64_t* out);
std::string hex_dump(const void* data, size_t n, size_t max = 64);
std::string url_decode(const std::string& s);
std::string url_encode(const std::string& s);
std::string html_escape(const std::string& s);

// ---- hashing
uint32_t murmurhash3_32(const void* key, size_t len, uint32_t seed = 0);
void murmurhash3_x64_128(const void* key, size_t len, uint32_t seed, uint64_t out[2]);
void md5(const void* data, size_t n, unsigned char out[16]);
uint32_t md5_hash32(const void* data, size_t n);
std::string sha1_hex(const void* data, size_t n);

// ---- base64
std::string base64_encode(const void* data, size_t n);
bool base64_decode(const std::string& in, std::string* out);

// ---- big endian packing
inline void pack_be32(void* p, uint32_t v) {
    uint8_t* b = (uint8_t*)p;
    b[0] = v >> 24; b[1] = v >> 16; b[2] = v >> 8; b[3] = v;
}
inline uint32_t unpack_be32(const void* p) {
    const uint8_t* b = (const uint8_t*)p;
    return ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
}
inline void pack_be16(void* p, uint16_t v) {
    uint8_t* b = (uint8_t*)p;
    b[0] = v >> 8; b[1] = v;
}
inline uint16_t unpack_be16(const void* p) {
    const uint8_t* b = (const uint8_t*)p;
    return (uint16_t)((b[0] << 8) | b[1]);
}
inline void pack_be64(void* p, uint64_t v) {
    pack_be32(p, (uint32_t)(v >> 32));
    pack_be32((char*)p + 4, (uint32_t)v);
}
inline uint64_t unpack_be64(const void* p) {
    return ((uint64_t)unpack_be32(p) << 32) | unpack_be32((const char*)p + 4);
}
inline void pack_le32(void* p, uint32_t v) { memcpy(p, &v, 4); }
inline uint32_t unpack_le32(const void* p) { uint32_t v; memcpy(&v, p, 4); return v; }

// ---- status
class Status {
public:
    Status() : _code(0) {}
    Status(int code, const std::string& msg) : _code(code), _msg(msg) {}
    static Status OK() { return Status(); }
    bool ok() const { return _code == 0; }
    int error_code() const { return _code; }
    const std::string& error_str() const { return _msg; }
    std::string to_string() const { return ok() ? "OK" : "[" + std::to_string(_code) + "] " + _msg; }
private:
    int _code;
    std::string _msg;
};

// ---- errno text registry (role of butil/errno.h + brpc errno.proto)
void RegisterErrorText(int code, const char* text);
const char* ErrorText(int code);

}  // namespace mrpc
