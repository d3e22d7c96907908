#include "base/util.h"

#include <openssl/md5.h>
#include <openssl/sha.h>
#include <unistd.h>

#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include "base/time.h"

namespace mrpc {

// ---------------------------------------------------------------- random
namespace {
struct XorShift128Plus {
    uint64_t s[2];
    XorShift128Plus() {
        uint64_t seed = (uint64_t)monotonic_ns() ^ ((uint64_t)getpid() << 32) ^ (uint64_t)(uintptr_t)this;
        // splitmix64 to fill the state
        for (int i = 0; i < 2; ++i) {
            seed += 0x9E3779B97F4A7C15ull;
            uint64_t z = seed;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            s[i] = z ^ (z >> 31);
        }
        if (!s[0] && !s[1]) s[0] = 1;
    }
    uint64_t next() {
        uint64_t s1 = s[0];
        const uint64_t s0 = s[1];
        s[0] = s0;
        s1 ^= s1 << 23;
        s[1] = s1 ^ s0 ^ (s1 >> 17) ^ (s0 >> 26);
        return s[1] + s0;
    }
};
thread_local XorShift128Plus tls_rng;
}  // namespace

uint64_t fast_rand() { return tls_rng.next(); }

uint64_t fast_rand_less_than(uint64_t range) {
    if (range == 0) return 0;
    // Lemire's nearly-divisionless reduction
    __uint128_t m = (__uint128_t)fast_rand() * range;
    return (uint64_t)(m >> 64);
}

int64_t fast_rand_in(int64_t lo, int64_t hi) {
    if (hi <= lo) return lo;
    return lo + (int64_t)fast_rand_less_than((uint64_t)(hi - lo) + 1);
}

double fast_rand_double() { return (fast_rand() >> 11) * (1.0 / 9007199254740992.0); }

// ---------------------------------------------------------------- strings
static void vappendf(std::string* out, const char* fmt, va_list ap) {
    char buf[512];
    va_list ap2;
    va_copy(ap2, ap);
    int n = vsnprintf(buf, sizeof(buf), fmt, ap2);
    va_end(ap2);
    if (n < 0) return;
    if ((size_t)n < sizeof(buf)) {
        out->append(buf, n);
        return;
    }
    size_t old = out->size();
    out->resize(old + n + 1);
    vsnprintf(&(*out)[old], n + 1, fmt, ap);
    out->resize(old + n);
}

std::string string_printf(const char* fmt, ...) {
    std::string s;
    va_list ap;
    va_start(ap, fmt);
    vappendf(&s, fmt, ap);
    va_end(ap);
    return s;
}

void string_appendf(std::string* out, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vappendf(out, fmt, ap);
    va_end(ap);
}

std::vector<std::string> split_string(const std::string& s, char sep, bool skip_empty) {
    std::vector<std::string> out;
    size_t b = 0;
    while (b <= s.size()) {
        size_t e = s.find(sep, b);
        if (e == std::string::npos) e = s.size();
        if (e > b || !skip_empty) out.push_back(s.substr(b, e - b));
        b = e + 1;
    }
    return out;
}

std::vector<std::string> split_string_any(const std::string& s, const char* seps, bool skip_empty) {
    std::vector<std::string> out;
    size_t b = 0;
    while (b <= s.size()) {
        size_t e = s.find_first_of(seps, b);
        if (e == std::string::npos) e = s.size();
        if (e > b || !skip_empty) out.push_back(s.substr(b, e - b));
        b = e + 1;
    }
    return out;
}

std::string trim(const std::string& s) {
    size_t b = s.find_first_not_of(" \t\r\n");
    if (b == std::string::npos) return "";
    size_t e = s.find_last_not_of(" \t\r\n");
    return s.substr(b, e - b + 1);
}

bool starts_with(const std::string& s, const std::string& p) { return s.compare(0, p.size(), p) == 0; }
bool ends_with(const std::string& s, const std::string& p) {
    return s.size() >= p.size() && s.compare(s.size() - p.size(), p.size(), p) == 0;
}
std::string to_lower(std::string s) {
    for (auto& c : s) c = (char)tolower((unsigned char)c);
    return s;
}
bool iequals(const std::string& a, const std::string& b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); ++i) {
        if (tolower((unsigned char)a[i]) != tolower((unsigned char)b[i])) return false;
    }
    return true;
}
std::string join(const std::vector<std::string>& v, const std::string& sep) {
    std::string out;
    for (size_t i = 0; i < v.size(); ++i) {
        if (i) out += sep;
        out += v[i];
    }
    return out;
}
bool parse_int64(const std::string& s, int64_t* out) {
    if (s.empty()) return false;
    errno = 0;
    char* end = nullptr;
    long long v = strtoll(s.c_str(), &end, 10);
    if (errno || *end) return false;
    *out = v;
    return true;
}

std::string hex_dump(const void* data, size_t n, size_t max) {
    static const char* H = "0123456789abcdef";
    std::string s;
    const uint8_t* p = (const uint8_t*)data;
    size_t m = n < max ? n : max;
    for (size_t i = 0; i < m; ++i) {
        s.push_back(H[p[i] >> 4]);
        s.push_back(H[p[i] & 15]);
    }
    if (m < n) s += "...";
    return s;
}

static int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

std::string url_decode(const std::string& s) {
    std::string out;
    out.reserve(s.size());
    for (size_t i = 0; i < s.size(); ++i) {
        if (s[i] == '%' && i + 2 < s.size() && hexval(s[i + 1]) >= 0 && hexval(s[i + 2]) >= 0) {
            out.push_back((char)(hexval(s[i + 1]) * 16 + hexval(s[i + 2])));
            i += 2;
        } else if (s[i] == '+') {
            out.push_back(' ');
        } else {
            out.push_back(s[i]);
        }
    }
    return out;
}

std::string url_encode(const std::string& s) {
    static const char* H = "0123456789ABCDEF";
    std::string out;
    for (unsigned char c : s) {
        if (isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~') {
            out.push_back((char)c);
        } else {
            out.push_back('%');
            out.push_back(H[c >> 4]);
            out.push_back(H[c & 15]);
        }
    }
    return out;
}

std::string html_escape(const std::string& s) {
    std::string out;
    for (char c : s) {
        switch (c) {
        case '<': out += "&lt;"; break;
        case '>': out += "&gt;"; break;
        case '&': out += "&amp;"; break;
        case '"': out += "&quot;"; break;
        default: out.push_back(c);
        }
    }
    return out;
}

// ---------------------------------------------------------------- hashing
static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint32_t fmix32(uint32_t h) {
    h ^= h >> 16; h *= 0x85ebca6b; h ^= h >> 13; h *= 0xc2b2ae35; h ^= h >> 16;
    return h;
}
static inline uint64_t fmix64(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
    return k;
}

uint32_t murmurhash3_32(const void* key, size_t len, uint32_t seed) {
    const uint8_t* data = (const uint8_t*)key;
    const size_t nblocks = len / 4;
    uint32_t h1 = seed;
    const uint32_t c1 = 0xcc9e2d51, c2 = 0x1b873593;
    for (size_t i = 0; i < nblocks; ++i) {
        uint32_t k1;
        memcpy(&k1, data + i * 4, 4);
        k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2;
        h1 ^= k1; h1 = rotl32(h1, 13); h1 = h1 * 5 + 0xe6546b64;
    }
    const uint8_t* tail = data + nblocks * 4;
    uint32_t k1 = 0;
    switch (len & 3) {
    case 3: k1 ^= tail[2] << 16; [[fallthrough]];
    case 2: k1 ^= tail[1] << 8; [[fallthrough]];
    case 1: k1 ^= tail[0]; k1 *= c1; k1 = rotl32(k1, 15); k1 *= c2; h1 ^= k1;
    }
    h1 ^= (uint32_t)len;
    return fmix32(h1);
}

void murmurhash3_x64_128(const void* key, size_t len, uint32_t seed, uint64_t out[2]) {
    const uint8_t* data = (const uint8_t*)key;
    const size_t nblocks = len / 16;
    uint64_t h1 = seed, h2 = seed;
    const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
    for (size_t i = 0; i < nblocks; ++i) {
        uint64_t k1, k2;
        memcpy(&k1, data + i * 16, 8);
        memcpy(&k2, data + i * 16 + 8, 8);
        k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
        h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
        k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
        h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
    }
    const uint8_t* tail = data + nblocks * 16;
    uint64_t k1 = 0, k2 = 0;
    switch (len & 15) {
    case 15: k2 ^= (uint64_t)tail[14] << 48; [[fallthrough]];
    case 14: k2 ^= (uint64_t)tail[13] << 40; [[fallthrough]];
    case 13: k2 ^= (uint64_t)tail[12] << 32; [[fallthrough]];
    case 12: k2 ^= (uint64_t)tail[11] << 24; [[fallthrough]];
    case 11: k2 ^= (uint64_t)tail[10] << 16; [[fallthrough]];
    case 10: k2 ^= (uint64_t)tail[9] << 8; [[fallthrough]];
    case 9: k2 ^= (uint64_t)tail[8]; k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2; [[fallthrough]];
    case 8: k1 ^= (uint64_t)tail[7] << 56; [[fallthrough]];
    case 7: k1 ^= (uint64_t)tail[6] << 48; [[fallthrough]];
    case 6: k1 ^= (uint64_t)tail[5] << 40; [[fallthrough]];
    case 5: k1 ^= (uint64_t)tail[4] << 32; [[fallthrough]];
    case 4: k1 ^= (uint64_t)tail[3] << 24; [[fallthrough]];
    case 3: k1 ^= (uint64_t)tail[2] << 16; [[fallthrough]];
    case 2: k1 ^= (uint64_t)tail[1] << 8; [[fallthrough]];
    case 1: k1 ^= (uint64_t)tail[0]; k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    }
    h1 ^= len; h2 ^= len;
    h1 += h2; h2 += h1;
    h1 = fmix64(h1); h2 = fmix64(h2);
    h1 += h2; h2 += h1;
    out[0] = h1;
    out[1] = h2;
}

#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wdeprecated-declarations"
void md5(const void* data, size_t n, unsigned char out[16]) { MD5((const unsigned char*)data, n, out); }
std::string sha1_hex(const void* data, size_t n) {
    unsigned char d[20];
    SHA1((const unsigned char*)data, n, d);
    return hex_dump(d, 20, 20);
}
#pragma GCC diagnostic pop

uint32_t md5_hash32(const void* data, size_t n) {
    unsigned char d[16];
    md5(data, n, d);
    uint32_t v;
    memcpy(&v, d, 4);
    return v;
}

// ---------------------------------------------------------------- base64
static const char* kB64 = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

std::string base64_encode(const void* data, size_t n) {
    const uint8_t* p = (const uint8_t*)data;
    std::string out;
    out.reserve((n + 2) / 3 * 4);
    size_t i = 0;
    for (; i + 2 < n; i += 3) {
        uint32_t v = (p[i] << 16) | (p[i + 1] << 8) | p[i + 2];
        out.push_back(kB64[v >> 18]);
        out.push_back(kB64[(v >> 12) & 63]);
        out.push_back(kB64[(v >> 6) & 63]);
        out.push_back(kB64[v & 63]);
    }
    if (i < n) {
        uint32_t v = p[i] << 16;
        if (i + 1 < n) v |= p[i + 1] << 8;
        out.push_back(kB64[v >> 18]);
        out.push_back(kB64[(v >> 12) & 63]);
        out.push_back(i + 1 < n ? kB64[(v >> 6) & 63] : '=');
        out.push_back('=');
    }
    return out;
}

bool base64_decode(const std::string& in, std::string* out) {
    int8_t rev[256];
    memset(rev, -1, sizeof(rev));
    for (int i = 0; i < 64; ++i) rev[(uint8_t)kB64[i]] = (int8_t)i;
    out->clear();
    uint32_t acc = 0;
    int bits = 0;
    size_t n = 0, pad = 0;
    for (char c : in) {
        if (c == '\n' || c == '\r' || c == ' ') continue;
        if (c == '=') {
            ++pad;
            continue;
        }
        if (pad) return false;  // data after padding
        int v = rev[(uint8_t)c];
        if (v < 0) return false;
        ++n;
        acc = (acc << 6) | (uint32_t)v;
        bits += 6;
        if (bits >= 8) {
            bits -= 8;
            out->push_back((char)((acc >> bits) & 0xff));
        }
    }
    // a lone trailing symbol carries no whole byte; padding, when present,
    // completes a 4-symbol group (unpadded input is accepted)
    if (n % 4 == 1 || pad > 2 || (pad && (n + pad) % 4 != 0)) return false;
    return true;
}

// ---------------------------------------------------------------- errno
namespace {
struct ErrTable {
    std::mutex mu;
    std::unordered_map<int, std::string> m;
};
ErrTable& errtable() {
    static ErrTable* t = new ErrTable;
    return *t;
}
}  // namespace

void RegisterErrorText(int code, const char* text) {
    ErrTable& t = errtable();
    std::lock_guard<std::mutex> g(t.mu);
    t.m[code] = text;
}

const char* ErrorText(int code) {
    {
        ErrTable& t = errtable();
        std::lock_guard<std::mutex> g(t.mu);
        auto it = t.m.find(code);
        if (it != t.m.end()) return it->second.c_str();
    }
    static thread_local char buf[128];
    const char* s = strerror_r(code, buf, sizeof(buf));
    return s;
}

}  // namespace mrpc
