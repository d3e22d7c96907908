#include "base/snappy.h"

#include <cstring>
#include <vector>

namespace mrpc {
namespace snappy {

namespace {
const size_t kBlockSize = 1 << 16;
const int kMaxHashBits = 14;

inline uint32_t load32(const char* p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}
inline uint64_t load64(const char* p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}
inline uint32_t hash32(uint32_t v, int shift) { return (v * 0x1e35a7bdu) >> shift; }

char* emit_literal(char* op, const char* lit, size_t len) {
    size_t n = len - 1;
    if (n < 60) {
        *op++ = (char)(n << 2);
    } else {
        int count = 0;
        size_t t = n;
        while (t > 0) {
            ++count;
            t >>= 8;
        }
        *op++ = (char)((59 + count) << 2);
        for (int i = 0; i < count; ++i) {
            *op++ = (char)(n & 0xff);
            n >>= 8;
        }
    }
    memcpy(op, lit, len);
    return op + len;
}

char* emit_copy_upto64(char* op, size_t offset, size_t len) {
    // len in [4, 64]
    if (len < 12 && offset < 2048) {
        *op++ = (char)(1 | ((len - 4) << 2) | ((offset >> 8) << 5));
        *op++ = (char)(offset & 0xff);
    } else {
        *op++ = (char)(2 | ((len - 1) << 2));
        *op++ = (char)(offset & 0xff);
        *op++ = (char)((offset >> 8) & 0xff);
    }
    return op;
}

char* emit_copy(char* op, size_t offset, size_t len) {
    while (len >= 68) {
        op = emit_copy_upto64(op, offset, 64);
        len -= 64;
    }
    if (len > 64) {
        op = emit_copy_upto64(op, offset, 60);
        len -= 60;
    }
    return emit_copy_upto64(op, offset, len);
}

size_t match_length(const char* s1, const char* s2, const char* s2_limit) {
    size_t matched = 0;
    while (s2 + 8 <= s2_limit) {
        uint64_t x = load64(s1 + matched) ^ load64(s2);
        if (x) return matched + (__builtin_ctzll(x) >> 3);
        matched += 8;
        s2 += 8;
    }
    while (s2 < s2_limit && s1[matched] == *s2) {
        ++matched;
        ++s2;
    }
    return matched;
}

char* write_varint(char* p, uint64_t v) {
    while (v >= 0x80) {
        *p++ = (char)(v | 0x80);
        v >>= 7;
    }
    *p++ = (char)v;
    return p;
}

bool read_varint(const char** p, const char* end, uint64_t* out) {
    uint64_t r = 0;
    for (int shift = 0; shift < 35; shift += 7) {
        if (*p >= end) return false;
        uint8_t b = (uint8_t)*(*p)++;
        r |= (uint64_t)(b & 0x7f) << shift;
        if (!(b & 0x80)) {
            *out = r;
            return true;
        }
    }
    return false;
}
}  // namespace

size_t MaxCompressedLength(size_t n) { return 32 + n + n / 6; }

size_t CompressFragment(const char* input, size_t n, char* out) {
    char* op = out;
    if (n < 15) {
        if (n) op = emit_literal(op, input, n);
        return op - out;
    }
    int bits = 8;
    while (bits < kMaxHashBits && (1u << bits) < n) ++bits;
    const int shift = 32 - bits;
    std::vector<uint16_t> table((size_t)1 << bits, 0);
    const char* ip = input;
    const char* base = input;
    const char* ip_end = input + n;
    const char* ip_limit = input + n - 15;
    const char* next_emit = ip;
    ++ip;
    uint32_t next_hash = hash32(load32(ip), shift);
    for (;;) {
        uint32_t skip = 32;
        const char* next_ip = ip;
        const char* candidate;
        do {
            ip = next_ip;
            const uint32_t h = next_hash;
            const uint32_t bytes_between = skip++ >> 5;
            next_ip = ip + bytes_between;
            if (next_ip > ip_limit) goto emit_remainder;
            next_hash = hash32(load32(next_ip), shift);
            candidate = base + table[h];
            table[h] = (uint16_t)(ip - base);
        } while (load32(ip) != load32(candidate));
        op = emit_literal(op, next_emit, ip - next_emit);
        do {
            const char* b = ip;
            size_t matched = 4 + match_length(candidate + 4, ip + 4, ip_end);
            ip += matched;
            op = emit_copy(op, (size_t)(b - candidate), matched);
            next_emit = ip;
            if (ip >= ip_limit) goto emit_remainder;
            // insert hash of ip-1 and look for an immediate match at ip
            table[hash32(load32(ip - 1), shift)] = (uint16_t)(ip - 1 - base);
            const uint32_t h = hash32(load32(ip), shift);
            candidate = base + table[h];
            table[h] = (uint16_t)(ip - base);
        } while (load32(ip) == load32(candidate));
        next_hash = hash32(load32(++ip), shift);
    }
emit_remainder:
    if (next_emit < ip_end) op = emit_literal(op, next_emit, ip_end - next_emit);
    return op - out;
}

size_t RawCompress(const char* in, size_t n, char* out) {
    char* op = write_varint(out, n);
    for (size_t off = 0; off < n; off += kBlockSize) {
        const size_t len = std::min(kBlockSize, n - off);
        op += CompressFragment(in + off, len, op);
    }
    return op - out;
}

bool Compress(const char* in, size_t n, std::string* out) {
    out->resize(MaxCompressedLength(n));
    size_t len = RawCompress(in, n, &(*out)[0]);
    out->resize(len);
    return true;
}

bool GetUncompressedLength(const char* in, size_t n, size_t* result) {
    uint64_t v;
    const char* p = in;
    if (!read_varint(&p, in + n, &v)) return false;
    *result = (size_t)v;
    return true;
}

// Copy len bytes from op - off to op inside out (the ranges may overlap).
// With 16 bytes of room after the copy, whole 8-byte words are moved: a
// short offset first widens its repeating pattern to at least 8 bytes (each
// step doubles it), then every word is read before it is overwritten. The
// last word may write up to 15 bytes past the copy; later elements or the
// final length check make those bytes correct (they are always inside out).
static inline void copy_match(char* out, size_t op, size_t off, size_t len, size_t out_len) {
    char* d = out + op;
    const char* s = d - off;
    if (out_len - op >= len + 16) {
        char* const stop = d + len;
        while ((size_t)(d - s) < 8) {  // widen the pattern
            uint64_t w;
            memcpy(&w, s, 8);
            memcpy(d, &w, 8);
            d += d - s;
            if (d >= stop) return;
        }
        // the pattern distance d - s is now a multiple of off and >= 8:
        // out[x] = out[x - (d - s)], so s walks along with d
        while (d < stop) {
            uint64_t w;
            memcpy(&w, s, 8);
            memcpy(d, &w, 8);
            memcpy(&w, s + 8, 8);
            memcpy(d + 8, &w, 8);
            d += 16;
            s += 16;
        }
        return;
    }
    for (size_t i = 0; i < len; ++i) d[i] = s[i];
}

static bool decompress_impl(const char* in, size_t n, char* out, size_t out_len, bool validate_only) {
    const char* ip = in;
    const char* end = in + n;
    uint64_t ulen;
    if (!read_varint(&ip, end, &ulen) || ulen != out_len) return false;
    size_t op = 0;
    while (ip < end) {
        const uint8_t tag = (uint8_t)*ip++;
        switch (tag & 3) {
        case 0: {
            size_t len = tag >> 2;
            if (len >= 60) {
                const int nb = (int)len - 59;
                if (end - ip < nb) return false;
                len = 0;
                for (int i = 0; i < nb; ++i) len |= (size_t)(uint8_t)ip[i] << (8 * i);
                ip += nb;
            }
            ++len;
            if ((size_t)(end - ip) < len || out_len - op < len) return false;
            if (!validate_only) {
                // short literals: one fixed 16-byte move when both sides have room
                if (len <= 16 && end - ip >= 16 && out_len - op >= 16) memcpy(out + op, ip, 16);
                else memcpy(out + op, ip, len);
            }
            ip += len;
            op += len;
            break;
        }
        case 1: {
            if (ip >= end) return false;
            const size_t len = 4 + ((tag >> 2) & 7);
            const size_t off = ((size_t)(tag >> 5) << 8) | (uint8_t)*ip++;
            if (off == 0 || off > op || out_len - op < len) return false;
            if (!validate_only) copy_match(out, op, off, len, out_len);
            op += len;
            break;
        }
        case 2: {
            if (end - ip < 2) return false;
            const size_t len = 1 + (tag >> 2);
            const size_t off = (uint8_t)ip[0] | ((size_t)(uint8_t)ip[1] << 8);
            ip += 2;
            if (off == 0 || off > op || out_len - op < len) return false;
            if (!validate_only) copy_match(out, op, off, len, out_len);
            op += len;
            break;
        }
        case 3: {
            if (end - ip < 4) return false;
            const size_t len = 1 + (tag >> 2);
            const size_t off = (size_t)load32(ip);
            ip += 4;
            if (off == 0 || off > op || out_len - op < len) return false;
            if (!validate_only) copy_match(out, op, off, len, out_len);
            op += len;
            break;
        }
        }
    }
    return op == out_len;
}

bool RawUncompress(const char* in, size_t n, char* out) {
    size_t len;
    if (!GetUncompressedLength(in, n, &len)) return false;
    return decompress_impl(in, n, out, len, false);
}

bool Uncompress(const char* in, size_t n, std::string* out) {
    size_t len;
    if (!GetUncompressedLength(in, n, &len)) return false;
    if (len > (size_t)1 << 32) return false;
    out->resize(len);
    return decompress_impl(in, n, len ? &(*out)[0] : nullptr, len, false);
}

bool IsValidCompressedBuffer(const char* in, size_t n) {
    size_t len;
    if (!GetUncompressedLength(in, n, &len)) return false;
    return decompress_impl(in, n, nullptr, len, true);
}

}  // namespace snappy
}  // namespace mrpc
