// proto2/proto3 wire format primitives: varint, zigzag, fixed, tags.
// Own implementation (libprotobuf is not available in this environment);
// byte-compatible with protobuf, verified against python protobuf in tests.
// The batched HIP codec kernels (ops/pb_codec.hip) implement the same
// varint rules on device.
#pragma once

#include <cstdint>
#include <cstring>
#include <string>

namespace mrpc {
namespace pb {

enum WireType : uint32_t {
    WIRETYPE_VARINT = 0,
    WIRETYPE_FIXED64 = 1,
    WIRETYPE_LENGTH_DELIMITED = 2,
    WIRETYPE_START_GROUP = 3,
    WIRETYPE_END_GROUP = 4,
    WIRETYPE_FIXED32 = 5,
};

inline uint32_t make_tag(int number, WireType wt) { return ((uint32_t)number << 3) | wt; }

inline size_t varint_size(uint64_t v) {
    // 1 + floor(log2(v|1)/7)
    int bits = 64 - __builtin_clzll(v | 1);
    return (size_t)((bits * 9 + 64) / 64);
}
inline size_t varint_size32(uint32_t v) { return varint_size(v); }
// Negative int32 are sign-extended to 10 bytes on the wire.
inline size_t int32_size(int32_t v) { return v < 0 ? 10 : varint_size((uint32_t)v); }

inline uint8_t* write_varint(uint8_t* p, uint64_t v) {
    while (v >= 0x80) {
        *p++ = (uint8_t)(v | 0x80);
        v >>= 7;
    }
    *p++ = (uint8_t)v;
    return p;
}
inline uint8_t* write_fixed32(uint8_t* p, uint32_t v) {
    memcpy(p, &v, 4);
    return p + 4;
}
inline uint8_t* write_fixed64(uint8_t* p, uint64_t v) {
    memcpy(p, &v, 8);
    return p + 8;
}
inline uint8_t* write_tag(uint8_t* p, int number, WireType wt) { return write_varint(p, make_tag(number, wt)); }

inline uint32_t zigzag32(int32_t v) { return ((uint32_t)v << 1) ^ (uint32_t)(v >> 31); }
inline uint64_t zigzag64(int64_t v) { return ((uint64_t)v << 1) ^ (uint64_t)(v >> 63); }
inline int32_t unzigzag32(uint32_t v) { return (int32_t)((v >> 1) ^ (~(v & 1) + 1)); }
inline int64_t unzigzag64(uint64_t v) { return (int64_t)((v >> 1) ^ (~(v & 1) + 1)); }

// Bounded reader over contiguous memory.
class CodedInput {
public:
    CodedInput(const void* data, size_t n)
        : _p((const uint8_t*)data), _end((const uint8_t*)data + n), _limit(_end), _depth(0) {}

    bool read_varint(uint64_t* v) {
        const uint8_t* p = _p;
        if (p < _limit && *p < 0x80) {
            *v = *p;
            _p = p + 1;
            return true;
        }
        uint64_t r = 0;
        for (int shift = 0; shift < 70; shift += 7) {
            if (p >= _limit) return false;
            uint8_t b = *p++;
            r |= (uint64_t)(b & 0x7f) << shift;
            if (!(b & 0x80)) {
                *v = r;
                _p = p;
                return true;
            }
        }
        return false;
    }
    bool read_varint32(uint32_t* v) {
        uint64_t x;
        if (!read_varint(&x)) return false;
        *v = (uint32_t)x;
        return true;
    }
    bool read_fixed32(uint32_t* v) {
        if (_limit - _p < 4) return false;
        memcpy(v, _p, 4);
        _p += 4;
        return true;
    }
    bool read_fixed64(uint64_t* v) {
        if (_limit - _p < 8) return false;
        memcpy(v, _p, 8);
        _p += 8;
        return true;
    }
    bool read_bytes(size_t n, const uint8_t** out) {
        if ((size_t)(_limit - _p) < n) return false;
        *out = _p;
        _p += n;
        return true;
    }
    bool read_string(std::string* s) {
        uint64_t n;
        const uint8_t* d;
        if (!read_varint(&n) || !read_bytes((size_t)n, &d)) return false;
        s->assign((const char*)d, (size_t)n);
        return true;
    }
    // Returns 0 at end of (limited) input.
    uint32_t read_tag() {
        if (_p >= _limit) return 0;
        uint64_t t;
        // a zero tag (field number 0) is malformed, not an end marker
        if (!read_varint(&t) || t > 0xFFFFFFFFu || t == 0) return 0xFFFFFFFFu;
        return (uint32_t)t;
    }
    bool skip_field(uint32_t tag, std::string* unknown);
    // Push a sub-limit of n bytes from the current position.
    bool push_limit(size_t n, const uint8_t** old) {
        if ((size_t)(_limit - _p) < n) return false;
        *old = _limit;
        _limit = _p + n;
        return true;
    }
    void pop_limit(const uint8_t* old) { _limit = old; }
    bool at_limit() const { return _p >= _limit; }
    const uint8_t* pos() const { return _p; }
    size_t bytes_left() const { return (size_t)(_limit - _p); }
    bool inc_depth() { return ++_depth <= 100; }
    void dec_depth() { --_depth; }

private:
    const uint8_t* _p;
    const uint8_t* _end;
    const uint8_t* _limit;
    int _depth;
};

inline bool CodedInput::skip_field(uint32_t tag, std::string* unknown) {
    const uint8_t* start = _p;
    uint64_t v;
    switch (tag & 7) {
    case WIRETYPE_VARINT:
        if (!read_varint(&v)) return false;
        break;
    case WIRETYPE_FIXED64:
        if (_limit - _p < 8) return false;
        _p += 8;
        break;
    case WIRETYPE_FIXED32:
        if (_limit - _p < 4) return false;
        _p += 4;
        break;
    case WIRETYPE_LENGTH_DELIMITED: {
        const uint8_t* d;
        if (!read_varint(&v) || !read_bytes((size_t)v, &d)) return false;
        break;
    }
    case WIRETYPE_START_GROUP: {
        const int number = (int)(tag >> 3);
        if (!inc_depth()) return false;
        for (;;) {
            uint32_t t = read_tag();
            if (t == 0 || t == 0xFFFFFFFFu) return false;
            if ((t & 7) == WIRETYPE_END_GROUP) {
                if ((int)(t >> 3) != number) return false;
                break;
            }
            if (!skip_field(t, nullptr)) return false;
        }
        dec_depth();
        break;
    }
    default:
        return false;
    }
    if (unknown) {
        uint8_t tb[10];
        uint8_t* e = write_varint(tb, tag);
        unknown->append((const char*)tb, e - tb);
        unknown->append((const char*)start, _p - start);
    }
    return true;
}

}  // namespace pb
}  // namespace mrpc
