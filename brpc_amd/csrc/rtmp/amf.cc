#include "rtmp/amf.h"

#include <cstring>
#include <sstream>

namespace mrpc {
namespace rtmp {

static const int kMaxDepth = 32;

AMFValue& AMFValue::Set(const std::string& key, const AMFValue& v) {
    for (auto& p : _props) {
        if (p.first == key) {
            p.second = v;
            return p.second;
        }
    }
    _props.emplace_back(key, v);
    return _props.back().second;
}

const AMFValue* AMFValue::Find(const std::string& key) const {
    for (auto& p : _props) {
        if (p.first == key) return &p.second;
    }
    return nullptr;
}

std::string AMFValue::DebugString() const {
    std::ostringstream os;
    switch (_type) {
    case AMF_NUMBER: os << _num; break;
    case AMF_BOOLEAN: os << (_num ? "true" : "false"); break;
    case AMF_STRING:
    case AMF_LONG_STRING: os << '"' << _str << '"'; break;
    case AMF_NULL: os << "null"; break;
    case AMF_UNDEFINED: os << "undefined"; break;
    case AMF_DATE: os << "Date(" << _num << ")"; break;
    case AMF_OBJECT:
    case AMF_ECMA_ARRAY: {
        os << '{';
        for (size_t i = 0; i < _props.size(); ++i) {
            os << (i ? ", " : "") << _props[i].first << ": " << _props[i].second.DebugString();
        }
        os << '}';
        break;
    }
    case AMF_STRICT_ARRAY: {
        os << '[';
        for (size_t i = 0; i < _items.size(); ++i) os << (i ? ", " : "") << _items[i].DebugString();
        os << ']';
        break;
    }
    default: os << "?";
    }
    return os.str();
}

static void put_u16(std::string* o, uint16_t v) {
    o->push_back((char)(v >> 8));
    o->push_back((char)v);
}
static void put_u32(std::string* o, uint32_t v) {
    for (int s = 24; s >= 0; s -= 8) o->push_back((char)(v >> s));
}
static void put_double(std::string* o, double d) {
    uint64_t b;
    memcpy(&b, &d, 8);
    for (int s = 56; s >= 0; s -= 8) o->push_back((char)(b >> s));
}
static uint16_t get_u16(const char* p) { return (uint16_t)(((uint8_t)p[0] << 8) | (uint8_t)p[1]); }
static uint32_t get_u32(const char* p) {
    return ((uint32_t)(uint8_t)p[0] << 24) | ((uint32_t)(uint8_t)p[1] << 16) | ((uint32_t)(uint8_t)p[2] << 8) |
           (uint32_t)(uint8_t)p[3];
}
static double get_double(const char* p) {
    uint64_t b = ((uint64_t)get_u32(p) << 32) | get_u32(p + 4);
    double d;
    memcpy(&d, &b, 8);
    return d;
}

static void put_key(std::string* o, const std::string& k) {
    put_u16(o, (uint16_t)k.size());
    o->append(k);
}

void WriteAMF(std::string* out, const AMFValue& v) {
    switch (v.type()) {
    case AMF_NUMBER:
        out->push_back((char)AMF_NUMBER);
        put_double(out, v.number());
        break;
    case AMF_BOOLEAN:
        out->push_back((char)AMF_BOOLEAN);
        out->push_back(v.boolean() ? 1 : 0);
        break;
    case AMF_STRING:
    case AMF_LONG_STRING:
        if (v.str().size() <= 0xffff) {
            out->push_back((char)AMF_STRING);
            put_u16(out, (uint16_t)v.str().size());
        } else {
            out->push_back((char)AMF_LONG_STRING);
            put_u32(out, (uint32_t)v.str().size());
        }
        out->append(v.str());
        break;
    case AMF_NULL: out->push_back((char)AMF_NULL); break;
    case AMF_UNDEFINED: out->push_back((char)AMF_UNDEFINED); break;
    case AMF_DATE:
        out->push_back((char)AMF_DATE);
        put_double(out, v.number());
        put_u16(out, 0);  // time zone
        break;
    case AMF_OBJECT:
    case AMF_ECMA_ARRAY:
        out->push_back((char)v.type());
        if (v.type() == AMF_ECMA_ARRAY) put_u32(out, (uint32_t)v.props().size());
        for (auto& p : v.props()) {
            put_key(out, p.first);
            WriteAMF(out, p.second);
        }
        put_u16(out, 0);
        out->push_back((char)AMF_OBJECT_END);
        break;
    case AMF_STRICT_ARRAY:
        out->push_back((char)AMF_STRICT_ARRAY);
        put_u32(out, (uint32_t)v.items().size());
        for (auto& i : v.items()) WriteAMF(out, i);
        break;
    default: out->push_back((char)AMF_UNDEFINED); break;
    }
}

// key/value pairs until the empty key + OBJECT_END marker
static size_t ReadProps(const char* p, size_t n, AMFValue* v, int depth) {
    size_t off = 0;
    for (;;) {
        if (n - off < 3) return 0;
        const uint16_t klen = get_u16(p + off);
        if (klen == 0 && (uint8_t)p[off + 2] == AMF_OBJECT_END) return off + 3;
        off += 2;
        if (n - off < klen) return 0;
        std::string key(p + off, klen);
        off += klen;
        AMFValue val;
        const size_t used = ReadAMF(p + off, n - off, &val, depth + 1);
        if (!used) return 0;
        off += used;
        v->Set(key, val);
    }
}

size_t ReadAMF(const char* p, size_t n, AMFValue* v, int depth) {
    if (n < 1 || depth > kMaxDepth) return 0;
    const uint8_t t = (uint8_t)p[0];
    switch (t) {
    case AMF_NUMBER:
        if (n < 9) return 0;
        *v = AMFValue::Number(get_double(p + 1));
        return 9;
    case AMF_BOOLEAN:
        if (n < 2) return 0;
        *v = AMFValue::Bool(p[1] != 0);
        return 2;
    case AMF_STRING: {
        if (n < 3) return 0;
        const uint16_t len = get_u16(p + 1);
        if (n - 3 < len) return 0;
        *v = AMFValue::String(std::string(p + 3, len));
        return 3 + len;
    }
    case AMF_LONG_STRING: {
        if (n < 5) return 0;
        const uint32_t len = get_u32(p + 1);
        if (n - 5 < len) return 0;
        *v = AMFValue::String(std::string(p + 5, len));
        return 5 + len;
    }
    case AMF_NULL: *v = AMFValue::Null(); return 1;
    case AMF_UNDEFINED: *v = AMFValue::Undefined(); return 1;
    case AMF_DATE:
        if (n < 11) return 0;
        *v = AMFValue::Date(get_double(p + 1));
        return 11;
    case AMF_OBJECT: {
        *v = AMFValue::Object();
        const size_t used = ReadProps(p + 1, n - 1, v, depth);
        return used ? 1 + used : 0;
    }
    case AMF_ECMA_ARRAY: {
        if (n < 5) return 0;
        *v = AMFValue::EcmaArray();
        const size_t used = ReadProps(p + 5, n - 5, v, depth);
        return used ? 5 + used : 0;
    }
    case AMF_STRICT_ARRAY: {
        if (n < 5) return 0;
        const uint32_t cnt = get_u32(p + 1);
        *v = AMFValue::StrictArray();
        size_t off = 5;
        if (cnt > n) return 0;
        for (uint32_t i = 0; i < cnt; ++i) {
            AMFValue x;
            const size_t used = ReadAMF(p + off, n - off, &x, depth + 1);
            if (!used) return 0;
            off += used;
            v->items().push_back(x);
        }
        return off;
    }
    default: return 0;
    }
}

bool ReadAMFList(const char* p, size_t n, std::vector<AMFValue>* out) {
    out->clear();
    size_t off = 0;
    while (off < n) {
        AMFValue v;
        const size_t used = ReadAMF(p + off, n - off, &v);
        if (!used) return false;
        off += used;
        out->push_back(v);
    }
    return true;
}

}  // namespace rtmp
}  // namespace mrpc
