#include "thrift/thrift.h"

#include <cstring>
#include <sstream>

#include "rpc/method_status.h"

namespace mrpc {

ThriftService::ThriftService() : _status(new MethodStatus) {}
ThriftService::~ThriftService() {}

namespace thrift {

static const int kMaxDepth = 64;

bool Value::operator==(const Value& o) const {
    if (_type != o._type) return false;
    switch (_type) {
    case T_BOOL: case T_BYTE: case T_I16: case T_I32: case T_I64: return _i == o._i;
    case T_DOUBLE: return _d == o._d;
    case T_STRING: return _s == o._s;
    case T_STRUCT: return _fields == o._fields;
    case T_LIST: case T_SET: return _elem == o._elem && _elems == o._elems;
    case T_MAP: return _key == o._key && _elem == o._elem && _pairs == o._pairs;
    default: return true;
    }
}

std::string Value::DebugString() const {
    std::ostringstream os;
    switch (_type) {
    case T_BOOL: os << (_i ? "true" : "false"); break;
    case T_BYTE: case T_I16: case T_I32: case T_I64: os << _i; break;
    case T_DOUBLE: os << _d; break;
    case T_STRING: os << '"' << _s << '"'; break;
    case T_STRUCT: {
        os << '{';
        bool first = true;
        for (auto& kv : _fields) {
            if (!first) os << ", ";
            first = false;
            os << kv.first << ": " << kv.second.DebugString();
        }
        os << '}';
        break;
    }
    case T_LIST: case T_SET: {
        os << '[';
        for (size_t i = 0; i < _elems.size(); ++i) os << (i ? ", " : "") << _elems[i].DebugString();
        os << ']';
        break;
    }
    case T_MAP: {
        os << '{';
        for (size_t i = 0; i < _pairs.size(); ++i) {
            os << (i ? ", " : "") << _pairs[i].first.DebugString() << ": " << _pairs[i].second.DebugString();
        }
        os << '}';
        break;
    }
    default: os << "void";
    }
    return os.str();
}

static void put_be16(std::string* o, uint16_t v) {
    o->push_back((char)(v >> 8));
    o->push_back((char)v);
}
static void put_be32(std::string* o, uint32_t v) {
    for (int s = 24; s >= 0; s -= 8) o->push_back((char)(v >> s));
}
static void put_be64(std::string* o, uint64_t v) {
    for (int s = 56; s >= 0; s -= 8) o->push_back((char)(v >> s));
}
static uint16_t get_be16(const char* p) { return (uint16_t)(((uint8_t)p[0] << 8) | (uint8_t)p[1]); }
static uint32_t get_be32(const char* p) {
    return ((uint32_t)(uint8_t)p[0] << 24) | ((uint32_t)(uint8_t)p[1] << 16) | ((uint32_t)(uint8_t)p[2] << 8) |
           (uint32_t)(uint8_t)p[3];
}
static uint64_t get_be64(const char* p) { return ((uint64_t)get_be32(p) << 32) | get_be32(p + 4); }

void WriteStruct(std::string* out, const Value& s) {
    for (auto& kv : s.fields()) {
        if (kv.second.is_void()) continue;
        out->push_back((char)kv.second.type());
        put_be16(out, (uint16_t)kv.first);
        WriteValue(out, kv.second);
    }
    out->push_back((char)T_STOP);
}

void WriteValue(std::string* out, const Value& v) {
    switch (v.type()) {
    case T_BOOL: case T_BYTE: out->push_back((char)v.as_int()); break;
    case T_I16: put_be16(out, (uint16_t)v.as_int()); break;
    case T_I32: put_be32(out, (uint32_t)v.as_int()); break;
    case T_I64: put_be64(out, (uint64_t)v.as_int()); break;
    case T_DOUBLE: {
        uint64_t bits;
        const double d = v.as_double();
        memcpy(&bits, &d, 8);
        put_be64(out, bits);
        break;
    }
    case T_STRING:
        put_be32(out, (uint32_t)v.as_string().size());
        out->append(v.as_string());
        break;
    case T_STRUCT: WriteStruct(out, v); break;
    case T_LIST: case T_SET:
        out->push_back((char)v.elem_type());
        put_be32(out, (uint32_t)v.elems().size());
        for (auto& e : v.elems()) WriteValue(out, e);
        break;
    case T_MAP:
        out->push_back((char)v.key_type());
        out->push_back((char)v.elem_type());
        put_be32(out, (uint32_t)v.pairs().size());
        for (auto& kv : v.pairs()) {
            WriteValue(out, kv.first);
            WriteValue(out, kv.second);
        }
        break;
    default: break;
    }
}

size_t ReadValue(const char* p, size_t n, TType type, Value* v, int depth) {
    if (depth > kMaxDepth) return 0;
    switch (type) {
    case T_BOOL:
        if (n < 1) return 0;
        *v = Value::Bool(p[0] != 0);
        return 1;
    case T_BYTE:
        if (n < 1) return 0;
        *v = Value::Byte((int8_t)p[0]);
        return 1;
    case T_I16:
        if (n < 2) return 0;
        *v = Value::I16((int16_t)get_be16(p));
        return 2;
    case T_I32:
        if (n < 4) return 0;
        *v = Value::I32((int32_t)get_be32(p));
        return 4;
    case T_I64:
        if (n < 8) return 0;
        *v = Value::I64((int64_t)get_be64(p));
        return 8;
    case T_DOUBLE: {
        if (n < 8) return 0;
        const uint64_t bits = get_be64(p);
        double d;
        memcpy(&d, &bits, 8);
        *v = Value::Double(d);
        return 8;
    }
    case T_STRING: {
        if (n < 4) return 0;
        const uint32_t len = get_be32(p);
        if (len > n - 4) return 0;
        *v = Value::String(std::string(p + 4, len));
        return 4 + len;
    }
    case T_STRUCT: {
        *v = Value::Struct();
        size_t off = 0;
        for (;;) {
            if (off >= n) return 0;
            const TType ft = (TType)(uint8_t)p[off++];
            if (ft == T_STOP) return off;
            if (n - off < 2) return 0;
            const int16_t id = (int16_t)get_be16(p + off);
            off += 2;
            Value fv;
            const size_t used = ReadValue(p + off, n - off, ft, &fv, depth + 1);
            if (!used) return 0;
            off += used;
            v->field(id) = std::move(fv);
        }
    }
    case T_LIST: case T_SET: {
        if (n < 5) return 0;
        const TType et = (TType)(uint8_t)p[0];
        const uint32_t cnt = get_be32(p + 1);
        *v = type == T_LIST ? Value::List(et) : Value::Set(et);
        size_t off = 5;
        if (cnt > n) return 0;  // every element takes >= 1 byte
        v->elems().reserve(cnt);
        for (uint32_t i = 0; i < cnt; ++i) {
            Value e;
            const size_t used = ReadValue(p + off, n - off, et, &e, depth + 1);
            if (!used) return 0;
            off += used;
            v->elems().push_back(std::move(e));
        }
        return off;
    }
    case T_MAP: {
        if (n < 6) return 0;
        const TType kt = (TType)(uint8_t)p[0];
        const TType vt = (TType)(uint8_t)p[1];
        const uint32_t cnt = get_be32(p + 2);
        *v = Value::Map(kt, vt);
        size_t off = 6;
        if (cnt > n) return 0;
        for (uint32_t i = 0; i < cnt; ++i) {
            Value k, x;
            size_t used = ReadValue(p + off, n - off, kt, &k, depth + 1);
            if (!used) return 0;
            off += used;
            used = ReadValue(p + off, n - off, vt, &x, depth + 1);
            if (!used) return 0;
            off += used;
            v->pairs().emplace_back(std::move(k), std::move(x));
        }
        return off;
    }
    default: return 0;
    }
}

void WriteMessage(std::string* out, const MessageHeader& h, const Value& body) {
    put_be32(out, 0x80010000u | h.type);
    put_be32(out, (uint32_t)h.name.size());
    out->append(h.name);
    put_be32(out, (uint32_t)h.seqid);
    WriteStruct(out, body);
}

bool ReadMessage(const char* p, size_t n, MessageHeader* h, Value* body) {
    if (n < 12) return false;
    const uint32_t ver = get_be32(p);
    if ((ver & 0xffff0000u) != 0x80010000u) return false;  // strict binary protocol only
    h->type = (MessageType)(ver & 0xff);
    const uint32_t len = get_be32(p + 4);
    if (len > n - 8 || n - 8 - len < 4) return false;
    h->name.assign(p + 8, len);
    h->seqid = (int32_t)get_be32(p + 8 + len);
    const size_t off = 12 + len;
    return ReadValue(p + off, n - off, T_STRUCT, body) == n - off;
}

}  // namespace thrift
}  // namespace mrpc
