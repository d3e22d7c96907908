#include "mcpack/mcpack.h"

#include <atomic>

#include <cstring>
#include <mutex>
#include <unordered_map>

#include "base/buf.h"
#include "base/logging.h"
#include "pb/message.h"

namespace mrpc {
namespace mcpack {

using pb::CppType;
using pb::FieldDescriptor;
using pb::Message;
using pb::Reflection;

const char* type2str(uint8_t type) {
    switch (type & ~FIELD_SHORT_MASK) {
    case FIELD_OBJECT: return "object";
    case FIELD_ARRAY: return "array";
    case FIELD_ISOARRAY: return "isoarray";
    case FIELD_OBJECTISOARRAY: return "object_isoarray";
    case FIELD_STRING: return "string";
    case FIELD_BINARY: return "binary";
    case FIELD_INT8: return "int8";
    case FIELD_INT16: return "int16";
    case FIELD_INT32: return "int32";
    case FIELD_INT64: return "int64";
    case FIELD_UINT8: return "uint8";
    case FIELD_UINT16: return "uint16";
    case FIELD_UINT32: return "uint32";
    case FIELD_UINT64: return "uint64";
    case FIELD_BOOL: return "bool";
    case FIELD_FLOAT: return "float";
    case FIELD_DOUBLE: return "double";
    case FIELD_DATE: return "date";
    case FIELD_NULL: return "null";
    default: return "unknown";
    }
}

static inline void put_le32(std::string* s, size_t pos, uint32_t v) {
    char b[4] = {(char)v, (char)(v >> 8), (char)(v >> 16), (char)(v >> 24)};
    memcpy(&(*s)[pos], b, 4);
}
static inline uint32_t get_le32(const char* p) {
    const unsigned char* u = (const unsigned char*)p;
    return (uint32_t)u[0] | ((uint32_t)u[1] << 8) | ((uint32_t)u[2] << 16) | ((uint32_t)u[3] << 24);
}

// ---------------------------------------------------------------- Serializer

bool Serializer::named_ok(const std::string& name) {
    if (!_good) return false;
    if (name.size() > 254) {
        LOG(ERROR) << "mcpack: name too long: " << name;
        _good = false;
        return false;
    }
    if (_stack.empty()) {
        LOG(ERROR) << "mcpack: field `" << name << "' added outside of any object";
        _good = false;
        return false;
    }
    Group& g = _stack.back();
    const bool in_object = g.type == FIELD_OBJECT;
    if (in_object == name.empty()) {
        LOG(ERROR) << "mcpack: " << (in_object ? "unnamed field in object" : "named item in array");
        _good = false;
        return false;
    }
    ++g.count;
    return true;
}

void Serializer::put_head(uint8_t type, const std::string& name, size_t value_size) {
    const uint8_t name_size = name.empty() ? 0 : (uint8_t)(name.size() + 1);
    if (is_primitive(type)) {
        _out->push_back((char)type);
        _out->push_back((char)name_size);
    } else if ((type == FIELD_STRING || type == FIELD_BINARY) && value_size <= 255) {
        _out->push_back((char)(type | FIELD_SHORT_MASK));
        _out->push_back((char)name_size);
        _out->push_back((char)value_size);
    } else {
        _out->push_back((char)type);
        _out->push_back((char)name_size);
        const size_t at = _out->size();
        _out->append(4, '\0');
        put_le32(_out, at, (uint32_t)value_size);
    }
    if (name_size) _out->append(name.c_str(), name.size() + 1);
}

void Serializer::add_fixed(const std::string& name, uint8_t type, const void* value, size_t size) {
    if (!_good) return;
    if (!_stack.empty() && _stack.back().iso) {
        Group& g = _stack.back();
        if (!name.empty() || g.item_type != type) {
            LOG(ERROR) << "mcpack: " << type2str(type) << " added to isoarray of " << type2str(g.item_type);
            _good = false;
            return;
        }
        ++g.count;
        _out->append((const char*)value, size);
        return;
    }
    if (!named_ok(name)) return;
    put_head(type, name, size);
    _out->append((const char*)value, size);
}

void Serializer::add_string(const std::string& name, const std::string& v) {
    if (!named_ok(name)) return;
    put_head(FIELD_STRING, name, v.size() + 1);
    _out->append(v.c_str(), v.size() + 1);
}

void Serializer::add_binary(const std::string& name, const void* data, size_t len) {
    if (!named_ok(name)) return;
    put_head(FIELD_BINARY, name, len);
    _out->append((const char*)data, len);
}

void Serializer::add_null(const std::string& name) {
    if (!named_ok(name)) return;
    put_head(FIELD_NULL, name, 1);
    _out->push_back('\0');
}

void Serializer::begin_object(const std::string& name) {
    if (!_good) return;
    if (!_stack.empty() && !named_ok(name)) return;
    Group g;
    g.type = FIELD_OBJECT;
    g.item_type = 0;
    g.iso = false;
    g.head_pos = _out->size();
    put_head(FIELD_OBJECT, name, 0);
    g.value_pos = _out->size();
    _out->append(4, '\0');
    g.count = 0;
    _stack.push_back(g);
}

void Serializer::end_object() {
    if (!_good) return;
    if (_stack.empty() || _stack.back().type != FIELD_OBJECT) {
        LOG(ERROR) << "mcpack: end_object without begin_object";
        _good = false;
        return;
    }
    const Group g = _stack.back();
    _stack.pop_back();
    put_le32(_out, g.head_pos + 2, (uint32_t)(_out->size() - g.value_pos));
    put_le32(_out, g.value_pos, g.count);
}

void Serializer::begin_array(const std::string& name, uint8_t item_type, Format fmt) {
    if (!named_ok(name)) return;
    Group g;
    g.iso = (fmt == FORMAT_COMPACK && is_primitive(item_type));
    g.type = FIELD_ARRAY;
    g.item_type = item_type;
    g.head_pos = _out->size();
    put_head(g.iso ? FIELD_ISOARRAY : FIELD_ARRAY, name, 0);
    g.value_pos = _out->size();
    if (g.iso) {
        _out->push_back((char)item_type);
    } else {
        _out->append(4, '\0');
    }
    g.count = 0;
    _stack.push_back(g);
}

void Serializer::end_array() {
    if (!_good) return;
    if (_stack.empty() || _stack.back().type != FIELD_ARRAY) {
        LOG(ERROR) << "mcpack: end_array without begin_array";
        _good = false;
        return;
    }
    const Group g = _stack.back();
    _stack.pop_back();
    put_le32(_out, g.head_pos + 2, (uint32_t)(_out->size() - g.value_pos));
    if (!g.iso) put_le32(_out, g.value_pos, g.count);
}

// ---------------------------------------------------------------- Parser

size_t DecodeField(const char* p, size_t n, std::string* name, Value* value) {
    if (n < 2) return 0;
    uint8_t type = (uint8_t)p[0];
    const uint8_t name_size = (uint8_t)p[1];
    size_t head, value_size;
    if (type & FIELD_FIXED_MASK) {
        head = 2;
        value_size = primitive_size(type);
    } else if (type & FIELD_SHORT_MASK) {
        if (n < 3) return 0;
        head = 3;
        value_size = (uint8_t)p[2];
        type &= ~FIELD_SHORT_MASK;
    } else {
        if (n < 6) return 0;
        head = 6;
        value_size = get_le32(p + 2);
    }
    const size_t total = head + name_size + value_size;
    if (total > n || total < head) return 0;
    if (name) {
        if (name_size) {
            name->assign(p + head, name_size - 1);
        } else {
            name->clear();
        }
    }
    *value = Value(type, p + head + name_size, value_size);
    return total;
}

bool ListItems(const Value& group, std::vector<Item>* items) {
    items->clear();
    const uint8_t t = group.type();
    if (t == FIELD_ISOARRAY) {
        if (group.size() < 1) return false;
        const uint8_t it = (uint8_t)group.data()[0];
        const size_t sz = primitive_size(it);
        if (!sz || (group.size() - 1) % sz) return false;
        const size_t cnt = (group.size() - 1) / sz;
        items->resize(cnt);
        for (size_t i = 0; i < cnt; ++i) (*items)[i].value = Value(it, group.data() + 1 + i * sz, sz);
        return true;
    }
    if (t != FIELD_OBJECT && t != FIELD_ARRAY && t != FIELD_OBJECTISOARRAY) return false;
    if (group.size() < 4) return false;
    const uint32_t cnt = get_le32(group.data());
    const char* p = group.data() + 4;
    size_t left = group.size() - 4;
    items->reserve(cnt);
    for (uint32_t i = 0; i < cnt; ++i) {
        Item item;
        const size_t used = DecodeField(p, left, &item.name, &item.value);
        if (!used) return false;
        p += used;
        left -= used;
        if ((item.value.type() & FIELD_NON_DELETED_MASK) == 0) continue;  // deleted field
        items->push_back(std::move(item));
    }
    return true;
}

template <typename T>
static T load(const char* p) {
    T v;
    memcpy(&v, p, sizeof(T));
    return v;
}

bool Value::to_int64(int64_t* v) const {
    switch (_type) {
    case FIELD_INT8: *v = load<int8_t>(_data); return true;
    case FIELD_INT16: *v = load<int16_t>(_data); return true;
    case FIELD_INT32: *v = load<int32_t>(_data); return true;
    case FIELD_INT64: *v = load<int64_t>(_data); return true;
    case FIELD_UINT8: *v = load<uint8_t>(_data); return true;
    case FIELD_UINT16: *v = load<uint16_t>(_data); return true;
    case FIELD_UINT32: *v = load<uint32_t>(_data); return true;
    case FIELD_UINT64: *v = (int64_t)load<uint64_t>(_data); return true;
    case FIELD_BOOL: *v = _data[0] ? 1 : 0; return true;
    default: return false;
    }
}

bool Value::to_uint64(uint64_t* v) const {
    int64_t s;
    if (_type == FIELD_UINT64) {
        *v = load<uint64_t>(_data);
        return true;
    }
    if (!to_int64(&s)) return false;
    *v = (uint64_t)s;
    return true;
}

bool Value::to_double(double* v) const {
    if (_type == FIELD_FLOAT) {
        *v = load<float>(_data);
        return true;
    }
    if (_type == FIELD_DOUBLE) {
        *v = load<double>(_data);
        return true;
    }
    int64_t s;
    if (_type == FIELD_UINT64) {
        *v = (double)load<uint64_t>(_data);
        return true;
    }
    if (!to_int64(&s)) return false;
    *v = (double)s;
    return true;
}

bool Value::to_bool(bool* v) const {
    int64_t s;
    if (!to_int64(&s)) return false;
    *v = s != 0;
    return true;
}

bool Value::to_string(std::string* v) const {
    if (_type == FIELD_STRING) {
        size_t n = _size;
        if (n && _data[n - 1] == '\0') --n;
        v->assign(_data, n);
        return true;
    }
    if (_type == FIELD_BINARY) {
        v->assign(_data, _size);
        return true;
    }
    return false;
}

std::string Value::DebugString() const {
    std::string s;
    int64_t i;
    double d;
    if (to_string(&s)) return "\"" + s + "\"";
    if (_type == FIELD_UINT64) return std::to_string(load<uint64_t>(_data));
    if (to_int64(&i)) return std::to_string(i);
    if (to_double(&d)) return std::to_string(d);
    if (_type == FIELD_NULL) return "null";
    std::vector<Item> items;
    if (!ListItems(*this, &items)) return std::string("<") + type2str(_type) + ">";
    const bool obj = _type == FIELD_OBJECT;
    s = obj ? "{" : "[";
    for (size_t k = 0; k < items.size(); ++k) {
        if (k) s += ",";
        if (obj) s += items[k].name + ":";
        s += items[k].value.DebugString();
    }
    s += obj ? "}" : "]";
    return s;
}

// ---------------------------------------------------------------- pb glue

static std::string option_value(const FieldDescriptor* f, const char* key) {
    auto it = f->options.find(std::string("(") + key + ")");
    if (it == f->options.end()) it = f->options.find(key);
    if (it == f->options.end()) return std::string();
    std::string v = it->second;
    if (v.size() >= 2 && (v[0] == '"' || v[0] == '\'') && v.back() == v[0]) v = v.substr(1, v.size() - 2);
    return v;
}

static const std::string& idl_name(const FieldDescriptor* f) {
    // Cached per field: the option lookup allocates.
    static std::mutex mu;
    static std::unordered_map<const FieldDescriptor*, std::string>* cache =
        new std::unordered_map<const FieldDescriptor*, std::string>;
    std::lock_guard<std::mutex> g(mu);
    auto it = cache->find(f);
    if (it != cache->end()) return it->second;
    std::string n = option_value(f, "idl_name");
    if (n.empty()) n = f->name;
    return (*cache)[f] = n;
}

// mcpack type a pb field is written as.
static uint8_t WireType(const FieldDescriptor* f) {
    const std::string idl = option_value(f, "idl_type");
    if (!idl.empty()) {
        static const struct { const char* n; uint8_t t; } kIdl[] = {
            {"IDL_INT8", FIELD_INT8},     {"IDL_INT16", FIELD_INT16},   {"IDL_INT32", FIELD_INT32},
            {"IDL_INT64", FIELD_INT64},   {"IDL_UINT8", FIELD_UINT8},   {"IDL_UINT16", FIELD_UINT16},
            {"IDL_UINT32", FIELD_UINT32}, {"IDL_UINT64", FIELD_UINT64}, {"IDL_BOOL", FIELD_BOOL},
            {"IDL_FLOAT", FIELD_FLOAT},   {"IDL_DOUBLE", FIELD_DOUBLE}, {"IDL_BINARY", FIELD_BINARY},
            {"IDL_STRING", FIELD_STRING},
        };
        for (auto& k : kIdl) {
            if (idl == k.n) return k.t;
        }
    }
    switch (f->type) {
    case pb::FieldType::INT32:
    case pb::FieldType::SINT32:
    case pb::FieldType::SFIXED32:
    case pb::FieldType::ENUM: return FIELD_INT32;
    case pb::FieldType::INT64:
    case pb::FieldType::SINT64:
    case pb::FieldType::SFIXED64: return FIELD_INT64;
    case pb::FieldType::UINT32:
    case pb::FieldType::FIXED32: return FIELD_UINT32;
    case pb::FieldType::UINT64:
    case pb::FieldType::FIXED64: return FIELD_UINT64;
    case pb::FieldType::BOOL: return FIELD_BOOL;
    case pb::FieldType::FLOAT: return FIELD_FLOAT;
    case pb::FieldType::DOUBLE: return FIELD_DOUBLE;
    case pb::FieldType::STRING: return FIELD_STRING;
    case pb::FieldType::BYTES: return FIELD_BINARY;
    default: return FIELD_OBJECT;
    }
}

// Writes an integral/floating value with the field's wire type.
void AddConverted(Serializer* sr, const std::string& name, uint8_t t, int64_t iv, uint64_t uv, double dv,
                      bool is_float_src, bool is_unsigned_src) {
    const int64_t si = is_float_src ? (int64_t)dv : (is_unsigned_src ? (int64_t)uv : iv);
    const uint64_t ui = is_float_src ? (uint64_t)dv : (is_unsigned_src ? uv : (uint64_t)iv);
    const double d = is_float_src ? dv : (is_unsigned_src ? (double)uv : (double)iv);
    switch (t) {
    case FIELD_INT8: sr->add_int8(name, (int8_t)si); break;
    case FIELD_INT16: sr->add_int16(name, (int16_t)si); break;
    case FIELD_INT32: sr->add_int32(name, (int32_t)si); break;
    case FIELD_INT64: sr->add_int64(name, si); break;
    case FIELD_UINT8: sr->add_uint8(name, (uint8_t)ui); break;
    case FIELD_UINT16: sr->add_uint16(name, (uint16_t)ui); break;
    case FIELD_UINT32: sr->add_uint32(name, (uint32_t)ui); break;
    case FIELD_UINT64: sr->add_uint64(name, ui); break;
    case FIELD_BOOL: sr->add_bool(name, si != 0 || d != 0); break;
    case FIELD_FLOAT: sr->add_float(name, (float)d); break;
    case FIELD_DOUBLE: sr->add_double(name, d); break;
    default: sr->add_int64(name, si); break;
    }
}

static void AddScalar(Serializer* sr, const std::string& name, const Message& m, const FieldDescriptor* f, int idx,
                      uint8_t t) {
    const bool rep = idx >= 0;
    switch (f->cpp_type()) {
    case CppType::INT32: {
        const int32_t v = rep ? Reflection::GetRepeatedInt32(m, f, idx) : Reflection::GetInt32(m, f);
        return AddConverted(sr, name, t, v, 0, 0, false, false);
    }
    case CppType::ENUM: {
        const int v = rep ? Reflection::GetRepeatedEnumValue(m, f, idx) : Reflection::GetEnumValue(m, f);
        return AddConverted(sr, name, t, v, 0, 0, false, false);
    }
    case CppType::INT64: {
        const int64_t v = rep ? Reflection::GetRepeatedInt64(m, f, idx) : Reflection::GetInt64(m, f);
        return AddConverted(sr, name, t, v, 0, 0, false, false);
    }
    case CppType::UINT32: {
        const uint32_t v = rep ? Reflection::GetRepeatedUInt32(m, f, idx) : Reflection::GetUInt32(m, f);
        return AddConverted(sr, name, t, 0, v, 0, false, true);
    }
    case CppType::UINT64: {
        const uint64_t v = rep ? Reflection::GetRepeatedUInt64(m, f, idx) : Reflection::GetUInt64(m, f);
        return AddConverted(sr, name, t, 0, v, 0, false, true);
    }
    case CppType::BOOL: {
        const bool v = rep ? Reflection::GetRepeatedBool(m, f, idx) : Reflection::GetBool(m, f);
        return AddConverted(sr, name, t, v ? 1 : 0, 0, 0, false, false);
    }
    case CppType::FLOAT: {
        const float v = rep ? Reflection::GetRepeatedFloat(m, f, idx) : Reflection::GetFloat(m, f);
        return AddConverted(sr, name, t, 0, 0, v, true, false);
    }
    case CppType::DOUBLE: {
        const double v = rep ? Reflection::GetRepeatedDouble(m, f, idx) : Reflection::GetDouble(m, f);
        return AddConverted(sr, name, t, 0, 0, v, true, false);
    }
    case CppType::STRING: {
        const std::string& v = rep ? Reflection::GetRepeatedString(m, f, idx) : Reflection::GetString(m, f);
        if (t == FIELD_STRING) {
            sr->add_string(name, v);
        } else {
            sr->add_binary(name, v.data(), v.size());
        }
        return;
    }
    case CppType::MESSAGE: return;
    }
}

namespace {
std::atomic<bool> g_generated_enabled{true};
}  // namespace

void RegisterMessageHandler(const pb::Descriptor* d, const MessageHandler* h) {
    const_cast<pb::Descriptor*>(d)->mcpack_handler.store(h, std::memory_order_release);
}

const MessageHandler* FindMessageHandler(const pb::Descriptor* d) {
    if (!g_generated_enabled.load(std::memory_order_relaxed)) return nullptr;
    return static_cast<const MessageHandler*>(d->mcpack_handler.load(std::memory_order_acquire));
}

void SetGeneratedHandlersEnabled(bool on) { g_generated_enabled.store(on, std::memory_order_relaxed); }

bool SerializeFields(const Message& msg, Format fmt, Serializer* sr) {
    if (const MessageHandler* h = FindMessageHandler(msg.GetDescriptor())) return h->serialize_fields(msg, fmt, sr);
    return SerializeFieldsByReflection(msg, fmt, sr);
}

bool SerializeFieldsByReflection(const Message& msg, Format fmt, Serializer* sr) {
    const pb::Descriptor* d = msg.GetDescriptor();
    for (int i = 0; i < d->field_count() && sr->good(); ++i) {
        const FieldDescriptor* f = d->field(i);
        if (f->is_map()) continue;  // no map type in mcpack
        const std::string& name = idl_name(f);
        const uint8_t t = WireType(f);
        if (f->is_repeated()) {
            const int n = Reflection::FieldSize(msg, f);
            if (n == 0) continue;
            if (f->cpp_type() == CppType::MESSAGE) {
                sr->begin_array(name, FIELD_OBJECT, fmt);
                for (int k = 0; k < n; ++k) {
                    sr->begin_object();
                    SerializeFields(Reflection::GetRepeatedMessage(msg, f, k), fmt, sr);
                    sr->end_object();
                }
            } else {
                sr->begin_array(name, t, fmt);
                for (int k = 0; k < n; ++k) AddScalar(sr, std::string(), msg, f, k, t);
            }
            sr->end_array();
            continue;
        }
        if (!Reflection::HasField(msg, f)) continue;
        if (f->cpp_type() == CppType::MESSAGE) {
            sr->begin_object(name);
            SerializeFields(Reflection::GetMessage(msg, f), fmt, sr);
            sr->end_object();
        } else {
            AddScalar(sr, name, msg, f, -1, t);
        }
    }
    return sr->good();
}

bool SerializeToString(const Message& msg, Format fmt, std::string* out) {
    out->clear();
    Serializer sr(out);
    sr.begin_object();
    SerializeFields(msg, fmt, &sr);
    sr.end_object();
    return sr.good();
}

bool SerializeToBuf(const Message& msg, Format fmt, Buf* out) {
    std::string s;
    if (!SerializeToString(msg, fmt, &s)) return false;
    out->append(s);
    return true;
}

static const FieldDescriptor* FindByIdlName(const pb::Descriptor* d, const std::string& name) {
    static std::mutex mu;
    typedef std::unordered_map<std::string, const FieldDescriptor*> NameMap;
    static std::unordered_map<const pb::Descriptor*, NameMap>* cache = new std::unordered_map<const pb::Descriptor*, NameMap>;
    const NameMap* nm;
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache->find(d);
        if (it == cache->end()) {
            NameMap m;
            for (int i = 0; i < d->field_count(); ++i) m[option_value(d->field(i), "idl_name").empty()
                                                             ? d->field(i)->name
                                                             : option_value(d->field(i), "idl_name")] = d->field(i);
            it = cache->emplace(d, std::move(m)).first;
        }
        nm = &it->second;
    }
    auto it = nm->find(name);
    return it == nm->end() ? nullptr : it->second;
}

// Sets (or adds, when repeated) one element of field f from value v.
static bool SetFromValue(Message* m, const FieldDescriptor* f, const Value& v) {
    const bool rep = f->is_repeated();
    int64_t i;
    uint64_t u;
    double d;
    bool b;
    std::string s;
    switch (f->cpp_type()) {
    case CppType::INT32:
        if (!v.to_int64(&i)) return false;
        rep ? Reflection::AddInt32(m, f, (int32_t)i) : Reflection::SetInt32(m, f, (int32_t)i);
        return true;
    case CppType::ENUM:
        if (!v.to_int64(&i)) return false;
        rep ? Reflection::AddEnumValue(m, f, (int)i) : Reflection::SetEnumValue(m, f, (int)i);
        return true;
    case CppType::INT64:
        if (!v.to_int64(&i)) return false;
        rep ? Reflection::AddInt64(m, f, i) : Reflection::SetInt64(m, f, i);
        return true;
    case CppType::UINT32:
        if (!v.to_uint64(&u)) return false;
        rep ? Reflection::AddUInt32(m, f, (uint32_t)u) : Reflection::SetUInt32(m, f, (uint32_t)u);
        return true;
    case CppType::UINT64:
        if (!v.to_uint64(&u)) return false;
        rep ? Reflection::AddUInt64(m, f, u) : Reflection::SetUInt64(m, f, u);
        return true;
    case CppType::BOOL:
        if (!v.to_bool(&b)) return false;
        rep ? Reflection::AddBool(m, f, b) : Reflection::SetBool(m, f, b);
        return true;
    case CppType::FLOAT:
        if (!v.to_double(&d)) return false;
        rep ? Reflection::AddFloat(m, f, (float)d) : Reflection::SetFloat(m, f, (float)d);
        return true;
    case CppType::DOUBLE:
        if (!v.to_double(&d)) return false;
        rep ? Reflection::AddDouble(m, f, d) : Reflection::SetDouble(m, f, d);
        return true;
    case CppType::STRING:
        if (!v.to_string(&s)) return false;
        rep ? Reflection::AddString(m, f, s) : Reflection::SetString(m, f, s);
        return true;
    case CppType::MESSAGE: {
        if (v.type() != FIELD_OBJECT) return false;
        Message* sub = rep ? Reflection::AddMessage(m, f) : Reflection::MutableMessage(m, f);
        return ParseFromObject(v, sub);
    }
    }
    return false;
}

// {a=[1,3],b=[2,4]} -> [{a=1,b=2},{a=3,b=4}] for a repeated message field.
bool ParseObjectIsoArrayField(const Value& v, Message* m, const FieldDescriptor* f) {
    std::vector<Item> cols;
    if (!ListItems(v, &cols)) return false;
    std::vector<Message*> rows;
    const pb::Descriptor* sub = f->message_type;
    for (const Item& col : cols) {
        const FieldDescriptor* sf = sub ? FindByIdlName(sub, col.name) : nullptr;
        if (!sf) continue;
        std::vector<Item> cells;
        if (!ListItems(col.value, &cells)) return false;
        while (rows.size() < cells.size()) rows.push_back(Reflection::AddMessage(m, f));
        for (size_t r = 0; r < cells.size(); ++r) {
            if (cells[r].value.is_null()) continue;
            if (!SetFromValue(rows[r], sf, cells[r].value)) return false;
        }
    }
    return true;
}

bool ParseFromObject(const Value& obj, Message* msg) {
    if (const MessageHandler* h = FindMessageHandler(msg->GetDescriptor())) return h->parse_object(obj, msg);
    return ParseFromObjectByReflection(obj, msg);
}

bool ParseFromObjectByReflection(const Value& obj, Message* msg) {
    if (obj.type() != FIELD_OBJECT) return false;
    std::vector<Item> items;
    if (!ListItems(obj, &items)) return false;
    const pb::Descriptor* d = msg->GetDescriptor();
    for (const Item& it : items) {
        if (it.value.is_null()) continue;
        const FieldDescriptor* f = FindByIdlName(d, it.name);
        if (!f || f->is_map()) continue;  // unknown field: skipped like the reference
        const uint8_t t = it.value.type();
        if (f->is_repeated()) {
            if (t == FIELD_OBJECTISOARRAY) {
                if (f->cpp_type() != CppType::MESSAGE || !ParseObjectIsoArrayField(it.value, msg, f)) return false;
                continue;
            }
            if (t == FIELD_ARRAY || t == FIELD_ISOARRAY) {
                std::vector<Item> elems;
                if (!ListItems(it.value, &elems)) return false;
                for (const Item& e : elems) {
                    if (e.value.is_null()) continue;
                    if (!SetFromValue(msg, f, e.value)) {
                        LOG(WARNING) << "mcpack: bad element of " << it.name << ": " << type2str(e.value.type());
                        return false;
                    }
                }
                continue;
            }
        }
        if (!SetFromValue(msg, f, it.value)) {
            LOG(WARNING) << "mcpack: field `" << it.name << "' of type " << type2str(t) << " does not fit "
                         << pb::FieldTypeName(f->type);
            return false;
        }
    }
    return true;
}

bool ParseFromArray(const char* data, size_t n, Message* msg) {
    std::string name;
    Value v;
    const size_t used = DecodeField(data, n, &name, &v);
    if (!used || v.type() != FIELD_OBJECT) return false;
    msg->Clear();
    return ParseFromObject(v, msg) && msg->IsInitialized();
}

bool ParseFromBuf(const Buf& buf, Message* msg) {
    const std::string s = buf.to_string();
    return ParseFromArray(s.data(), s.size(), msg);
}

}  // namespace mcpack
}  // namespace mrpc
