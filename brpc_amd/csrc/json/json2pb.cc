#include "json/json2pb.h"

#include <charconv>

#include <strings.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "base/util.h"

namespace mrpc {
namespace json2pb {

using pb::CppType;
using pb::FieldDescriptor;
using pb::Message;
using pb::Reflection;

namespace {

// Fields jsonified as {"key": value}: real map fields, and (like the
// reference's IsProtobufMap, src/json2pb/protobuf_map.cpp) any repeated
// message of exactly a string `key` and a `value` field.
bool json_map(const FieldDescriptor* f) {
    if (f->is_map()) return true;
    if (!f->is_repeated() || f->cpp_type() != CppType::MESSAGE || !f->message_type) return false;
    const pb::Descriptor* e = f->message_type;
    return e->field_count() == 2 && e->field(0)->name == "key" && !e->field(0)->is_repeated() &&
           e->field(0)->cpp_type() == CppType::STRING && e->field(1)->name == "value";
}

// JSON key of a field: proto names cannot hold characters like '@' or '%',
// so such keys are spelled _Zddd_ (decimal char code) in the .proto; the
// JSON side sees the decoded name (reference: src/json2pb/encode_decode.cpp).
const std::string& json_key(const std::string& name, std::string* tmp) {
    if (name.find("_Z") == std::string::npos) return name;
    tmp->clear();
    size_t i = 0;
    bool changed = false;
    while (i < name.size()) {
        if (i + 6 <= name.size() && name[i] == '_' && name[i + 1] == 'Z' && name[i + 5] == '_' && isdigit((unsigned char)name[i + 2]) &&
            isdigit((unsigned char)name[i + 3]) && isdigit((unsigned char)name[i + 4])) {
            const int c = (name[i + 2] - '0') * 100 + (name[i + 3] - '0') * 10 + (name[i + 4] - '0');
            if (c < 256) {
                tmp->push_back((char)c);
                i += 6;
                changed = true;
                continue;
            }
        }
        tmp->push_back(name[i++]);
    }
    return changed ? *tmp : name;
}

json::Value scalar_to_json(const Message& m, const FieldDescriptor* f, int idx, const Pb2JsonOptions& opt) {
    const bool rep = idx >= 0;
    switch (f->cpp_type()) {
    case CppType::INT32: return json::Value((int64_t)(rep ? Reflection::GetRepeatedInt32(m, f, idx) : Reflection::GetInt32(m, f)));
    case CppType::INT64: return json::Value((int64_t)(rep ? Reflection::GetRepeatedInt64(m, f, idx) : Reflection::GetInt64(m, f)));
    case CppType::UINT32: return json::Value((uint64_t)(rep ? Reflection::GetRepeatedUInt32(m, f, idx) : Reflection::GetUInt32(m, f)));
    case CppType::UINT64: return json::Value((uint64_t)(rep ? Reflection::GetRepeatedUInt64(m, f, idx) : Reflection::GetUInt64(m, f)));
    case CppType::FLOAT: return json::Value((double)(rep ? Reflection::GetRepeatedFloat(m, f, idx) : Reflection::GetFloat(m, f)));
    case CppType::DOUBLE: return json::Value(rep ? Reflection::GetRepeatedDouble(m, f, idx) : Reflection::GetDouble(m, f));
    case CppType::BOOL: return json::Value(rep ? Reflection::GetRepeatedBool(m, f, idx) : Reflection::GetBool(m, f));
    case CppType::ENUM: {
        const int v = rep ? Reflection::GetRepeatedEnumValue(m, f, idx) : Reflection::GetEnumValue(m, f);
        if (opt.enum_option_as_string && f->enum_type) {
            const pb::EnumValueDescriptor* ev = f->enum_type->FindValueByNumber(v);
            if (ev) return json::Value(ev->name);
        }
        return json::Value((int64_t)v);
    }
    case CppType::STRING: {
        const std::string& s = rep ? Reflection::GetRepeatedString(m, f, idx) : Reflection::GetString(m, f);
        if (f->type == pb::FieldType::BYTES && opt.bytes_to_base64) return json::Value(base64_encode(s.data(), s.size()));
        return json::Value(s);
    }
    case CppType::MESSAGE: break;
    }
    return json::Value();
}

bool msg_to_value(const Message& m, json::Value* out, const Pb2JsonOptions& opt, std::string* err);

bool field_value(const Message& m, const FieldDescriptor* f, int idx, json::Value* out, const Pb2JsonOptions& opt,
                 std::string* err) {
    if (f->cpp_type() == CppType::MESSAGE) {
        const Message& sub = idx >= 0 ? Reflection::GetRepeatedMessage(m, f, idx) : Reflection::GetMessage(m, f);
        return msg_to_value(sub, out, opt, err);
    }
    *out = scalar_to_json(m, f, idx, opt);
    return true;
}

std::atomic<Pb2JsonArrayOffload> g_array_offload{nullptr};
std::atomic<size_t> g_array_offload_min{(size_t)-1};

// Run kinds of gpu/kernels.h PbRunKind (decimal output prints the value,
// so sint fields use their signed kinds).
bool array_kind(const FieldDescriptor* f, const Pb2JsonOptions& opt, uint32_t* kind) {
    switch (f->cpp_type()) {
    case CppType::INT32: *kind = 0; return true;
    case CppType::UINT32: *kind = 1; return true;
    case CppType::INT64: *kind = 3; return true;
    case CppType::UINT64: *kind = 4; return true;
    case CppType::BOOL: *kind = 6; return true;
    case CppType::ENUM: *kind = 0; return !(opt.enum_option_as_string && f->enum_type);
    default: return false;
    }
}

bool array_offload(const Message& m, const FieldDescriptor* f, const Pb2JsonOptions& opt, std::string* text) {
    Pb2JsonArrayOffload fn = g_array_offload.load(std::memory_order_acquire);
    uint32_t kind;
    if (!fn || opt.pretty_json || !array_kind(f, opt, &kind)) return false;
    size_t n = 0, eb = 0;
    const void* data = Reflection::RepeatedScalarData(m, f, &n, &eb);
    if (!data || n < g_array_offload_min.load(std::memory_order_relaxed)) return false;
    return fn(data, n, kind, text);
}

// The host twin of the device printer: the array's elements as decimal
// text straight from the field's storage (std::to_chars), one string for
// the whole array instead of a json::Value per element. Same text as
// Value-by-Value printing.
bool array_print_host(const Message& m, const FieldDescriptor* f, const Pb2JsonOptions& opt, std::string* text) {
    uint32_t kind;
    if (opt.pretty_json || !array_kind(f, opt, &kind)) return false;
    size_t n = 0, eb = 0;
    const void* data = Reflection::RepeatedScalarData(m, f, &n, &eb);
    if (!data || n == 0) return false;
    text->reserve(n * (kind == 3 || kind == 4 ? 12 : 6) + 2);
    char buf[24];
    for (size_t i = 0; i < n; ++i) {
        if (i) text->push_back(',');
        char* e = buf;
        switch (kind) {
        case 0: e = std::to_chars(buf, buf + sizeof(buf), static_cast<const int32_t*>(data)[i]).ptr; break;
        case 1: e = std::to_chars(buf, buf + sizeof(buf), static_cast<const uint32_t*>(data)[i]).ptr; break;
        case 3: e = std::to_chars(buf, buf + sizeof(buf), static_cast<const int64_t*>(data)[i]).ptr; break;
        case 4: e = std::to_chars(buf, buf + sizeof(buf), static_cast<const uint64_t*>(data)[i]).ptr; break;
        case 6: {
            const bool b = eb == 1 ? static_cast<const uint8_t*>(data)[i] != 0 : static_cast<const int32_t*>(data)[i] != 0;
            text->append(b ? "true" : "false");
            continue;
        }
        default: return false;
        }
        text->append(buf, (size_t)(e - buf));
    }
    return true;
}

bool msg_to_value(const Message& m, json::Value* out, const Pb2JsonOptions& opt, std::string* err) {
    *out = json::Value::Object();
    const pb::Descriptor* d = m.GetDescriptor();
    for (const FieldDescriptor& fd : d->fields) {
        const FieldDescriptor* f = &fd;
        std::string tmp;
        const std::string& key = opt.use_json_name ? f->json_name : json_key(f->name, &tmp);
        if (json_map(f)) {
            const int n = Reflection::FieldSize(m, f);
            if (n == 0 && !opt.jsonify_empty_array) continue;
            json::Value obj = json::Value::Object();
            const FieldDescriptor* kf = f->message_type->field(0);
            const FieldDescriptor* vf = f->message_type->field(1);
            for (int i = 0; i < n; ++i) {
                const Message& e = Reflection::GetRepeatedMessage(m, f, i);
                json::Value k = scalar_to_json(e, kf, -1, opt);
                std::string ks = k.is_string() ? k.as_string() : k.ToString();
                json::Value v;
                if (vf->is_repeated()) {  // {"key": [values...]}
                    v = json::Value::Array();
                    for (int j = 0, nv = Reflection::FieldSize(e, vf); j < nv; ++j) {
                        json::Value x;
                        if (!field_value(e, vf, j, &x, opt, err)) return false;
                        v.push_back(std::move(x));
                    }
                } else if (!field_value(e, vf, -1, &v, opt, err)) {
                    return false;
                }
                obj.set(ks, std::move(v));
            }
            out->set(key, std::move(obj));
            continue;
        }
        if (f->is_repeated()) {
            const int n = Reflection::FieldSize(m, f);
            if (n == 0 && !opt.jsonify_empty_array) continue;
            std::string printed;
            if (n > 0 && (array_offload(m, f, opt, &printed) || array_print_host(m, f, opt, &printed))) {
                printed.insert(printed.begin(), '[');
                printed.push_back(']');
                out->set(key, json::Value::Raw(std::move(printed)));
                continue;
            }
            json::Value arr = json::Value::Array();
            for (int i = 0; i < n; ++i) {
                json::Value v;
                if (!field_value(m, f, i, &v, opt, err)) return false;
                arr.push_back(std::move(v));
            }
            out->set(key, std::move(arr));
            continue;
        }
        if (!Reflection::HasField(m, f)) {
            if (f->is_required()) {  // reference pb_to_json.cpp: a hard error
                if (err) *err = "Missing required field: " + d->full_name + "." + f->name;
                return false;
            }
            if (!opt.always_print_primitive_fields || f->cpp_type() == CppType::MESSAGE) continue;
        }
        json::Value v;
        if (!field_value(m, f, -1, &v, opt, err)) return false;
        out->set(key, std::move(v));
    }
    return true;
}

// ---------------------------------------------------------------- json -> pb
// Conversion rules and error texts follow the reference's json2pb
// (src/json2pb/json_to_pb.cpp) so callers that log or compare them see the
// same thing: descriptor fields are visited in declaration order; a value of
// the wrong kind in an OPTIONAL field is reported ("Invalid value `v' for
// optional field `pkg.Msg.f' which SHOULD be T") and skipped while the
// conversion goes on, in a required or repeated field it fails the
// conversion; every error is appended to *err with ", ".
class J2P {
public:
    J2P(const Json2PbOptions& opt, std::string* err) : _opt(opt), _err(err) {}

    bool message(const json::Value& v, Message* m) {
        const pb::Descriptor* d = m->GetDescriptor();
        if (!v.is_object()) {
            append("The input is not a json object [" + d->name + "]");
            return false;
        }
        if (!_opt.allow_unknown_fields) {
            for (const auto& kv : v.members()) {
                if (!find_field(d, kv.first)) {
                    append("Unknown field `" + kv.first + "' in " + d->full_name);
                    return false;
                }
            }
        }
        for (int i = 0; i < d->field_count(); ++i) {
            const FieldDescriptor* f = d->field(i);
            std::string tmp;
            const json::Value* fv = v.find(json_key(f->name, &tmp));
            if (!fv && !f->json_name.empty() && f->json_name != f->name) fv = v.find(f->json_name);
            if (!fv) {
                if (f->is_required()) {
                    append("Missing required field: " + full_name(f));
                    return false;
                }
                continue;
            }
            if (json_map(f) && fv->is_object()) {
                if (!map(*fv, f, m)) return false;
            } else if (!field(*fv, f, m)) {
                return false;
            }
        }
        return true;
    }

private:
    static const FieldDescriptor* find_field(const pb::Descriptor* d, const std::string& key) {
        if (const FieldDescriptor* f = d->FindFieldByName(key)) return f;
        if (const FieldDescriptor* f = d->FindFieldByJsonName(key)) return f;
        std::string tmp;
        for (int i = 0; i < d->field_count(); ++i) {
            if (json_key(d->field(i)->name, &tmp) == key) return d->field(i);
        }
        return nullptr;
    }

    static std::string full_name(const FieldDescriptor* f) {
        return f->containing_type ? f->containing_type->full_name + "." + f->name : f->name;
    }

    void append(const std::string& s) {
        if (!_err) return;
        if (!_err->empty()) *_err += ", ";
        *_err += s;
    }

    static std::string describe(const json::Value& v) {
        char b[64];
        switch (v.type()) {
        case json::Value::NUL: return "null";
        case json::Value::BOOL: return v.as_bool() ? "true" : "false";
        case json::Value::INT: snprintf(b, sizeof(b), "%lld", (long long)v.as_int()); return b;
        case json::Value::UINT: snprintf(b, sizeof(b), "%llu", (unsigned long long)v.as_uint()); return b;
        case json::Value::DOUBLE: snprintf(b, sizeof(b), "%f", v.as_double()); return b;
        case json::Value::STRING: return "\"" + v.as_string() + "\"";
        case json::Value::ARRAY: return "array";
        case json::Value::OBJECT: return "object";
        case json::Value::RAW: return v.as_string();
        }
        return "";
    }

    // a value of the wrong kind: soft for optional fields, fatal otherwise
    bool invalid(const FieldDescriptor* f, const char* type, const json::Value& v) {
        const bool optional = f->label == pb::Label::OPTIONAL;
        append("Invalid value `" + describe(v) + "' for " + (optional ? "optional " : "") + "field `" + full_name(f) +
               "' which SHOULD be " + type);
        return optional;
    }

    static bool integral(const json::Value& v, int64_t lo, uint64_t hi) {
        if (v.type() == json::Value::INT) return v.as_int() >= lo && (v.as_int() < 0 || (uint64_t)v.as_int() <= hi);
        if (v.type() == json::Value::UINT) return v.as_uint() <= hi;
        return false;
    }

    static bool parse_int64(const std::string& s, int64_t* out) {
        if (s.empty()) return false;
        char* end = nullptr;
        errno = 0;
        const long long x = strtoll(s.c_str(), &end, 10);
        if (errno || *end) return false;
        *out = x;
        return true;
    }
    static bool parse_uint64(const std::string& s, uint64_t* out) {
        if (s.empty() || s[0] == '-') return false;
        char* end = nullptr;
        errno = 0;
        const unsigned long long x = strtoull(s.c_str(), &end, 10);
        if (errno || *end) return false;
        *out = x;
        return true;
    }

    // one value of a scalar (non-message) field
    bool scalar(const json::Value& v, const FieldDescriptor* f, Message* m, bool rep) {
        switch (f->cpp_type()) {
        case CppType::INT32:
            if (!integral(v, INT32_MIN, (uint64_t)INT32_MAX)) return invalid(f, "INT32", v);
            rep ? Reflection::AddInt32(m, f, (int32_t)v.as_int()) : Reflection::SetInt32(m, f, (int32_t)v.as_int());
            return true;
        case CppType::UINT32:
            if (!integral(v, 0, UINT32_MAX)) return invalid(f, "UINT32", v);
            rep ? Reflection::AddUInt32(m, f, (uint32_t)v.as_uint()) : Reflection::SetUInt32(m, f, (uint32_t)v.as_uint());
            return true;
        case CppType::BOOL:
            if (!v.is_bool()) return invalid(f, "BOOL", v);
            rep ? Reflection::AddBool(m, f, v.as_bool()) : Reflection::SetBool(m, f, v.as_bool());
            return true;
        case CppType::INT64: {
            int64_t x = 0;
            if (integral(v, INT64_MIN, (uint64_t)INT64_MAX)) x = v.as_int();
            else if (!(v.is_string() && parse_int64(v.as_string(), &x))) return invalid(f, "INT64", v);
            rep ? Reflection::AddInt64(m, f, x) : Reflection::SetInt64(m, f, x);
            return true;
        }
        case CppType::UINT64: {
            uint64_t x = 0;
            if (integral(v, 0, UINT64_MAX)) x = v.as_uint();
            else if (!(v.is_string() && parse_uint64(v.as_string(), &x))) return invalid(f, "UINT64", v);
            rep ? Reflection::AddUInt64(m, f, x) : Reflection::SetUInt64(m, f, x);
            return true;
        }
        case CppType::FLOAT:
        case CppType::DOUBLE: {
            const bool is_float = f->cpp_type() == CppType::FLOAT;
            double x;
            if (v.is_number()) {
                x = v.as_double();
            } else if (v.is_string()) {
                // only the three special values travel as strings; the
                // reference names the type by its typeid ("f" / "d") here
                const char* t = v.as_string().c_str();
                if (strcasecmp(t, "NaN") == 0) x = NAN;
                else if (strcasecmp(t, "Infinity") == 0) x = INFINITY;
                else if (strcasecmp(t, "-Infinity") == 0) x = -INFINITY;
                else return invalid(f, is_float ? "f" : "d", v);
            } else {
                return invalid(f, is_float ? "float" : "double", v);
            }
            if (is_float) rep ? Reflection::AddFloat(m, f, (float)x) : Reflection::SetFloat(m, f, (float)x);
            else rep ? Reflection::AddDouble(m, f, x) : Reflection::SetDouble(m, f, x);
            return true;
        }
        case CppType::ENUM: {
            const pb::EnumValueDescriptor* ev = nullptr;
            if (f->enum_type && integral(v, INT32_MIN, (uint64_t)INT32_MAX)) {
                ev = f->enum_type->FindValueByNumber((int)v.as_int());
            } else if (f->enum_type && v.is_string()) {
                ev = f->enum_type->FindValueByName(v.as_string());
            }
            if (!ev) return invalid(f, "enum", v);
            rep ? Reflection::AddEnumValue(m, f, ev->number) : Reflection::SetEnumValue(m, f, ev->number);
            return true;
        }
        case CppType::STRING: {
            if (!v.is_string()) return invalid(f, "string", v);
            std::string str = v.as_string();
            if (f->type == pb::FieldType::BYTES && _opt.base64_to_bytes) {
                std::string d;
                if (!base64_decode(str, &d)) {
                    append("Fail to decode base64 string=" + str + " [" + m->GetDescriptor()->name + "]");
                    return false;
                }
                str.swap(d);
            }
            rep ? Reflection::AddString(m, f, str) : Reflection::SetString(m, f, str);
            return true;
        }
        case CppType::MESSAGE:
            break;
        }
        return false;
    }

    // Integers parsed in bulk (json::SetIntArrayOffload) appended without a
    // Value per element; false (nothing appended) when a value is out of the
    // field's range or the type needs the element-wise rules, which then
    // report it exactly as before.
    static bool bulk_ints(const std::vector<int64_t>& xs, const FieldDescriptor* f, Message* m) {
        switch (f->cpp_type()) {
        case CppType::INT32:
            for (int64_t x : xs) {
                if (x < INT32_MIN || x > INT32_MAX) return false;
            }
            for (int64_t x : xs) Reflection::AddInt32(m, f, (int32_t)x);
            return true;
        case CppType::UINT32:
            for (int64_t x : xs) {
                if (x < 0 || x > (int64_t)UINT32_MAX) return false;
            }
            for (int64_t x : xs) Reflection::AddUInt32(m, f, (uint32_t)x);
            return true;
        case CppType::INT64:
            for (int64_t x : xs) Reflection::AddInt64(m, f, x);
            return true;
        case CppType::UINT64:
            for (int64_t x : xs) {
                if (x < 0) return false;
            }
            for (int64_t x : xs) Reflection::AddUInt64(m, f, (uint64_t)x);
            return true;
        default: return false;
        }
    }

    bool field(const json::Value& v, const FieldDescriptor* f, Message* m) {
        if (v.is_null()) {
            if (f->is_required()) {
                append("Missing required field: " + full_name(f));
                return false;
            }
            return true;
        }
        if (f->is_repeated()) {
            if (!v.is_array()) {
                append("Invalid value for repeated field: " + full_name(f));
                return false;
            }
            if (const std::vector<int64_t>* ints = v.packed_ints()) {
                if (bulk_ints(*ints, f, m)) return true;
            }
            for (const json::Value& e : v.array()) {
                if (f->cpp_type() == CppType::MESSAGE) {
                    if (!e.is_object()) {
                        if (!invalid(f, "message", e)) return false;
                        continue;
                    }
                    if (!message(e, Reflection::AddMessage(m, f))) return false;
                } else if (!scalar(e, f, m, true)) {
                    return false;
                }
            }
            return true;
        }
        if (f->cpp_type() == CppType::MESSAGE) return message(v, Reflection::MutableMessage(m, f));
        return scalar(v, f, m, false);
    }

    // {"key": value, ...} into a map field (keys converted to the key type)
    bool map(const json::Value& v, const FieldDescriptor* f, Message* m) {
        const FieldDescriptor* kf = f->message_type->field(0);
        const FieldDescriptor* vf = f->message_type->field(1);
        for (const auto& kv : v.members()) {
            Message* e = Reflection::AddMessage(m, f);
            json::Value key(kv.first);
            if (kf->cpp_type() != CppType::STRING) {
                json::Value parsed;
                if (json::Parse(kv.first, &parsed)) key = parsed;
            }
            if (!scalar(key, kf, e, false)) return false;
            if (!field(kv.second, vf, e)) return false;
        }
        return true;
    }

    const Json2PbOptions& _opt;
    std::string* _err;
};

bool value_to_msg(const json::Value& v, Message* m, const Json2PbOptions& opt, std::string* err) {
    if (err) err->clear();
    return J2P(opt, err).message(v, m);
}

}  // namespace

bool ProtoMessageToJsonValue(const pb::Message& msg, json::Value* out, const Pb2JsonOptions& opt, std::string* error) {
    return msg_to_value(msg, out, opt, error);
}

bool ProtoMessageToJson(const pb::Message& msg, std::string* out, const Pb2JsonOptions& opt, std::string* error) {
    json::Value v;
    if (!msg_to_value(msg, &v, opt, error)) return false;
    *out = v.ToString(opt.pretty_json);
    return true;
}

bool JsonValueToProtoMessage(const json::Value& v, pb::Message* msg, const Json2PbOptions& opt, std::string* error) {
    return value_to_msg(v, msg, opt, error);
}

namespace {
std::atomic<JsonIndexOffload> g_index_offload{nullptr};
size_t g_index_min = (size_t)-1;
}  // namespace

void SetPb2JsonArrayOffload(Pb2JsonArrayOffload fn, size_t min_elems) {
    g_array_offload_min.store(fn ? std::max<size_t>(1, min_elems) : (size_t)-1, std::memory_order_relaxed);
    g_array_offload.store(fn, std::memory_order_release);
}

void SetJsonIndexOffload(JsonIndexOffload fn, size_t min_bytes) {
    g_index_min = min_bytes;
    g_index_offload.store(fn, std::memory_order_release);
}

bool JsonToProtoMessage(const std::string& text, pb::Message* msg, const Json2PbOptions& opt, std::string* error) {
    json::Value v;
    JsonIndexOffload off = g_index_offload.load(std::memory_order_acquire);
    std::vector<uint32_t> index;
    if (off && text.size() >= g_index_min && off(text.data(), text.size(), &index)) {
        if (!json::ParseWithIndex(text.data(), text.size(), index.data(), index.size(), &v, error)) return false;
    } else if (!json::Parse(text, &v, error)) {
        return false;
    }
    return value_to_msg(v, msg, opt, error);
}

bool JsonToProtoMessage(const Buf& text, pb::Message* msg, const Json2PbOptions& opt, std::string* error) {
    return JsonToProtoMessage(text.to_string(), msg, opt, error);
}

}  // namespace json2pb
}  // namespace mrpc
