#include "json/json2pb.h"

#include <atomic>
#include <cmath>

#include "base/util.h"

namespace mrpc {
namespace json2pb {

using pb::CppType;
using pb::FieldDescriptor;
using pb::Message;
using pb::Reflection;

namespace {

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

bool msg_to_value(const Message& m, json::Value* out, const Pb2JsonOptions& opt, std::string* err) {
    *out = json::Value::Object();
    const pb::Descriptor* d = m.GetDescriptor();
    for (const FieldDescriptor& fd : d->fields) {
        const FieldDescriptor* f = &fd;
        const std::string& key = opt.use_json_name ? f->json_name : f->name;
        if (f->is_map()) {
            const int n = Reflection::FieldSize(m, f);
            if (n == 0 && !opt.jsonify_empty_array) continue;
            json::Value obj = json::Value::Object();
            const FieldDescriptor* kf = f->message_type->FindFieldByNumber(1);
            const FieldDescriptor* vf = f->message_type->FindFieldByNumber(2);
            for (int i = 0; i < n; ++i) {
                const Message& e = Reflection::GetRepeatedMessage(m, f, i);
                json::Value k = scalar_to_json(e, kf, -1, opt);
                std::string ks = k.is_string() ? k.as_string() : k.ToString();
                json::Value v;
                if (!field_value(e, vf, -1, &v, opt, err)) return false;
                obj.set(ks, std::move(v));
            }
            out->set(key, std::move(obj));
            continue;
        }
        if (f->is_repeated()) {
            const int n = Reflection::FieldSize(m, f);
            if (n == 0 && !opt.jsonify_empty_array) continue;
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
            if (!opt.always_print_primitive_fields || f->cpp_type() == CppType::MESSAGE) continue;
        }
        json::Value v;
        if (!field_value(m, f, -1, &v, opt, err)) return false;
        out->set(key, std::move(v));
    }
    return true;
}

bool set_scalar(Message* m, const FieldDescriptor* f, const json::Value& v, bool rep, const Json2PbOptions& opt,
                std::string* err) {
    auto bad = [&](const char* what) {
        if (err) *err = "invalid value for field `" + f->name + "': expect " + what;
        return false;
    };
    // integers may arrive quoted (64-bit values from JavaScript): the whole
    // string must be a number
    if (v.is_string() && f->cpp_type() != CppType::STRING && f->cpp_type() != CppType::ENUM &&
        f->cpp_type() != CppType::FLOAT && f->cpp_type() != CppType::DOUBLE) {
        const std::string& s = v.as_string();
        char* end = nullptr;
        if (s.empty()) return bad("number");
        (void)strtod(s.c_str(), &end);
        if (*end != '\0') return bad("number");
    }
    switch (f->cpp_type()) {
    case CppType::INT32: {
        if (!v.is_number() && !v.is_string()) return bad("int32");
        int32_t x = (int32_t)v.as_int();
        rep ? Reflection::AddInt32(m, f, x) : Reflection::SetInt32(m, f, x);
        return true;
    }
    case CppType::INT64: {
        if (!v.is_number() && !v.is_string()) return bad("int64");
        int64_t x = v.as_int();
        rep ? Reflection::AddInt64(m, f, x) : Reflection::SetInt64(m, f, x);
        return true;
    }
    case CppType::UINT32: {
        if (!v.is_number() && !v.is_string()) return bad("uint32");
        uint32_t x = (uint32_t)v.as_uint();
        rep ? Reflection::AddUInt32(m, f, x) : Reflection::SetUInt32(m, f, x);
        return true;
    }
    case CppType::UINT64: {
        if (!v.is_number() && !v.is_string()) return bad("uint64");
        uint64_t x = v.as_uint();
        rep ? Reflection::AddUInt64(m, f, x) : Reflection::SetUInt64(m, f, x);
        return true;
    }
    case CppType::FLOAT:
    case CppType::DOUBLE: {
        double x;
        if (v.is_number()) x = v.as_double();
        else if (v.is_string() && (v.as_string() == "NaN" || v.as_string() == "Infinity" || v.as_string() == "-Infinity"))
            x = v.as_string() == "NaN" ? NAN : (v.as_string()[0] == '-' ? -INFINITY : INFINITY);
        else return bad("number");
        if (f->cpp_type() == CppType::FLOAT) rep ? Reflection::AddFloat(m, f, (float)x) : Reflection::SetFloat(m, f, (float)x);
        else rep ? Reflection::AddDouble(m, f, x) : Reflection::SetDouble(m, f, x);
        return true;
    }
    case CppType::BOOL: {
        if (!v.is_bool() && !v.is_number()) return bad("bool");
        rep ? Reflection::AddBool(m, f, v.as_bool()) : Reflection::SetBool(m, f, v.as_bool());
        return true;
    }
    case CppType::ENUM: {
        int x;
        if (v.is_string()) {
            const pb::EnumValueDescriptor* ev = f->enum_type ? f->enum_type->FindValueByName(v.as_string()) : nullptr;
            if (!ev) return bad("enum name");
            x = ev->number;
        } else if (v.is_number()) {
            x = (int)v.as_int();
        } else {
            return bad("enum");
        }
        rep ? Reflection::AddEnumValue(m, f, x) : Reflection::SetEnumValue(m, f, x);
        return true;
    }
    case CppType::STRING: {
        if (!v.is_string()) return bad("string");
        std::string s = v.as_string();
        if (f->type == pb::FieldType::BYTES && opt.base64_to_bytes) {
            std::string d;
            if (base64_decode(s, &d)) s.swap(d);
        }
        rep ? Reflection::AddString(m, f, s) : Reflection::SetString(m, f, s);
        return true;
    }
    case CppType::MESSAGE: break;
    }
    return false;
}

bool value_to_msg(const json::Value& v, Message* m, const Json2PbOptions& opt, std::string* err);

bool set_field(Message* m, const FieldDescriptor* f, const json::Value& v, const Json2PbOptions& opt, std::string* err) {
    if (v.is_null()) return true;
    if (f->is_map()) {
        if (!v.is_object()) {
            if (err) *err = "field `" + f->name + "' expects an object (map)";
            return false;
        }
        const FieldDescriptor* kf = f->message_type->FindFieldByNumber(1);
        const FieldDescriptor* vf = f->message_type->FindFieldByNumber(2);
        for (auto& kv : v.members()) {
            Message* e = Reflection::AddMessage(m, f);
            json::Value key(kv.first);
            if (kf->cpp_type() != CppType::STRING) {
                json::Value parsed;
                if (json::Parse(kv.first, &parsed)) key = parsed;
            }
            if (!set_scalar(e, kf, key, false, opt, err)) return false;
            if (vf->cpp_type() == CppType::MESSAGE) {
                if (!value_to_msg(kv.second, Reflection::MutableMessage(e, vf), opt, err)) return false;
            } else if (!set_scalar(e, vf, kv.second, false, opt, err)) {
                return false;
            }
        }
        return true;
    }
    if (f->is_repeated()) {
        if (!v.is_array()) {
            if (err) *err = "field `" + f->name + "' expects an array";
            return false;
        }
        for (const json::Value& e : v.array()) {
            if (f->cpp_type() == CppType::MESSAGE) {
                if (!value_to_msg(e, Reflection::AddMessage(m, f), opt, err)) return false;
            } else if (!set_scalar(m, f, e, true, opt, err)) {
                return false;
            }
        }
        return true;
    }
    if (f->cpp_type() == CppType::MESSAGE) return value_to_msg(v, Reflection::MutableMessage(m, f), opt, err);
    return set_scalar(m, f, v, false, opt, err);
}

bool value_to_msg(const json::Value& v, Message* m, const Json2PbOptions& opt, std::string* err) {
    if (!v.is_object()) {
        if (err) *err = "expect a json object for " + m->GetDescriptor()->full_name;
        return false;
    }
    const pb::Descriptor* d = m->GetDescriptor();
    for (auto& kv : v.members()) {
        const FieldDescriptor* f = d->FindFieldByName(kv.first);
        if (!f) f = d->FindFieldByJsonName(kv.first);
        if (!f) {
            if (opt.allow_unknown_fields) continue;
            if (err) *err = "unknown field `" + kv.first + "' in " + d->full_name;
            return false;
        }
        if (!set_field(m, f, kv.second, opt, err)) return false;
    }
    if (!m->IsInitialized()) {
        if (err) *err = "missing required fields: " + m->InitializationErrorString();
        return false;
    }
    return true;
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
