#include "pb/descriptor.h"

#include <string>

#include "pb/message.h"

namespace mrpc {
namespace pb {

Descriptor::~Descriptor() {
    if (owns_prototype) delete prototype;
}

const char* FieldTypeName(FieldType t) {
    switch (t) {
    case FieldType::DOUBLE: return "double";
    case FieldType::FLOAT: return "float";
    case FieldType::INT64: return "int64";
    case FieldType::UINT64: return "uint64";
    case FieldType::INT32: return "int32";
    case FieldType::FIXED64: return "fixed64";
    case FieldType::FIXED32: return "fixed32";
    case FieldType::BOOL: return "bool";
    case FieldType::STRING: return "string";
    case FieldType::GROUP: return "group";
    case FieldType::MESSAGE: return "message";
    case FieldType::BYTES: return "bytes";
    case FieldType::UINT32: return "uint32";
    case FieldType::ENUM: return "enum";
    case FieldType::SFIXED32: return "sfixed32";
    case FieldType::SFIXED64: return "sfixed64";
    case FieldType::SINT32: return "sint32";
    case FieldType::SINT64: return "sint64";
    }
    return "?";
}

size_t CppTypeSize(CppType t) {
    switch (t) {
    case CppType::INT32:
    case CppType::UINT32:
    case CppType::ENUM:
    case CppType::FLOAT: return 4;
    case CppType::INT64:
    case CppType::UINT64:
    case CppType::DOUBLE: return 8;
    case CppType::BOOL: return 1;
    case CppType::STRING: return sizeof(std::string);
    case CppType::MESSAGE: return sizeof(void*);
    }
    return 8;
}

size_t CppTypeAlign(CppType t) {
    switch (t) {
    case CppType::BOOL: return 1;
    case CppType::INT32:
    case CppType::UINT32:
    case CppType::ENUM:
    case CppType::FLOAT: return 4;
    default: return 8;
    }
}

std::string ToJsonName(const std::string& s) {
    std::string out;
    bool up = false;
    for (char c : s) {
        if (c == '_') {
            up = true;
        } else if (up) {
            out.push_back((char)toupper((unsigned char)c));
            up = false;
        } else {
            out.push_back(c);
        }
    }
    return out;
}

bool FieldDescriptor::is_map() const { return is_repeated() && message_type && message_type->map_entry; }

const EnumValueDescriptor* EnumDescriptor::FindValueByNumber(int n) const {
    for (auto& v : values) {
        if (v.number == n) return &v;
    }
    return nullptr;
}

const EnumValueDescriptor* EnumDescriptor::FindValueByName(const std::string& s) const {
    for (auto& v : values) {
        if (v.name == s) return &v;
    }
    return nullptr;
}

void Descriptor::BuildIndex() {
    _by_number.clear();
    _by_number_sparse.clear();
    _by_name.clear();
    for (size_t i = 0; i < fields.size(); ++i) {
        FieldDescriptor& f = fields[i];
        f.index = (int)i;
        f.containing_type = this;
        if (f.json_name.empty()) f.json_name = ToJsonName(f.name);
        if (f.number > 0 && f.number < 256) {
            if ((int)_by_number.size() <= f.number) _by_number.resize(f.number + 1, 0);
            _by_number[f.number] = (int)i + 1;
        } else {
            _by_number_sparse[f.number] = (int)i;
        }
        _by_name[f.name] = (int)i;
    }
}

const FieldDescriptor* Descriptor::FindFieldByNumber(int n) const {
    if (n > 0 && n < (int)_by_number.size()) {
        int i = _by_number[n];
        return i ? &fields[i - 1] : nullptr;
    }
    auto it = _by_number_sparse.find(n);
    return it == _by_number_sparse.end() ? nullptr : &fields[it->second];
}

const FieldDescriptor* Descriptor::FindFieldByName(const std::string& s) const {
    auto it = _by_name.find(s);
    return it == _by_name.end() ? nullptr : &fields[it->second];
}

const FieldDescriptor* Descriptor::FindFieldByJsonName(const std::string& s) const {
    for (auto& f : fields) {
        if (f.json_name == s) return &f;
    }
    return nullptr;
}

Message* Descriptor::NewMessage() const {
    if (factory) return factory();
    if (prototype) return prototype->New();
    return nullptr;
}

const MethodDescriptor* ServiceDescriptor::FindMethodByName(const std::string& n) const {
    for (auto& m : methods) {
        if (m.name == n) return &m;
    }
    return nullptr;
}

DescriptorPool* DescriptorPool::generated_pool() {
    static DescriptorPool* p = new DescriptorPool;
    return p;
}

void DescriptorPool::add_message(Descriptor* d) {
    _messages[d->full_name] = d;
    for (Descriptor* n : d->nested_types) add_message(n);
    for (EnumDescriptor* e : d->enum_types) _enums[e->full_name] = e;
}

void DescriptorPool::AddFile(FileDescriptor* f) {
    std::lock_guard<std::mutex> g(_mu);
    _files.emplace_back(f);
    _file_by_name[f->name] = f;
    for (Descriptor* d : f->message_types) add_message(d);
    for (EnumDescriptor* e : f->enum_types) _enums[e->full_name] = e;
    for (ServiceDescriptor* s : f->services) _services[s->full_name] = s;
}

const FileDescriptor* DescriptorPool::FindFileByName(const std::string& n) const {
    std::lock_guard<std::mutex> g(_mu);
    auto it = _file_by_name.find(n);
    return it == _file_by_name.end() ? nullptr : it->second;
}

static std::string strip_dot(const std::string& s) { return (!s.empty() && s[0] == '.') ? s.substr(1) : s; }

const Descriptor* DescriptorPool::FindMessageTypeByName(const std::string& n) const {
    std::lock_guard<std::mutex> g(_mu);
    auto it = _messages.find(strip_dot(n));
    return it == _messages.end() ? nullptr : it->second;
}

const EnumDescriptor* DescriptorPool::FindEnumTypeByName(const std::string& n) const {
    std::lock_guard<std::mutex> g(_mu);
    auto it = _enums.find(strip_dot(n));
    return it == _enums.end() ? nullptr : it->second;
}

const ServiceDescriptor* DescriptorPool::FindServiceByName(const std::string& n) const {
    std::lock_guard<std::mutex> g(_mu);
    auto it = _services.find(strip_dot(n));
    return it == _services.end() ? nullptr : it->second;
}

const MethodDescriptor* DescriptorPool::FindMethodByName(const std::string& n) const {
    std::string s = strip_dot(n);
    size_t dot = s.rfind('.');
    if (dot == std::string::npos) return nullptr;
    const ServiceDescriptor* sd = FindServiceByName(s.substr(0, dot));
    return sd ? sd->FindMethodByName(s.substr(dot + 1)) : nullptr;
}

std::vector<const FileDescriptor*> DescriptorPool::files() const {
    std::lock_guard<std::mutex> g(_mu);
    std::vector<const FileDescriptor*> out;
    for (auto& f : _files) out.push_back(f.get());
    return out;
}

std::vector<const ServiceDescriptor*> DescriptorPool::services() const {
    std::lock_guard<std::mutex> g(_mu);
    std::vector<const ServiceDescriptor*> out;
    for (auto& kv : _services) out.push_back(kv.second);
    return out;
}

}  // namespace pb
}  // namespace mrpc
