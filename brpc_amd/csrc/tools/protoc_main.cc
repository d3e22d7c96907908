// mrpc_protoc: .proto -> C++ code generator (no protoc in this environment).
// Generates message classes whose storage follows pb/message.h conventions,
// a static descriptor table with offsets (so the table-driven codec,
// reflection, json and /protobufs work on them), enums, and services with
// the Service base + _Stub client (role of protoc's cc_generic_services the
// reference relies on).
//
// Usage: mrpc_protoc --cpp_out=DIR --proto_path=DIR [--include_prefix=P] a.proto ...
//        mrpc_protoc --mcpack_out=DIR --proto_path=DIR a.proto ...   (per-message mcpack codec)
#include <cstdio>
#include <fstream>
#include <functional>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "pb/descriptor.h"
#include "pb/parser.h"

using namespace mrpc::pb;

namespace {

std::string replace_all(std::string s, const std::string& a, const std::string& b) {
    size_t p = 0;
    while ((p = s.find(a, p)) != std::string::npos) {
        s.replace(p, a.size(), b);
        p += b.size();
    }
    return s;
}

std::string ns_of(const std::string& package) { return package.empty() ? "" : "::" + replace_all(package, ".", "::"); }

std::string local_name(const std::string& full_name, const std::string& package) {
    std::string rel = package.empty() ? full_name : full_name.substr(package.size() + 1);
    return replace_all(rel, ".", "_");
}

std::string cpp_class(const Descriptor* d) { return ns_of(d->file->package) + "::" + local_name(d->full_name, d->file->package); }
std::string cpp_enum(const EnumDescriptor* e) { return ns_of(e->file->package) + "::" + local_name(e->full_name, e->file->package); }

std::string basename_noext(const std::string& path) {
    std::string b = path;
    size_t s = b.rfind('/');
    if (s != std::string::npos) b = b.substr(s + 1);
    if (b.size() > 6 && b.compare(b.size() - 6, 6, ".proto") == 0) b = b.substr(0, b.size() - 6);
    return b;
}

std::string ident_of(const std::string& path) {
    std::string b = path;
    for (auto& c : b) {
        if (!isalnum((unsigned char)c)) c = '_';
    }
    return b;
}

std::string scalar_cpp(const FieldDescriptor& f) {
    switch (f.cpp_type()) {
    case CppType::INT32: return "int32_t";
    case CppType::INT64: return "int64_t";
    case CppType::UINT32: return "uint32_t";
    case CppType::UINT64: return "uint64_t";
    case CppType::DOUBLE: return "double";
    case CppType::FLOAT: return "float";
    case CppType::BOOL: return "bool";
    case CppType::ENUM: return cpp_enum(f.enum_type);
    case CppType::STRING: return "std::string";
    case CppType::MESSAGE: return cpp_class(f.message_type);
    }
    return "?";
}

std::string storage_cpp(const FieldDescriptor& f) {
    if (f.is_repeated()) {
        switch (f.cpp_type()) {
        case CppType::BOOL: return "std::vector<uint8_t>";
        case CppType::ENUM: return "std::vector<int32_t>";
        case CppType::STRING: return "std::vector<std::string>";
        case CppType::MESSAGE: return "::mrpc::pb::RepeatedPtrField<" + cpp_class(f.message_type) + ">";
        default: return "std::vector<" + scalar_cpp(f) + ">";
        }
    }
    switch (f.cpp_type()) {
    case CppType::ENUM: return "int32_t";
    case CppType::MESSAGE: return "::mrpc::pb::Message*";
    default: return scalar_cpp(f);
    }
}

std::string default_literal(const FieldDescriptor& f) {
    char b[64];
    switch (f.cpp_type()) {
    case CppType::INT32:
    case CppType::ENUM: snprintf(b, sizeof(b), "%lld", (long long)f.default_int); return std::string("int32_t(") + b + ")";
    case CppType::INT64: snprintf(b, sizeof(b), "%lldLL", (long long)f.default_int); return std::string("int64_t(") + b + ")";
    case CppType::UINT32: snprintf(b, sizeof(b), "%lluu", (unsigned long long)f.default_uint); return b;
    case CppType::UINT64: snprintf(b, sizeof(b), "%lluULL", (unsigned long long)f.default_uint); return b;
    case CppType::DOUBLE:
    case CppType::FLOAT:
        if (f.default_double != f.default_double) return "(0.0/0.0)";
        if (f.default_double == 1.0 / 0.0) return "(1.0/0.0)";
        if (f.default_double == -1.0 / 0.0) return "(-1.0/0.0)";
        snprintf(b, sizeof(b), "%.17g", f.default_double);
        return std::string(f.cpp_type() == CppType::FLOAT ? "float(" : "double(") + b + ")";
    case CppType::BOOL: return f.default_int ? "true" : "false";
    default: return "";
    }
}

std::string cstr_literal(const std::string& s) {
    std::string out = "\"";
    for (unsigned char c : s) {
        char b[8];
        if (c == '"' || c == '\\') {
            out.push_back('\\');
            out.push_back((char)c);
        } else if (c < 0x20 || c >= 0x7f) {
            snprintf(b, sizeof(b), "\\%03o", c);
            out += b;
        } else {
            out.push_back((char)c);
        }
    }
    return out + "\"";
}

struct Gen {
    const FileDescriptor* file;
    std::string prefix;
    std::ostringstream h, c, hi;
    std::vector<const Descriptor*> msgs;  // all, pre-order
    std::vector<const EnumDescriptor*> enums;
    std::string fid;

    void collect(const Descriptor* d) {
        msgs.push_back(d);
        for (const EnumDescriptor* e : d->enum_types) enums.push_back(e);
        for (const Descriptor* n : d->nested_types) collect(n);
    }

    int msg_index(const Descriptor* d) const {
        for (size_t i = 0; i < msgs.size(); ++i) {
            if (msgs[i] == d) return (int)i;
        }
        return -1;
    }
    int enum_index(const EnumDescriptor* e) const {
        for (size_t i = 0; i < enums.size(); ++i) {
            if (enums[i] == e) return (int)i;
        }
        return -1;
    }

    void open_ns(std::ostringstream& o) {
        if (file->package.empty()) return;
        std::stringstream ss(file->package);
        std::string part;
        while (std::getline(ss, part, '.')) o << "namespace " << part << " {\n";
    }
    void close_ns(std::ostringstream& o) {
        if (file->package.empty()) return;
        std::stringstream ss(file->package);
        std::string part;
        while (std::getline(ss, part, '.')) o << "}  // namespace\n";
    }

    void gen_enum_decl(const EnumDescriptor* e) {
        std::string n = local_name(e->full_name, file->package);
        h << "enum " << n << " : int {\n";
        std::set<int> seen;
        for (auto& v : e->values) {
            std::string vn = is_nested_enum(e) ? n + "_" + v.name : v.name;
            h << "  " << vn << " = " << v.number << ",\n";
        }
        h << "};\n";
        h << "const ::mrpc::pb::EnumDescriptor* " << n << "_descriptor();\n";
        h << "bool " << n << "_IsValid(int value);\n";
        h << "const std::string& " << n << "_Name(int value);\n";
        h << "bool " << n << "_Parse(const std::string& name, " << n << "* value);\n\n";
    }

    bool is_nested_enum(const EnumDescriptor* e) const {
        std::string top = file->package.empty() ? e->name : file->package + "." + e->name;
        return e->full_name != top;
    }

    void gen_enum_impl(const EnumDescriptor* e) {
        std::string n = local_name(e->full_name, file->package);
        c << "const ::mrpc::pb::EnumDescriptor* " << n << "_descriptor() { return " << fid << "_file()->enums["
          << enum_index(e) << "]; }\n";
        c << "bool " << n << "_IsValid(int value) { return " << n << "_descriptor()->FindValueByNumber(value) != nullptr; }\n";
        c << "const std::string& " << n << "_Name(int value) {\n"
          << "  static const std::string empty;\n"
          << "  const ::mrpc::pb::EnumValueDescriptor* v = " << n << "_descriptor()->FindValueByNumber(value);\n"
          << "  return v ? v->name : empty;\n}\n";
        c << "bool " << n << "_Parse(const std::string& name, " << n << "* value) {\n"
          << "  const ::mrpc::pb::EnumValueDescriptor* v = " << n << "_descriptor()->FindValueByName(name);\n"
          << "  if (!v) return false;\n  *value = (" << n << ")v->number;\n  return true;\n}\n\n";
    }

    void gen_class_decl(const Descriptor* d) {
        std::string cn = local_name(d->full_name, file->package);
        h << "class " << cn << " : public ::mrpc::pb::Message {\n public:\n";
        h << "  " << cn << "();\n  ~" << cn << "() override;\n";
        h << "  " << cn << "(const " << cn << "& from);\n";
        h << "  " << cn << "& operator=(const " << cn << "& from);\n";
        h << "  static const ::mrpc::pb::Descriptor* descriptor();\n";
        h << "  static const " << cn << "& default_instance();\n";
        h << "  const ::mrpc::pb::Descriptor* GetDescriptor() const override { return descriptor(); }\n";
        h << "  " << cn << "* New() const override { return new " << cn << "; }\n";
        h << "  void Swap(" << cn << "* other);\n";
        for (const Descriptor* n : d->nested_types) {
            h << "  typedef " << local_name(n->full_name, file->package) << " " << n->name << ";\n";
        }
        for (const EnumDescriptor* e : d->enum_types) {
            std::string en = local_name(e->full_name, file->package);
            h << "  typedef " << en << " " << e->name << ";\n";
            for (auto& v : e->values) h << "  static const " << en << " " << v.name << " = " << en << "_" << v.name << ";\n";
            h << "  static bool " << e->name << "_IsValid(int v) { return " << en << "_IsValid(v); }\n";
            h << "  static const std::string& " << e->name << "_Name(int v) { return " << en << "_Name(v); }\n";
        }
        for (const FieldDescriptor& f : d->fields) gen_accessors_decl(d, f);
        // storage
        h << "\n  // storage (public so that the descriptor table can use offsetof)\n";
        int nbits = 0;
        for (const FieldDescriptor& f : d->fields) {
            if (has_bit_for(f)) ++nbits;
        }
        h << "  uint32_t _has_bits_[" << std::max(1, (nbits + 31) / 32) << "];\n";
        for (const FieldDescriptor& f : d->fields) h << "  " << storage_cpp(f) << " " << f.name << "_;\n";
        h << "};\n\n";
    }

    static bool has_bit_for(const FieldDescriptor& f) {
        return !f.is_repeated() && f.cpp_type() != CppType::MESSAGE && !f.proto3_implicit;
    }

    void gen_accessors_decl(const Descriptor* d, const FieldDescriptor& f) {
        std::string n = f.name;
        std::string kname = "k";
        bool up = true;
        for (char ch : n) {
            if (ch == '_') {
                up = true;
                continue;
            }
            kname.push_back(up ? (char)toupper((unsigned char)ch) : ch);
            up = false;
        }
        h << "  static const int " << kname << "FieldNumber = " << f.number << ";\n";
        const std::string fidx = std::to_string(f.index);
        const std::string fdesc = "descriptor()->field(" + fidx + ")";
        const std::string T = scalar_cpp(f);
        if (f.is_repeated()) {
            h << "  int " << n << "_size() const { return (int)" << n << "_.size(); }\n";
            h << "  void clear_" << n << "() { " << n << "_." << (f.cpp_type() == CppType::MESSAGE ? "Clear" : "clear") << "(); }\n";
            switch (f.cpp_type()) {
            case CppType::MESSAGE:
                h << "  const " << T << "& " << n << "(int i) const { return " << n << "_.Get(i); }\n";
                h << "  " << T << "* mutable_" << n << "(int i) { return " << n << "_.Mutable(i); }\n";
                h << "  " << T << "* add_" << n << "() { return " << n << "_.Add(); }\n";
                h << "  const ::mrpc::pb::RepeatedPtrField<" << T << ">& " << n << "() const { return " << n << "_; }\n";
                h << "  ::mrpc::pb::RepeatedPtrField<" << T << ">* mutable_" << n << "() { return &" << n << "_; }\n";
                break;
            case CppType::STRING:
                h << "  const std::string& " << n << "(int i) const { return " << n << "_[i]; }\n";
                h << "  std::string* mutable_" << n << "(int i) { return &" << n << "_[i]; }\n";
                h << "  void set_" << n << "(int i, const std::string& v) { " << n << "_[i] = v; }\n";
                h << "  void add_" << n << "(const std::string& v) { " << n << "_.push_back(v); }\n";
                h << "  void add_" << n << "(const char* v, size_t len) { " << n << "_.emplace_back(v, len); }\n";
                h << "  std::string* add_" << n << "() { " << n << "_.emplace_back(); return &" << n << "_.back(); }\n";
                h << "  const std::vector<std::string>& " << n << "() const { return " << n << "_; }\n";
                h << "  std::vector<std::string>* mutable_" << n << "() { return &" << n << "_; }\n";
                break;
            default: {
                std::string S = storage_cpp(f);
                h << "  " << T << " " << n << "(int i) const { return (" << T << ")" << n << "_[i]; }\n";
                h << "  void set_" << n << "(int i, " << T << " v) { " << n << "_[i] = v; }\n";
                h << "  void add_" << n << "(" << T << " v) { " << n << "_.push_back(v); }\n";
                h << "  const " << S << "& " << n << "() const { return " << n << "_; }\n";
                h << "  " << S << "* mutable_" << n << "() { return &" << n << "_; }\n";
            }
            }
            return;
        }
        const bool hb = has_bit_for(f);
        int bit = -1;
        if (hb) {
            int k = 0;
            for (const FieldDescriptor& o : d->fields) {
                if (&o == &f) break;
                if (has_bit_for(o)) ++k;
            }
            bit = k;
        }
        const std::string set_has = hb ? "_has_bits_[" + std::to_string(bit / 32) + "] |= " + std::to_string(1u << (bit % 32)) + "u; " : "";
        const std::string clr_has = hb ? "_has_bits_[" + std::to_string(bit / 32) + "] &= ~" + std::to_string(1u << (bit % 32)) + "u; " : "";
        const std::string oneof = f.oneof_index >= 0 ? "::mrpc::pb::ClearOneofSiblings(this, " + fdesc + "); " : "";
        switch (f.cpp_type()) {
        case CppType::MESSAGE: {
            // Bodies need the complete sub-message type: defined after all classes.
            const std::string cls = local_name(d->full_name, file->package);
            h << "  bool has_" << n << "() const { return " << n << "_ != nullptr; }\n";
            h << "  void clear_" << n << "() { delete " << n << "_; " << n << "_ = nullptr; }\n";
            h << "  const " << T << "& " << n << "() const;\n";
            h << "  " << T << "* mutable_" << n << "();\n";
            h << "  " << T << "* release_" << n << "();\n";
            h << "  void set_allocated_" << n << "(" << T << "* p);\n";
            hi << "inline const " << T << "& " << cls << "::" << n << "() const { return " << n << "_ ? *static_cast<const " << T
               << "*>(" << n << "_) : " << T << "::default_instance(); }\n";
            hi << "inline " << T << "* " << cls << "::mutable_" << n << "() { if (!" << n << "_) { " << oneof << n << "_ = new " << T
               << "; } return static_cast<" << T << "*>(" << n << "_); }\n";
            hi << "inline " << T << "* " << cls << "::release_" << n << "() { " << T << "* p = static_cast<" << T << "*>(" << n
               << "_); " << n << "_ = nullptr; return p; }\n";
            hi << "inline void " << cls << "::set_allocated_" << n << "(" << T << "* p) { delete " << n << "_; if (p) { " << oneof
               << "} " << n << "_ = p; }\n";
            break;
        }
        case CppType::STRING:
            if (hb) h << "  bool has_" << n << "() const { return (_has_bits_[" << bit / 32 << "] >> " << bit % 32 << ") & 1; }\n";
            else h << "  bool has_" << n << "() const { return !" << n << "_.empty(); }\n";
            h << "  void clear_" << n << "() { " << n << "_ = " << cstr_literal(f.default_string) << "; " << clr_has << "}\n";
            h << "  const std::string& " << n << "() const { return " << n << "_; }\n";
            h << "  void set_" << n << "(const std::string& v) { " << oneof << n << "_ = v; " << set_has << "}\n";
            h << "  void set_" << n << "(std::string&& v) { " << oneof << n << "_ = std::move(v); " << set_has << "}\n";
            h << "  void set_" << n << "(const char* v) { " << oneof << n << "_ = v; " << set_has << "}\n";
            h << "  void set_" << n << "(const void* v, size_t len) { " << oneof << n << "_.assign((const char*)v, len); " << set_has << "}\n";
            h << "  std::string* mutable_" << n << "() { " << oneof << set_has << "return &" << n << "_; }\n";
            break;
        default: {
            std::string zero = default_literal(f);
            if (hb) h << "  bool has_" << n << "() const { return (_has_bits_[" << bit / 32 << "] >> " << bit % 32 << ") & 1; }\n";
            else h << "  bool has_" << n << "() const { return " << n << "_ != " << (f.cpp_type() == CppType::ENUM ? "0" : zero) << "; }\n";
            h << "  void clear_" << n << "() { " << n << "_ = " << zero << "; " << clr_has << "}\n";
            h << "  " << T << " " << n << "() const { return (" << T << ")" << n << "_; }\n";
            h << "  void set_" << n << "(" << T << " v) { " << oneof << n << "_ = v; " << set_has << "}\n";
        }
        }
    }

    void gen_class_impl(const Descriptor* d) {
        std::string cn = local_name(d->full_name, file->package);
        // ctor
        c << cn << "::" << cn << "() {\n  memset(_has_bits_, 0, sizeof(_has_bits_));\n";
        for (const FieldDescriptor& f : d->fields) {
            if (f.is_repeated()) continue;
            if (f.cpp_type() == CppType::MESSAGE) c << "  " << f.name << "_ = nullptr;\n";
            else if (f.cpp_type() == CppType::STRING) {
                if (!f.default_string.empty()) c << "  " << f.name << "_ = " << cstr_literal(f.default_string) << ";\n";
            } else {
                c << "  " << f.name << "_ = " << default_literal(f) << ";\n";
            }
        }
        c << "}\n";
        c << cn << "::~" << cn << "() {\n";
        for (const FieldDescriptor& f : d->fields) {
            if (!f.is_repeated() && f.cpp_type() == CppType::MESSAGE) c << "  delete " << f.name << "_;\n";
        }
        c << "}\n";
        c << cn << "::" << cn << "(const " << cn << "& from) : " << cn << "() { MergeFrom(from); }\n";
        c << cn << "& " << cn << "::operator=(const " << cn << "& from) { CopyFrom(from); return *this; }\n";
        c << "void " << cn << "::Swap(" << cn << "* other) { " << cn << " tmp(*this); CopyFrom(*other); other->CopyFrom(tmp); }\n";
        c << "const ::mrpc::pb::Descriptor* " << cn << "::descriptor() { return " << fid << "_file()->msgs[" << msg_index(d)
          << "]; }\n";
        c << "const " << cn << "& " << cn << "::default_instance() { static const " << cn << "* d = new " << cn
          << "; return *d; }\n\n";
    }

    void gen_descriptor_build() {
        c << "namespace {\n";
        c << "struct " << fid << "_File {\n  ::mrpc::pb::FileDescriptor* file;\n  ::mrpc::pb::Descriptor* msgs["
          << std::max<size_t>(1, msgs.size()) << "];\n  ::mrpc::pb::EnumDescriptor* enums["
          << std::max<size_t>(1, enums.size()) << "];\n  ::mrpc::pb::ServiceDescriptor* services["
          << std::max<size_t>(1, file->services.size()) << "];\n};\n";
        c << fid << "_File* " << fid << "_build();\n";
        c << fid << "_File* " << fid << "_file() { static " << fid << "_File* f = " << fid << "_build(); return f; }\n";
        c << "}  // namespace\n\n";
    }

    void gen_build_fn() {
        c << "namespace {\n" << fid << "_File* " << fid << "_build() {\n";
        c << "  " << fid << "_File* r = new " << fid << "_File;\n";
        c << "  ::mrpc::pb::FileDescriptor* f = new ::mrpc::pb::FileDescriptor;\n  r->file = f;\n";
        c << "  f->name = " << cstr_literal(file->name) << ";\n  f->package = " << cstr_literal(file->package) << ";\n";
        c << "  f->syntax = " << cstr_literal(file->syntax) << ";\n";
        c << "  f->source = " << cstr_literal(file->source) << ";\n";
        for (auto& dep : file->dependencies) c << "  f->dependencies.push_back(" << cstr_literal(dep) << ");\n";
        // enums
        for (size_t i = 0; i < enums.size(); ++i) {
            const EnumDescriptor* e = enums[i];
            c << "  {\n    ::mrpc::pb::EnumDescriptor* e = new ::mrpc::pb::EnumDescriptor;\n";
            c << "    e->name = " << cstr_literal(e->name) << "; e->full_name = " << cstr_literal(e->full_name) << "; e->file = f;\n";
            for (auto& v : e->values) c << "    e->values.push_back({" << cstr_literal(v.name) << ", " << v.number << "});\n";
            c << "    r->enums[" << i << "] = e;\n  }\n";
        }
        for (size_t i = 0; i < msgs.size(); ++i) c << "  r->msgs[" << i << "] = new ::mrpc::pb::Descriptor;\n";
        for (size_t i = 0; i < msgs.size(); ++i) {
            const Descriptor* d = msgs[i];
            std::string cn = local_name(d->full_name, file->package);
            c << "  {\n    ::mrpc::pb::Descriptor* d = r->msgs[" << i << "];\n";
            c << "    d->name = " << cstr_literal(d->name) << "; d->full_name = " << cstr_literal(d->full_name)
              << "; d->file = f;\n";
            c << "    d->map_entry = " << (d->map_entry ? "true" : "false") << "; d->proto3 = " << (d->proto3 ? "true" : "false") << ";\n";
            if (d->containing_type) c << "    d->containing_type = r->msgs[" << msg_index(d->containing_type) << "];\n";
            for (auto& on : d->oneof_names) c << "    d->oneof_names.push_back(" << cstr_literal(on) << ");\n";
            for (const Descriptor* n : d->nested_types) c << "    d->nested_types.push_back(r->msgs[" << msg_index(n) << "]);\n";
            for (const EnumDescriptor* e : d->enum_types) c << "    d->enum_types.push_back(r->enums[" << enum_index(e) << "]);\n";
            c << "    d->has_bits_offset = offsetof(" << cn << ", _has_bits_);\n";
            c << "    d->object_size = sizeof(" << cn << ");\n";
            c << "    d->factory = []() -> ::mrpc::pb::Message* { return new " << cn << "; };\n";
            int bit = 0;
            for (const FieldDescriptor& fd : d->fields) {
                c << "    {\n      ::mrpc::pb::FieldDescriptor x;\n";
                c << "      x.name = " << cstr_literal(fd.name) << "; x.json_name = " << cstr_literal(fd.json_name) << ";\n";
                c << "      x.number = " << fd.number << "; x.type = (::mrpc::pb::FieldType)" << (int)fd.type
                  << "; x.label = (::mrpc::pb::Label)" << (int)fd.label << ";\n";
                c << "      x.packed = " << (fd.packed ? "true" : "false") << "; x.proto3_implicit = "
                  << (fd.proto3_implicit ? "true" : "false") << "; x.oneof_index = " << fd.oneof_index << ";\n";
                c << "      x.type_name = " << cstr_literal(fd.type_name) << ";\n";
                if (fd.message_type) {
                    int mi = msg_index(fd.message_type);
                    if (mi >= 0) c << "      x.message_type = r->msgs[" << mi << "];\n";
                    else c << "      x.message_type = " << cpp_class(fd.message_type) << "::descriptor();\n";
                }
                if (fd.enum_type) {
                    int ei = enum_index(fd.enum_type);
                    if (ei >= 0) c << "      x.enum_type = r->enums[" << ei << "];\n";
                    else c << "      x.enum_type = " << cpp_enum(fd.enum_type) << "_descriptor();\n";
                }
                c << "      x.has_default = " << (fd.has_default ? "true" : "false") << "; x.default_str = " << cstr_literal(fd.default_str) << ";\n";
                c << "      x.default_int = " << fd.default_int << "LL; x.default_uint = " << fd.default_uint << "ULL;\n";
                if (fd.cpp_type() == CppType::DOUBLE || fd.cpp_type() == CppType::FLOAT) c << "      x.default_double = " << default_literal(fd) << ";\n";
                c << "      x.default_string = " << cstr_literal(fd.default_string) << ";\n";
                for (auto& kv : fd.options) c << "      x.options[" << cstr_literal(kv.first) << "] = " << cstr_literal(kv.second) << ";\n";
                c << "      x.offset = offsetof(" << cn << ", " << fd.name << "_);\n";
                if (has_bit_for(fd)) c << "      x.has_bit = " << bit++ << ";\n";
                c << "      d->fields.push_back(x);\n    }\n";
            }
            c << "    d->num_has_bits = " << bit << ";\n";
            c << "    d->BuildIndex();\n";
            c << "    d->prototype = &" << cn << "::default_instance();\n";
            c << "  }\n";
        }
        for (const Descriptor* d : file->message_types) c << "  f->message_types.push_back(r->msgs[" << msg_index(d) << "]);\n";
        for (const EnumDescriptor* e : file->enum_types) c << "  f->enum_types.push_back(r->enums[" << enum_index(e) << "]);\n";
        for (size_t si = 0; si < file->services.size(); ++si) {
            const ServiceDescriptor* s = file->services[si];
            c << "  {\n    ::mrpc::pb::ServiceDescriptor* s = new ::mrpc::pb::ServiceDescriptor;\n";
            c << "    s->name = " << cstr_literal(s->name) << "; s->full_name = " << cstr_literal(s->full_name) << "; s->file = f;\n";
            for (auto& kv : s->options) c << "    s->options[" << cstr_literal(kv.first) << "] = " << cstr_literal(kv.second) << ";\n";
            for (const MethodDescriptor& m : s->methods) {
                c << "    {\n      ::mrpc::pb::MethodDescriptor m;\n";
                c << "      m.name = " << cstr_literal(m.name) << "; m.full_name = " << cstr_literal(m.full_name)
                  << "; m.index = " << m.index << ";\n";
                c << "      m.input_type_name = " << cstr_literal(m.input_type->full_name) << "; m.output_type_name = "
                  << cstr_literal(m.output_type->full_name) << ";\n";
                int ii = msg_index(m.input_type), oi = msg_index(m.output_type);
                c << "      m.input_type = " << (ii >= 0 ? "r->msgs[" + std::to_string(ii) + "]" : cpp_class(m.input_type) + "::descriptor()") << ";\n";
                c << "      m.output_type = " << (oi >= 0 ? "r->msgs[" + std::to_string(oi) + "]" : cpp_class(m.output_type) + "::descriptor()") << ";\n";
                c << "      m.client_streaming = " << (m.client_streaming ? "true" : "false") << "; m.server_streaming = "
                  << (m.server_streaming ? "true" : "false") << ";\n";
                for (auto& kv : m.options) c << "      m.options[" << cstr_literal(kv.first) << "] = " << cstr_literal(kv.second) << ";\n";
                c << "      s->methods.push_back(m);\n    }\n";
            }
            c << "    for (auto& m : s->methods) m.service = s;\n";
            c << "    f->services.push_back(s);\n    r->services[" << si << "] = s;\n  }\n";
        }
        c << "  ::mrpc::pb::DescriptorPool::generated_pool()->AddFile(f);\n";
        c << "  return r;\n}\n";
        c << "struct " << fid << "_StaticInit { " << fid << "_StaticInit() { " << fid << "_file(); } } " << fid
          << "_static_init;\n";
        c << "}  // namespace\n\n";
    }

    void gen_service_decl(const ServiceDescriptor* s) {
        h << "class " << s->name << "_Stub;\n";
        h << "class " << s->name << " : public ::mrpc::Service {\n protected:\n  " << s->name << "() {}\n public:\n";
        h << "  typedef " << s->name << "_Stub Stub;\n";
        h << "  ~" << s->name << "() override {}\n";
        h << "  static const ::mrpc::pb::ServiceDescriptor* descriptor();\n";
        h << "  const ::mrpc::pb::ServiceDescriptor* GetDescriptor() override { return descriptor(); }\n";
        for (const MethodDescriptor& m : s->methods) {
            h << "  virtual void " << m.name << "(::mrpc::RpcController* controller, const " << cpp_class(m.input_type)
              << "* request, " << cpp_class(m.output_type) << "* response, ::mrpc::Closure* done);\n";
        }
        h << "  void CallMethod(const ::mrpc::pb::MethodDescriptor* method, ::mrpc::RpcController* controller,\n"
          << "                  const ::mrpc::pb::Message* request, ::mrpc::pb::Message* response, ::mrpc::Closure* done) override;\n";
        h << "  const ::mrpc::pb::Message& GetRequestPrototype(const ::mrpc::pb::MethodDescriptor* method) const override;\n";
        h << "  const ::mrpc::pb::Message& GetResponsePrototype(const ::mrpc::pb::MethodDescriptor* method) const override;\n";
        h << "};\n\n";
        h << "class " << s->name << "_Stub : public " << s->name << " {\n public:\n";
        h << "  explicit " << s->name << "_Stub(::mrpc::RpcChannel* channel) : channel_(channel) {}\n";
        h << "  ::mrpc::RpcChannel* channel() { return channel_; }\n";
        for (const MethodDescriptor& m : s->methods) {
            h << "  void " << m.name << "(::mrpc::RpcController* controller, const " << cpp_class(m.input_type)
              << "* request, " << cpp_class(m.output_type) << "* response, ::mrpc::Closure* done) override;\n";
        }
        h << " private:\n  ::mrpc::RpcChannel* channel_;\n};\n\n";
    }

    void gen_service_impl(const ServiceDescriptor* s, int si) {
        c << "const ::mrpc::pb::ServiceDescriptor* " << s->name << "::descriptor() { return " << fid << "_file()->services[" << si << "]; }\n";
        for (const MethodDescriptor& m : s->methods) {
            c << "void " << s->name << "::" << m.name << "(::mrpc::RpcController* controller, const " << cpp_class(m.input_type)
              << "*, " << cpp_class(m.output_type) << "*, ::mrpc::Closure* done) {\n"
              << "  controller->SetFailed(\"Method " << m.name << "() not implemented.\");\n  done->Run();\n}\n";
        }
        c << "void " << s->name << "::CallMethod(const ::mrpc::pb::MethodDescriptor* method, ::mrpc::RpcController* controller,\n"
          << "    const ::mrpc::pb::Message* request, ::mrpc::pb::Message* response, ::mrpc::Closure* done) {\n"
          << "  switch (method->index) {\n";
        for (const MethodDescriptor& m : s->methods) {
            c << "  case " << m.index << ": " << m.name << "(controller, static_cast<const " << cpp_class(m.input_type)
              << "*>(request), static_cast<" << cpp_class(m.output_type) << "*>(response), done); break;\n";
        }
        c << "  default: controller->SetFailed(\"bad method index\"); done->Run();\n  }\n}\n";
        c << "const ::mrpc::pb::Message& " << s->name << "::GetRequestPrototype(const ::mrpc::pb::MethodDescriptor* method) const {\n"
          << "  switch (method->index) {\n";
        for (const MethodDescriptor& m : s->methods) c << "  case " << m.index << ": return " << cpp_class(m.input_type) << "::default_instance();\n";
        c << "  default: return *method->input_type->prototype;\n  }\n}\n";
        c << "const ::mrpc::pb::Message& " << s->name << "::GetResponsePrototype(const ::mrpc::pb::MethodDescriptor* method) const {\n"
          << "  switch (method->index) {\n";
        for (const MethodDescriptor& m : s->methods) c << "  case " << m.index << ": return " << cpp_class(m.output_type) << "::default_instance();\n";
        c << "  default: return *method->output_type->prototype;\n  }\n}\n";
        for (const MethodDescriptor& m : s->methods) {
            c << "void " << s->name << "_Stub::" << m.name << "(::mrpc::RpcController* controller, const " << cpp_class(m.input_type)
              << "* request, " << cpp_class(m.output_type) << "* response, ::mrpc::Closure* done) {\n"
              << "  channel_->CallMethod(descriptor()->method(" << m.index << "), controller, request, response, done);\n}\n";
        }
        c << "\n";
    }

    void run(const std::string& base) {
        fid = "mrpc_pb_" + ident_of(base);
        for (const Descriptor* d : file->message_types) collect(d);
        for (const EnumDescriptor* e : file->enum_types) enums.insert(enums.begin(), e);
        // keep top-level enums first but preserve nested order after
        std::string guard = "MRPC_PB_" + ident_of(base) + "_H";
        h << "// Generated by mrpc_protoc from " << file->name << ". DO NOT EDIT.\n";
        h << "#pragma once\n#include <cstdint>\n#include <string>\n#include <vector>\n";
        h << "#include \"pb/message.h\"\n#include \"pb/service.h\"\n";
        for (auto& dep : file->dependencies) {
            if (dep.compare(0, 16, "google/protobuf/") == 0) continue;
            h << "#include \"" << prefix << basename_noext(dep) << ".pb.h\"\n";
        }
        h << "\n";
        open_ns(h);
        for (const Descriptor* d : msgs) h << "class " << local_name(d->full_name, file->package) << ";\n";
        h << "\n";
        for (const EnumDescriptor* e : enums) gen_enum_decl(e);
        // classes: nested types must be declared before their containers
        std::vector<const Descriptor*> order;
        std::function<void(const Descriptor*)> post = [&](const Descriptor* d) {
            for (const Descriptor* n : d->nested_types) post(n);
            order.push_back(d);
        };
        for (const Descriptor* d : file->message_types) post(d);
        for (const Descriptor* d : order) gen_class_decl(d);
        h << hi.str() << "\n";
        for (const ServiceDescriptor* s : file->services) gen_service_decl(s);
        close_ns(h);

        c << "// Generated by mrpc_protoc from " << file->name << ". DO NOT EDIT.\n";
        c << "#include \"" << prefix << base << ".pb.h\"\n#include <cstddef>\n#include <cstring>\n\n";
        open_ns(c);
        gen_descriptor_build();
        for (const EnumDescriptor* e : enums) gen_enum_impl(e);
        for (const Descriptor* d : msgs) gen_class_impl(d);
        for (size_t i = 0; i < file->services.size(); ++i) gen_service_impl(file->services[i], (int)i);
        gen_build_fn();
        close_ns(c);
    }
};


// ------------------------------------------------------------ --mcpack_out
// Per-message mcpack codec (role of the reference's protoc-gen-mcpack,
// src/mcpack2pb/generator.cpp): straight-line serialize/parse functions
// over the generated accessors, registered as the message's
// mcpack::MessageHandler. Wire types and names follow the same rules as the
// descriptor-driven codec (mcpack/mcpack.cc: idl_name / idl_type options).
std::string mc_option(const FieldDescriptor& f, const char* key) {
    auto it = f.options.find(std::string("(") + key + ")");
    if (it == f.options.end()) it = f.options.find(key);
    if (it == f.options.end()) return std::string();
    std::string v = it->second;
    if (v.size() >= 2 && (v[0] == '"' || v[0] == '\'') && v.back() == v[0]) v = v.substr(1, v.size() - 2);
    return v;
}

std::string mc_wire_type(const FieldDescriptor& f) {
    const std::string idl = mc_option(f, "idl_type");
    static const char* kIdl[][2] = {
        {"IDL_INT8", "FIELD_INT8"},     {"IDL_INT16", "FIELD_INT16"},   {"IDL_INT32", "FIELD_INT32"},
        {"IDL_INT64", "FIELD_INT64"},   {"IDL_UINT8", "FIELD_UINT8"},   {"IDL_UINT16", "FIELD_UINT16"},
        {"IDL_UINT32", "FIELD_UINT32"}, {"IDL_UINT64", "FIELD_UINT64"}, {"IDL_BOOL", "FIELD_BOOL"},
        {"IDL_FLOAT", "FIELD_FLOAT"},   {"IDL_DOUBLE", "FIELD_DOUBLE"}, {"IDL_BINARY", "FIELD_BINARY"},
        {"IDL_STRING", "FIELD_STRING"},
    };
    for (auto& k : kIdl) {
        if (idl == k[0]) return k[1];
    }
    switch (f.type) {
    case FieldType::INT32: case FieldType::SINT32: case FieldType::SFIXED32: case FieldType::ENUM: return "FIELD_INT32";
    case FieldType::INT64: case FieldType::SINT64: case FieldType::SFIXED64: return "FIELD_INT64";
    case FieldType::UINT32: case FieldType::FIXED32: return "FIELD_UINT32";
    case FieldType::UINT64: case FieldType::FIXED64: return "FIELD_UINT64";
    case FieldType::BOOL: return "FIELD_BOOL";
    case FieldType::FLOAT: return "FIELD_FLOAT";
    case FieldType::DOUBLE: return "FIELD_DOUBLE";
    case FieldType::STRING: return "FIELD_STRING";
    case FieldType::BYTES: return "FIELD_BINARY";
    default: return "FIELD_OBJECT";
    }
}

struct McpackGen {
    const FileDescriptor* file;
    std::string prefix;
    std::vector<const Descriptor*> msgs;
    std::ostringstream c;

    void collect(const Descriptor* d) {
        msgs.push_back(d);
        for (const Descriptor* n : d->nested_types) collect(n);
    }
    bool local(const Descriptor* d) const {
        for (const Descriptor* m : msgs) {
            if (m == d) return true;
        }
        return false;
    }
    std::string fn(const Descriptor* d, const char* what) const { return std::string("mc_") + what + "_" + ident_of(d->full_name); }
    std::string kname(const Descriptor* d, const FieldDescriptor& f) const { return "kMc_" + ident_of(d->full_name) + "_" + f.name; }

    // value expression -> Serializer call with wire type t
    std::string add_call(const FieldDescriptor& f, const std::string& t, const std::string& name, const std::string& v) const {
        const CppType ct = f.cpp_type();
        if (ct == CppType::STRING) {
            return t == "FIELD_STRING" ? "sr->add_string(" + name + ", " + v + ");"
                                       : "{ const std::string& s_ = " + v + "; sr->add_binary(" + name + ", s_.data(), s_.size()); }";
        }
        struct Nat { CppType ct; const char* t; const char* call; };
        static const Nat kNat[] = {
            {CppType::INT32, "FIELD_INT32", "add_int32"}, {CppType::ENUM, "FIELD_INT32", "add_int32"},
            {CppType::INT64, "FIELD_INT64", "add_int64"}, {CppType::UINT32, "FIELD_UINT32", "add_uint32"},
            {CppType::UINT64, "FIELD_UINT64", "add_uint64"}, {CppType::BOOL, "FIELD_BOOL", "add_bool"},
            {CppType::FLOAT, "FIELD_FLOAT", "add_float"}, {CppType::DOUBLE, "FIELD_DOUBLE", "add_double"},
        };
        for (auto& n : kNat) {
            if (n.ct == ct && t == n.t) {
                const std::string cast = ct == CppType::ENUM ? "(int32_t)" : "";
                return "sr->" + std::string(n.call) + "(" + name + ", " + cast + v + ");";
            }
        }
        // idl_type asked for another width/kind: same conversion as the reflective codec
        const bool is_float = ct == CppType::FLOAT || ct == CppType::DOUBLE;
        const bool is_unsigned = ct == CppType::UINT32 || ct == CppType::UINT64;
        std::string iv = "0", uv = "0", dv = "0";
        if (is_float) dv = "(double)" + v;
        else if (is_unsigned) uv = "(uint64_t)" + v;
        else iv = "(int64_t)" + v;
        return "::mrpc::mcpack::AddConverted(sr, " + name + ", ::mrpc::mcpack::" + t + ", " + iv + ", " + uv + ", " + dv +
               ", " + (is_float ? "true" : "false") + ", " + (is_unsigned ? "true" : "false") + ");";
    }

    // parse one Value `val` into field f (set or add) of `m`
    std::string set_code(const Descriptor* d, const FieldDescriptor& f, const std::string& val) const {
        (void)d;
        const bool rep = f.is_repeated();
        const std::string op = rep ? "add_" + f.name : "set_" + f.name;
        switch (f.cpp_type()) {
        case CppType::INT32:
            return "{ int64_t v_; if (!" + val + ".to_int64(&v_)) return false; m->" + op + "((int32_t)v_); }";
        case CppType::ENUM:
            return "{ int64_t v_; if (!" + val + ".to_int64(&v_)) return false; m->" + op + "((" + cpp_enum(f.enum_type) +
                   ")(int)v_); }";
        case CppType::INT64:
            return "{ int64_t v_; if (!" + val + ".to_int64(&v_)) return false; m->" + op + "(v_); }";
        case CppType::UINT32:
            return "{ uint64_t v_; if (!" + val + ".to_uint64(&v_)) return false; m->" + op + "((uint32_t)v_); }";
        case CppType::UINT64:
            return "{ uint64_t v_; if (!" + val + ".to_uint64(&v_)) return false; m->" + op + "(v_); }";
        case CppType::BOOL:
            return "{ bool v_; if (!" + val + ".to_bool(&v_)) return false; m->" + op + "(v_); }";
        case CppType::FLOAT:
            return "{ double v_; if (!" + val + ".to_double(&v_)) return false; m->" + op + "((float)v_); }";
        case CppType::DOUBLE:
            return "{ double v_; if (!" + val + ".to_double(&v_)) return false; m->" + op + "(v_); }";
        case CppType::STRING:
            if (rep) return "{ if (!" + val + ".to_string(m->add_" + f.name + "())) return false; }";
            return "{ if (!" + val + ".to_string(m->mutable_" + f.name + "())) return false; }";
        case CppType::MESSAGE: {
            const std::string target = rep ? "m->add_" + f.name + "()" : "m->mutable_" + f.name + "()";
            const std::string parse = local(f.message_type) ? fn(f.message_type, "parse") + "(" + val + ", " + target + ")"
                                                            : "::mrpc::mcpack::ParseFromObject(" + val + ", " + target + ")";
            return "{ if (" + val + ".type() != ::mrpc::mcpack::FIELD_OBJECT || !" + parse + ") return false; }";
        }
        }
        return "";
    }

    void gen_message(const Descriptor* d) {
        const std::string cls = cpp_class(d);
        for (const FieldDescriptor& f : d->fields) {
            if (f.is_map()) continue;
            std::string n = mc_option(f, "idl_name");
            if (n.empty()) n = f.name;
            c << "const std::string " << kname(d, f) << "(" << cstr_literal(n) << ");\n";
        }
        // serialize
        c << "bool " << fn(d, "ser") << "(const ::mrpc::pb::Message& m_, ::mrpc::mcpack::Format fmt, ::mrpc::mcpack::Serializer* sr) {\n";
        c << "  const " << cls << "& m = static_cast<const " << cls << "&>(m_);\n  (void)m; (void)fmt;\n";
        for (const FieldDescriptor& f : d->fields) {
            if (f.is_map()) continue;
            const std::string K = kname(d, f), t = mc_wire_type(f);
            if (f.is_repeated()) {
                c << "  if (m." << f.name << "_size() > 0) {\n";
                if (f.cpp_type() == CppType::MESSAGE) {
                    c << "    sr->begin_array(" << K << ", ::mrpc::mcpack::FIELD_OBJECT, fmt);\n";
                    c << "    for (int i = 0; i < m." << f.name << "_size(); ++i) {\n      sr->begin_object();\n";
                    c << "      " << (local(f.message_type) ? fn(f.message_type, "ser") : std::string("::mrpc::mcpack::SerializeFields"))
                      << "(m." << f.name << "(i), fmt, sr);\n      sr->end_object();\n    }\n";
                } else {
                    c << "    sr->begin_array(" << K << ", ::mrpc::mcpack::" << t << ", fmt);\n";
                    c << "    for (int i = 0; i < m." << f.name << "_size(); ++i) " << add_call(f, t, "kMcEmpty", "m." + f.name + "(i)")
                      << "\n";
                }
                c << "    sr->end_array();\n  }\n";
                continue;
            }
            c << "  if (m.has_" << f.name << "()) {\n";
            if (f.cpp_type() == CppType::MESSAGE) {
                c << "    sr->begin_object(" << K << ");\n    "
                  << (local(f.message_type) ? fn(f.message_type, "ser") : std::string("::mrpc::mcpack::SerializeFields")) << "(m."
                  << f.name << "(), fmt, sr);\n    sr->end_object();\n";
            } else {
                c << "    " << add_call(f, t, K, "m." + f.name + "()") << "\n";
            }
            c << "  }\n";
        }
        c << "  return sr->good();\n}\n";
        // parse
        c << "bool " << fn(d, "parse") << "(const ::mrpc::mcpack::Value& obj, ::mrpc::pb::Message* m_) {\n";
        c << "  if (obj.type() != ::mrpc::mcpack::FIELD_OBJECT) return false;\n";
        c << "  " << cls << "* m = static_cast<" << cls << "*>(m_);\n";
        c << "  std::vector<::mrpc::mcpack::Item> items;\n  if (!::mrpc::mcpack::ListItems(obj, &items)) return false;\n";
        c << "  for (const ::mrpc::mcpack::Item& it : items) {\n    if (it.value.is_null()) continue;\n";
        c << "    const uint8_t t_ = it.value.type();\n    (void)t_;\n";
        bool first = true;
        for (const FieldDescriptor& f : d->fields) {
            if (f.is_map()) continue;
            c << "    " << (first ? "" : "} else ") << "if (it.name == " << kname(d, f) << ") {\n";
            first = false;
            if (f.is_repeated()) {
                if (f.cpp_type() == CppType::MESSAGE) {
                    c << "      if (t_ == ::mrpc::mcpack::FIELD_OBJECTISOARRAY) {\n"
                      << "        if (!::mrpc::mcpack::ParseObjectIsoArrayField(it.value, m, " << cls << "::descriptor()->field("
                      << f.index << "))) return false;\n        continue;\n      }\n";
                } else {
                    c << "      if (t_ == ::mrpc::mcpack::FIELD_OBJECTISOARRAY) return false;\n";
                }
                c << "      if (t_ == ::mrpc::mcpack::FIELD_ARRAY || t_ == ::mrpc::mcpack::FIELD_ISOARRAY) {\n"
                  << "        std::vector<::mrpc::mcpack::Item> elems;\n"
                  << "        if (!::mrpc::mcpack::ListItems(it.value, &elems)) return false;\n"
                  << "        for (const ::mrpc::mcpack::Item& e : elems) {\n          if (e.value.is_null()) continue;\n"
                  << "          " << set_code(d, f, "e.value") << "\n        }\n        continue;\n      }\n";
            }
            c << "      " << set_code(d, f, "it.value") << "\n";
        }
        if (!first) c << "    }\n";
        c << "  }\n  return true;\n}\n";
        c << "const ::mrpc::mcpack::MessageHandler " << fn(d, "handler") << " = {&" << fn(d, "ser") << ", &" << fn(d, "parse")
          << "};\n\n";
    }

    void run(const std::string& base) {
        for (const Descriptor* d : file->message_types) collect(d);
        c << "// Generated by mrpc_protoc --mcpack_out from " << file->name << ". DO NOT EDIT.\n";
        c << "#include \"" << prefix << base << ".pb.h\"\n#include <string>\n#include <vector>\n";
        c << "#include \"mcpack/mcpack.h\"\n\nnamespace {\n\nconst std::string kMcEmpty;\n\n";
        for (const Descriptor* d : msgs) {
            if (d->map_entry) continue;
            c << "bool " << fn(d, "ser") << "(const ::mrpc::pb::Message&, ::mrpc::mcpack::Format, ::mrpc::mcpack::Serializer*);\n";
            c << "bool " << fn(d, "parse") << "(const ::mrpc::mcpack::Value&, ::mrpc::pb::Message*);\n";
        }
        c << "\n";
        for (const Descriptor* d : msgs) {
            if (!d->map_entry) gen_message(d);
        }
        c << "struct McpackRegistrar {\n  McpackRegistrar() {\n";
        for (const Descriptor* d : msgs) {
            if (!d->map_entry) {
                c << "    ::mrpc::mcpack::RegisterMessageHandler(" << cpp_class(d) << "::descriptor(), &" << fn(d, "handler")
                  << ");\n";
            }
        }
        c << "  }\n} mc_registrar_" << ident_of(base) << ";\n\n}  // namespace\n";
    }
};

}  // namespace

int main(int argc, char** argv) {
    std::string out_dir = ".", prefix, mcpack_out;
    bool cpp_out = false;
    std::vector<std::string> paths, files;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a.compare(0, 10, "--cpp_out=") == 0) {
            out_dir = a.substr(10);
            cpp_out = true;
        }
        else if (a.compare(0, 13, "--proto_path=") == 0) paths.push_back(a.substr(13));
        else if (a.compare(0, 2, "-I") == 0) paths.push_back(a.substr(2));
        else if (a.compare(0, 17, "--include_prefix=") == 0) prefix = a.substr(17);
        else if (a.compare(0, 13, "--mcpack_out=") == 0) mcpack_out = a.substr(13);
        else files.push_back(a);
    }
    if (files.empty()) {
        fprintf(stderr, "usage: %s --cpp_out=DIR --proto_path=DIR [--include_prefix=P] file.proto...\n", argv[0]);
        return 1;
    }
    Importer imp(paths);
    for (const std::string& fpath : files) {
        std::string rel = fpath;
        for (const std::string& p : paths) {
            std::string pp = p;
            if (!pp.empty() && pp.back() != '/') pp += "/";
            if (rel.compare(0, pp.size(), pp) == 0) {
                rel = rel.substr(pp.size());
                break;
            }
        }
        std::string err;
        const FileDescriptor* fd = imp.Import(rel, &err);
        if (!fd) {
            fprintf(stderr, "mrpc_protoc: %s\n", err.c_str());
            return 1;
        }
        std::string base = basename_noext(rel);
        if (!mcpack_out.empty()) {
            McpackGen mg;
            mg.file = fd;
            mg.prefix = prefix;
            mg.run(base);
            std::ofstream(mcpack_out + "/" + base + ".pb.mcpack.cc") << mg.c.str();
            if (!cpp_out) continue;  // --mcpack_out alone: no message classes
        }
        Gen g;
        g.file = fd;
        g.prefix = prefix;
        g.run(base);
        std::ofstream(out_dir + "/" + base + ".pb.h") << g.h.str();
        std::ofstream(out_dir + "/" + base + ".pb.cc") << g.c.str();
    }
    return 0;
}
