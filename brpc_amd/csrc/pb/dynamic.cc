#include "pb/dynamic.h"

#include <cstdlib>
#include <new>

#include "base/logging.h"

namespace mrpc {
namespace pb {

namespace {
inline char* at(void* base, uint32_t off) { return reinterpret_cast<char*>(base) + off; }

void construct_field(void* m, const FieldDescriptor& f) {
    char* p = at(m, f.offset);
    if (f.is_repeated()) {
        switch (f.cpp_type()) {
        case CppType::BOOL: new (p) std::vector<uint8_t>(); break;
        case CppType::INT32:
        case CppType::ENUM: new (p) std::vector<int32_t>(); break;
        case CppType::UINT32: new (p) std::vector<uint32_t>(); break;
        case CppType::FLOAT: new (p) std::vector<float>(); break;
        case CppType::INT64: new (p) std::vector<int64_t>(); break;
        case CppType::UINT64: new (p) std::vector<uint64_t>(); break;
        case CppType::DOUBLE: new (p) std::vector<double>(); break;
        case CppType::STRING: new (p) std::vector<std::string>(); break;
        case CppType::MESSAGE: new (p) RepeatedPtrBase(); break;
        }
        return;
    }
    switch (f.cpp_type()) {
    case CppType::BOOL: *(bool*)p = f.default_int != 0; break;
    case CppType::INT32:
    case CppType::ENUM: *(int32_t*)p = (int32_t)f.default_int; break;
    case CppType::UINT32: *(uint32_t*)p = (uint32_t)f.default_uint; break;
    case CppType::FLOAT: *(float*)p = (float)f.default_double; break;
    case CppType::INT64: *(int64_t*)p = f.default_int; break;
    case CppType::UINT64: *(uint64_t*)p = f.default_uint; break;
    case CppType::DOUBLE: *(double*)p = f.default_double; break;
    case CppType::STRING: new (p) std::string(f.default_string); break;
    case CppType::MESSAGE: *(Message**)p = nullptr; break;
    }
}

void destroy_field(void* m, const FieldDescriptor& f) {
    char* p = at(m, f.offset);
    if (f.is_repeated()) {
        switch (f.cpp_type()) {
        case CppType::BOOL: ((std::vector<uint8_t>*)p)->~vector(); break;
        case CppType::INT32:
        case CppType::ENUM: ((std::vector<int32_t>*)p)->~vector(); break;
        case CppType::UINT32: ((std::vector<uint32_t>*)p)->~vector(); break;
        case CppType::FLOAT: ((std::vector<float>*)p)->~vector(); break;
        case CppType::INT64: ((std::vector<int64_t>*)p)->~vector(); break;
        case CppType::UINT64: ((std::vector<uint64_t>*)p)->~vector(); break;
        case CppType::DOUBLE: ((std::vector<double>*)p)->~vector(); break;
        case CppType::STRING: ((std::vector<std::string>*)p)->~vector(); break;
        case CppType::MESSAGE: ((RepeatedPtrBase*)p)->~RepeatedPtrBase(); break;
        }
        return;
    }
    if (f.cpp_type() == CppType::STRING) {
        using std::string;
        ((string*)p)->~string();
    } else if (f.cpp_type() == CppType::MESSAGE) {
        delete *(Message**)p;
    }
}

size_t align_up(size_t v, size_t a) { return (v + a - 1) & ~(a - 1); }
}  // namespace

DynamicMessage* DynamicMessage::Create(const Descriptor* d) {
    void* mem = ::malloc(d->object_size);
    CHECK(mem);
    memset(mem, 0, d->object_size);
    DynamicMessage* m = new (mem) DynamicMessage(d);
    for (const FieldDescriptor& f : d->fields) construct_field(m, f);
    return m;
}

DynamicMessage::~DynamicMessage() {
    for (const FieldDescriptor& f : _desc->fields) destroy_field(this, f);
}

void ResolveDefaultValue(FieldDescriptor* f) {
    if (!f->has_default) {
        if (f->cpp_type() == CppType::ENUM && f->enum_type && !f->enum_type->values.empty()) {
            f->default_int = f->enum_type->values[0].number;
        }
        return;
    }
    const std::string& s = f->default_str;
    switch (f->cpp_type()) {
    case CppType::BOOL: f->default_int = (s == "true" || s == "1"); break;
    case CppType::INT32:
    case CppType::INT64: f->default_int = strtoll(s.c_str(), nullptr, 0); break;
    case CppType::UINT32:
    case CppType::UINT64: f->default_uint = strtoull(s.c_str(), nullptr, 0); break;
    case CppType::FLOAT:
    case CppType::DOUBLE:
        if (s == "inf") f->default_double = 1.0 / 0.0;
        else if (s == "-inf") f->default_double = -1.0 / 0.0;
        else if (s == "nan") f->default_double = 0.0 / 0.0;
        else f->default_double = strtod(s.c_str(), nullptr);
        break;
    case CppType::ENUM: {
        const EnumValueDescriptor* ev = f->enum_type ? f->enum_type->FindValueByName(s) : nullptr;
        f->default_int = ev ? ev->number : strtoll(s.c_str(), nullptr, 0);
        break;
    }
    case CppType::STRING: f->default_string = s; break;
    case CppType::MESSAGE: break;
    }
}

void PrepareDynamicLayout(Descriptor* d) {
    for (Descriptor* n : d->nested_types) PrepareDynamicLayout(n);
    if (d->factory) return;  // generated type: layout comes from the C++ class
    size_t off = align_up(sizeof(DynamicMessage), 8);
    uint32_t nbits = 0;
    for (FieldDescriptor& f : d->fields) {
        if (!f.is_repeated() && f.cpp_type() != CppType::MESSAGE && !f.proto3_implicit) f.has_bit = (int32_t)nbits++;
        else f.has_bit = -1;
    }
    d->num_has_bits = nbits;
    d->has_bits_offset = (uint32_t)off;
    off += ((nbits + 31) / 32) * 4;
    if (nbits == 0) off += 4;  // keep a valid has-bits word
    for (FieldDescriptor& f : d->fields) {
        size_t sz, al;
        if (f.is_repeated()) {
            sz = sizeof(std::vector<int64_t>);
            al = 8;
        } else {
            sz = CppTypeSize(f.cpp_type());
            al = CppTypeAlign(f.cpp_type());
        }
        off = align_up(off, al);
        f.offset = (uint32_t)off;
        off += sz;
    }
    d->object_size = (uint32_t)align_up(off, 8);
    d->BuildIndex();
    if (!d->prototype) {
        d->prototype = DynamicMessage::Create(d);
        d->owns_prototype = true;
    }
}

}  // namespace pb
}  // namespace mrpc
