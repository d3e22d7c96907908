#include "pb/message.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <sstream>

#include "base/buf.h"
#include "base/logging.h"

namespace mrpc {
namespace pb {

namespace {

template <typename T>
inline T& ref(Message* m, const FieldDescriptor* f) {
    return *reinterpret_cast<T*>(reinterpret_cast<char*>(m) + f->offset);
}
template <typename T>
inline const T& cref(const Message& m, const FieldDescriptor* f) {
    return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(&m) + f->offset);
}
inline uint32_t* has_bits(Message* m) {
    return reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(m) + m->GetDescriptor()->has_bits_offset);
}
inline const uint32_t* has_bits(const Message& m) {
    return reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(&m) + m.GetDescriptor()->has_bits_offset);
}

WireType wire_type_of(FieldType t) {
    switch (t) {
    case FieldType::DOUBLE:
    case FieldType::FIXED64:
    case FieldType::SFIXED64: return WIRETYPE_FIXED64;
    case FieldType::FLOAT:
    case FieldType::FIXED32:
    case FieldType::SFIXED32: return WIRETYPE_FIXED32;
    case FieldType::STRING:
    case FieldType::BYTES:
    case FieldType::MESSAGE: return WIRETYPE_LENGTH_DELIMITED;
    case FieldType::GROUP: return WIRETYPE_START_GROUP;
    default: return WIRETYPE_VARINT;
    }
}

// Size of one scalar element (no tag).
size_t scalar_size(FieldType t, const void* p) {
    switch (t) {
    case FieldType::DOUBLE:
    case FieldType::FIXED64:
    case FieldType::SFIXED64: return 8;
    case FieldType::FLOAT:
    case FieldType::FIXED32:
    case FieldType::SFIXED32: return 4;
    case FieldType::BOOL: return 1;
    case FieldType::INT32:
    case FieldType::ENUM: return int32_size(*(const int32_t*)p);
    case FieldType::SINT32: return varint_size(zigzag32(*(const int32_t*)p));
    case FieldType::UINT32: return varint_size(*(const uint32_t*)p);
    case FieldType::INT64: return varint_size((uint64_t)*(const int64_t*)p);
    case FieldType::SINT64: return varint_size(zigzag64(*(const int64_t*)p));
    case FieldType::UINT64: return varint_size(*(const uint64_t*)p);
    default: return 0;
    }
}

uint8_t* write_scalar(uint8_t* o, FieldType t, const void* p) {
    switch (t) {
    case FieldType::DOUBLE:
    case FieldType::FIXED64:
    case FieldType::SFIXED64: return write_fixed64(o, *(const uint64_t*)p);
    case FieldType::FLOAT:
    case FieldType::FIXED32:
    case FieldType::SFIXED32: return write_fixed32(o, *(const uint32_t*)p);
    case FieldType::BOOL: *o++ = (*(const uint8_t*)p) ? 1 : 0; return o;
    case FieldType::INT32:
    case FieldType::ENUM: return write_varint(o, (uint64_t)(int64_t)*(const int32_t*)p);
    case FieldType::SINT32: return write_varint(o, zigzag32(*(const int32_t*)p));
    case FieldType::UINT32: return write_varint(o, *(const uint32_t*)p);
    case FieldType::INT64: return write_varint(o, (uint64_t)*(const int64_t*)p);
    case FieldType::SINT64: return write_varint(o, zigzag64(*(const int64_t*)p));
    case FieldType::UINT64: return write_varint(o, *(const uint64_t*)p);
    default: return o;
    }
}

// Payload bytes of elements [0, n) of a repeated scalar field in its vector
// layout: typed, branch-free loops (varint size = (bit width * 9 + 64) / 64)
// instead of a per-element switch and loop; packed runs of 10^4..10^5
// elements are sized twice per serialization.
inline size_t vsize64(uint64_t v) { return (size_t)(((63 - __builtin_clzll(v | 1)) * 9 + 73) >> 6); }
size_t repeated_payload_bytes(FieldType t, const char* data, size_t n) {
    size_t s = 0;
    switch (t) {
    case FieldType::DOUBLE:
    case FieldType::FIXED64:
    case FieldType::SFIXED64: return 8 * n;
    case FieldType::FLOAT:
    case FieldType::FIXED32:
    case FieldType::SFIXED32: return 4 * n;
    case FieldType::BOOL: return n;
    case FieldType::INT32:
    case FieldType::ENUM: {
        const int32_t* v = reinterpret_cast<const int32_t*>(data);
        for (size_t i = 0; i < n; ++i) s += vsize64((uint64_t)(int64_t)v[i]);
        return s;
    }
    case FieldType::SINT32: {
        const int32_t* v = reinterpret_cast<const int32_t*>(data);
        for (size_t i = 0; i < n; ++i) s += vsize64(zigzag32(v[i]));
        return s;
    }
    case FieldType::UINT32: {
        const uint32_t* v = reinterpret_cast<const uint32_t*>(data);
        for (size_t i = 0; i < n; ++i) s += vsize64(v[i]);
        return s;
    }
    case FieldType::INT64:
    case FieldType::UINT64: {
        const uint64_t* v = reinterpret_cast<const uint64_t*>(data);
        for (size_t i = 0; i < n; ++i) s += vsize64(v[i]);
        return s;
    }
    case FieldType::SINT64: {
        const int64_t* v = reinterpret_cast<const int64_t*>(data);
        for (size_t i = 0; i < n; ++i) s += vsize64(zigzag64(v[i]));
        return s;
    }
    default: return 0;
    }
}

size_t elem_bytes(FieldType t) {
    switch (CppTypeOf(t)) {
    case CppType::BOOL: return 1;
    case CppType::INT32:
    case CppType::UINT32:
    case CppType::ENUM:
    case CppType::FLOAT: return 4;
    default: return 8;
    }
}

// vector of raw bytes-per-elem, independent of T for reading purposes
struct RawVec {
    const char* data;
    size_t n;
};
RawVec raw_repeated(const Message& m, const FieldDescriptor* f) {
    const char* base = reinterpret_cast<const char*>(&m) + f->offset;
    switch (f->cpp_type()) {
    case CppType::BOOL: {
        auto& v = *(const std::vector<uint8_t>*)base;
        return RawVec{(const char*)v.data(), v.size()};
    }
    case CppType::INT32:
    case CppType::ENUM: {
        auto& v = *(const std::vector<int32_t>*)base;
        return RawVec{(const char*)v.data(), v.size()};
    }
    case CppType::UINT32: {
        auto& v = *(const std::vector<uint32_t>*)base;
        return RawVec{(const char*)v.data(), v.size()};
    }
    case CppType::FLOAT: {
        auto& v = *(const std::vector<float>*)base;
        return RawVec{(const char*)v.data(), v.size()};
    }
    case CppType::INT64: {
        auto& v = *(const std::vector<int64_t>*)base;
        return RawVec{(const char*)v.data(), v.size()};
    }
    case CppType::UINT64: {
        auto& v = *(const std::vector<uint64_t>*)base;
        return RawVec{(const char*)v.data(), v.size()};
    }
    case CppType::DOUBLE: {
        auto& v = *(const std::vector<double>*)base;
        return RawVec{(const char*)v.data(), v.size()};
    }
    default: return RawVec{nullptr, 0};
    }
}

bool is_default_scalar(const Message& m, const FieldDescriptor* f) {
    switch (f->cpp_type()) {
    case CppType::BOOL: return !cref<bool>(m, f);
    case CppType::INT32:
    case CppType::ENUM: return cref<int32_t>(m, f) == 0;
    case CppType::UINT32: return cref<uint32_t>(m, f) == 0;
    case CppType::FLOAT: {
        float v = cref<float>(m, f);
        uint32_t bits;
        memcpy(&bits, &v, 4);
        return bits == 0;
    }
    case CppType::INT64: return cref<int64_t>(m, f) == 0;
    case CppType::UINT64: return cref<uint64_t>(m, f) == 0;
    case CppType::DOUBLE: {
        double v = cref<double>(m, f);
        uint64_t bits;
        memcpy(&bits, &v, 8);
        return bits == 0;
    }
    case CppType::STRING: return cref<std::string>(m, f).empty();
    case CppType::MESSAGE: return cref<Message*>(m, f) == nullptr;
    }
    return true;
}

bool field_present(const Message& m, const FieldDescriptor* f) {
    if (f->cpp_type() == CppType::MESSAGE) return cref<Message*>(m, f) != nullptr;
    if (f->has_bit >= 0) return (has_bits(m)[f->has_bit >> 5] >> (f->has_bit & 31)) & 1;
    return !is_default_scalar(m, f);
}

void set_has(Message* m, const FieldDescriptor* f) {
    if (f->has_bit >= 0) has_bits(m)[f->has_bit >> 5] |= (1u << (f->has_bit & 31));
}

void clear_has(Message* m, const FieldDescriptor* f) {
    if (f->has_bit >= 0) has_bits(m)[f->has_bit >> 5] &= ~(1u << (f->has_bit & 31));
}

void set_scalar_default(Message* m, const FieldDescriptor* f) {
    switch (f->cpp_type()) {
    case CppType::BOOL: ref<bool>(m, f) = f->default_int != 0; break;
    case CppType::INT32:
    case CppType::ENUM: ref<int32_t>(m, f) = (int32_t)f->default_int; break;
    case CppType::UINT32: ref<uint32_t>(m, f) = (uint32_t)f->default_uint; break;
    case CppType::FLOAT: ref<float>(m, f) = (float)f->default_double; break;
    case CppType::INT64: ref<int64_t>(m, f) = f->default_int; break;
    case CppType::UINT64: ref<uint64_t>(m, f) = f->default_uint; break;
    case CppType::DOUBLE: ref<double>(m, f) = f->default_double; break;
    case CppType::STRING: ref<std::string>(m, f) = f->default_string; break;
    case CppType::MESSAGE: break;
    }
}

void clear_repeated(Message* m, const FieldDescriptor* f) {
    char* base = reinterpret_cast<char*>(m) + f->offset;
    switch (f->cpp_type()) {
    case CppType::BOOL: ((std::vector<uint8_t>*)base)->clear(); break;
    case CppType::INT32:
    case CppType::ENUM: ((std::vector<int32_t>*)base)->clear(); break;
    case CppType::UINT32: ((std::vector<uint32_t>*)base)->clear(); break;
    case CppType::FLOAT: ((std::vector<float>*)base)->clear(); break;
    case CppType::INT64: ((std::vector<int64_t>*)base)->clear(); break;
    case CppType::UINT64: ((std::vector<uint64_t>*)base)->clear(); break;
    case CppType::DOUBLE: ((std::vector<double>*)base)->clear(); break;
    case CppType::STRING: ((std::vector<std::string>*)base)->clear(); break;
    case CppType::MESSAGE: ((RepeatedPtrBase*)base)->Clear(); break;
    }
}

template <typename T>
void push_raw(Message* m, const FieldDescriptor* f, T v) {
    ref<std::vector<T>>(m, f).push_back(v);
}

// Store a decoded varint/fixed value into field f (singular or repeated).
void store_number(Message* m, const FieldDescriptor* f, uint64_t raw) {
    const bool rep = f->is_repeated();
    switch (f->type) {
    case FieldType::INT32:
    case FieldType::ENUM:
    case FieldType::SFIXED32: {
        int32_t v = (int32_t)raw;
        if (rep) push_raw<int32_t>(m, f, v); else ref<int32_t>(m, f) = v;
        break;
    }
    case FieldType::SINT32: {
        int32_t v = unzigzag32((uint32_t)raw);
        if (rep) push_raw<int32_t>(m, f, v); else ref<int32_t>(m, f) = v;
        break;
    }
    case FieldType::UINT32:
    case FieldType::FIXED32: {
        uint32_t v = (uint32_t)raw;
        if (rep) push_raw<uint32_t>(m, f, v); else ref<uint32_t>(m, f) = v;
        break;
    }
    case FieldType::INT64:
    case FieldType::SFIXED64: {
        int64_t v = (int64_t)raw;
        if (rep) push_raw<int64_t>(m, f, v); else ref<int64_t>(m, f) = v;
        break;
    }
    case FieldType::SINT64: {
        int64_t v = unzigzag64(raw);
        if (rep) push_raw<int64_t>(m, f, v); else ref<int64_t>(m, f) = v;
        break;
    }
    case FieldType::UINT64:
    case FieldType::FIXED64: {
        if (rep) push_raw<uint64_t>(m, f, raw); else ref<uint64_t>(m, f) = raw;
        break;
    }
    case FieldType::BOOL: {
        uint8_t v = raw != 0;
        if (rep) push_raw<uint8_t>(m, f, v); else ref<bool>(m, f) = v;
        break;
    }
    case FieldType::FLOAT: {
        uint32_t b = (uint32_t)raw;
        float v;
        memcpy(&v, &b, 4);
        if (rep) push_raw<float>(m, f, v); else ref<float>(m, f) = v;
        break;
    }
    case FieldType::DOUBLE: {
        double v;
        memcpy(&v, &raw, 8);
        if (rep) push_raw<double>(m, f, v); else ref<double>(m, f) = v;
        break;
    }
    default: break;
    }
    if (!rep) {
        if (f->oneof_index >= 0) ClearOneofSiblings(m, f);
        set_has(m, f);
    }
}

bool read_number(CodedInput* in, FieldType t, uint64_t* out) {
    switch (wire_type_of(t)) {
    case WIRETYPE_VARINT: return in->read_varint(out);
    case WIRETYPE_FIXED32: {
        uint32_t v;
        if (!in->read_fixed32(&v)) return false;
        *out = v;
        return true;
    }
    case WIRETYPE_FIXED64: return in->read_fixed64(out);
    default: return false;
    }
}

bool parse_message(Message* m, CodedInput* in);

// Packed payload p[0, len) appended to a repeated scalar field in bulk:
// fixed-width types are one memcpy, varints are counted first (one pass
// over the terminator bits, so the vector grows once) and decoded by a
// typed loop instead of a per-element switch. Same results and the same
// failures as the element-wise path.
template <typename T, typename Conv>
bool bulk_varints(Message* m, const FieldDescriptor* f, const uint8_t* p, size_t len, Conv conv) {
    size_t n = 0;
    for (size_t i = 0; i < len; ++i) n += (p[i] >> 7) ^ 1;
    auto& vec = ref<std::vector<T>>(m, f);
    const size_t base = vec.size();
    vec.resize(base + n);
    T* out = vec.data() + base;
    CodedInput in(p, len);
    for (size_t k = 0; k < n; ++k) {
        uint64_t v;
        if (!in.read_varint(&v)) {
            vec.resize(base + k);
            return false;
        }
        out[k] = conv(v);
    }
    return in.at_limit();
}

template <typename T>
bool bulk_fixed(Message* m, const FieldDescriptor* f, const uint8_t* p, size_t len) {
    if (len % sizeof(T)) return false;
    auto& vec = ref<std::vector<T>>(m, f);
    const size_t base = vec.size();
    vec.resize(base + len / sizeof(T));
    memcpy(vec.data() + base, p, len);
    return true;
}

bool parse_packed(Message* m, const FieldDescriptor* f, const uint8_t* p, size_t len) {
    switch (f->type) {
    case FieldType::INT32:
    case FieldType::ENUM: return bulk_varints<int32_t>(m, f, p, len, [](uint64_t v) { return (int32_t)v; });
    case FieldType::SINT32:
        return bulk_varints<int32_t>(m, f, p, len, [](uint64_t v) { return unzigzag32((uint32_t)v); });
    case FieldType::UINT32: return bulk_varints<uint32_t>(m, f, p, len, [](uint64_t v) { return (uint32_t)v; });
    case FieldType::INT64: return bulk_varints<int64_t>(m, f, p, len, [](uint64_t v) { return (int64_t)v; });
    case FieldType::SINT64: return bulk_varints<int64_t>(m, f, p, len, [](uint64_t v) { return unzigzag64(v); });
    case FieldType::UINT64: return bulk_varints<uint64_t>(m, f, p, len, [](uint64_t v) { return v; });
    case FieldType::BOOL: return bulk_varints<uint8_t>(m, f, p, len, [](uint64_t v) { return (uint8_t)(v != 0); });
    case FieldType::FIXED32:
    case FieldType::SFIXED32: return f->cpp_type() == CppType::UINT32 ? bulk_fixed<uint32_t>(m, f, p, len)
                                                                      : bulk_fixed<int32_t>(m, f, p, len);
    case FieldType::FIXED64: return bulk_fixed<uint64_t>(m, f, p, len);
    case FieldType::SFIXED64: return bulk_fixed<int64_t>(m, f, p, len);
    case FieldType::FLOAT: return bulk_fixed<float>(m, f, p, len);
    case FieldType::DOUBLE: return bulk_fixed<double>(m, f, p, len);
    default: return false;
    }
}

bool parse_field(Message* m, const FieldDescriptor* f, uint32_t tag, CodedInput* in) {
    const WireType wt = (WireType)(tag & 7);
    const WireType expected = wire_type_of(f->type);
    if (f->is_repeated() && f->is_packable() && wt == WIRETYPE_LENGTH_DELIMITED) {
        uint64_t len;
        const uint8_t* p;
        if (!in->read_varint(&len) || !in->read_bytes((size_t)len, &p)) return false;
        return parse_packed(m, f, p, (size_t)len);
    }
    if (wt != expected) {
        // Mismatched wire type: keep as unknown field (protobuf semantics).
        return in->skip_field(tag, m->mutable_unknown_fields());
    }
    switch (f->cpp_type()) {
    case CppType::STRING: {
        uint64_t len;
        const uint8_t* d;
        if (!in->read_varint(&len) || !in->read_bytes((size_t)len, &d)) return false;
        if (f->is_repeated()) {
            ref<std::vector<std::string>>(m, f).emplace_back((const char*)d, (size_t)len);
        } else {
            if (f->oneof_index >= 0) ClearOneofSiblings(m, f);
            ref<std::string>(m, f).assign((const char*)d, (size_t)len);
            set_has(m, f);
        }
        return true;
    }
    case CppType::MESSAGE: {
        if (f->type == FieldType::GROUP) return in->skip_field(tag, m->mutable_unknown_fields());
        uint64_t len;
        const uint8_t* old;
        if (!in->read_varint(&len) || !in->push_limit((size_t)len, &old)) return false;
        Message* sub = f->is_repeated() ? Reflection::AddMessage(m, f) : Reflection::MutableMessage(m, f);
        if (!in->inc_depth()) return false;
        if (!parse_message(sub, in)) return false;
        in->dec_depth();
        if (!in->at_limit()) return false;
        in->pop_limit(old);
        return true;
    }
    default: {
        uint64_t v;
        if (!read_number(in, f->type, &v)) return false;
        store_number(m, f, v);
        return true;
    }
    }
}

bool parse_message(Message* m, CodedInput* in) { return m->MergePartialFromCodedInput(in); }

}  // namespace

// ---------------------------------------------------------------- Message

Message::~Message() {}

void Message::Clear() {
    const Descriptor* d = GetDescriptor();
    for (const FieldDescriptor& fd : d->fields) {
        const FieldDescriptor* f = &fd;
        if (f->is_repeated()) {
            clear_repeated(this, f);
        } else if (f->cpp_type() == CppType::MESSAGE) {
            Message*& sub = ref<Message*>(this, f);
            if (sub) sub->Clear();
            delete sub;
            sub = nullptr;
        } else {
            set_scalar_default(this, f);
        }
    }
    uint32_t* hb = has_bits(this);
    for (uint32_t i = 0; i < (d->num_has_bits + 31) / 32; ++i) hb[i] = 0;
    _unknown.clear();
}

size_t Message::ByteSizeLong() const {
    const Descriptor* d = GetDescriptor();
    size_t total = 0;
    for (const FieldDescriptor& fd : d->fields) {
        const FieldDescriptor* f = &fd;
        const size_t tag_size = varint_size(make_tag(f->number, WIRETYPE_VARINT));
        if (f->is_repeated()) {
            switch (f->cpp_type()) {
            case CppType::STRING: {
                const auto& v = cref<std::vector<std::string>>(*this, f);
                for (const auto& s : v) total += tag_size + varint_size(s.size()) + s.size();
                break;
            }
            case CppType::MESSAGE: {
                const auto& v = cref<RepeatedPtrBase>(*this, f);
                for (int i = 0; i < v.size(); ++i) {
                    size_t s = v.Get(i)->ByteSizeLong();
                    total += tag_size + varint_size(s) + s;
                }
                break;
            }
            default: {
                RawVec rv = raw_repeated(*this, f);
                if (rv.n == 0) break;
                const size_t data = repeated_payload_bytes(f->type, rv.data, rv.n);
                if (f->packed) total += tag_size + varint_size(data) + data;
                else total += tag_size * rv.n + data;
            }
            }
            continue;
        }
        if (!field_present(*this, f)) continue;
        switch (f->cpp_type()) {
        case CppType::STRING: {
            const auto& s = cref<std::string>(*this, f);
            total += tag_size + varint_size(s.size()) + s.size();
            break;
        }
        case CppType::MESSAGE: {
            size_t s = cref<Message*>(*this, f)->ByteSizeLong();
            total += tag_size + varint_size(s) + s;
            break;
        }
        default:
            total += tag_size + scalar_size(f->type, reinterpret_cast<const char*>(this) + f->offset);
        }
    }
    total += _unknown.size();
    _cached_size = (int)total;
    return total;
}

const void* Reflection::RepeatedScalarData(const Message& m, const FieldDescriptor* f, size_t* n, size_t* eb) {
    *n = 0;
    *eb = 0;
    if (!f->is_repeated() || f->cpp_type() == CppType::STRING || f->cpp_type() == CppType::MESSAGE) return nullptr;
    RawVec rv = raw_repeated(m, f);
    *n = rv.n;
    *eb = elem_bytes(f->type);
    return rv.data;
}

static thread_local PackedRunSink* tls_run_sink = nullptr;

PackedRunSink* SetThreadPackedRunSink(PackedRunSink* sink) {
    PackedRunSink* prev = tls_run_sink;
    tls_run_sink = sink;
    return prev;
}

bool IsVarintFieldType(FieldType t) {
    switch (t) {
    case FieldType::INT32:
    case FieldType::ENUM:
    case FieldType::SINT32:
    case FieldType::UINT32:
    case FieldType::INT64:
    case FieldType::SINT64:
    case FieldType::UINT64:
    case FieldType::BOOL: return true;
    default: return false;
    }
}

void EncodePackedRunOnHost(const PackedRun& run) {
    uint8_t* o = run.dst;
    const char* v = static_cast<const char*>(run.values);
    for (size_t i = 0; i < run.n; ++i) o = write_scalar(o, run.type, v + i * run.elem_bytes);
}

uint8_t* Message::SerializeWithCachedSizesToArray(uint8_t* o) const {
    const Descriptor* d = GetDescriptor();
    for (const FieldDescriptor& fd : d->fields) {
        const FieldDescriptor* f = &fd;
        if (f->is_repeated()) {
            switch (f->cpp_type()) {
            case CppType::STRING: {
                for (const auto& s : cref<std::vector<std::string>>(*this, f)) {
                    o = write_tag(o, f->number, WIRETYPE_LENGTH_DELIMITED);
                    o = write_varint(o, s.size());
                    memcpy(o, s.data(), s.size());
                    o += s.size();
                }
                break;
            }
            case CppType::MESSAGE: {
                const auto& v = cref<RepeatedPtrBase>(*this, f);
                for (int i = 0; i < v.size(); ++i) {
                    const Message* sub = v.Get(i);
                    o = write_tag(o, f->number, WIRETYPE_LENGTH_DELIMITED);
                    o = write_varint(o, (uint64_t)sub->GetCachedSize());
                    o = sub->SerializeWithCachedSizesToArray(o);
                }
                break;
            }
            default: {
                RawVec rv = raw_repeated(*this, f);
                if (rv.n == 0) break;
                const size_t eb = elem_bytes(f->type);
                PackedRunSink* sink = tls_run_sink;
                if (f->packed && sink && rv.n >= sink->min_elems() && IsVarintFieldType(f->type)) {
                    PackedRun run;
                    run.values = rv.data;
                    run.n = rv.n;
                    run.elem_bytes = eb;
                    run.type = f->type;
                    run.chunk_bytes.reserve((rv.n + kPackedRunChunkElems - 1) / kPackedRunChunkElems);
                    size_t data = 0;
                    for (size_t c = 0; c < rv.n; c += kPackedRunChunkElems) {
                        const size_t e = std::min(rv.n, c + kPackedRunChunkElems);
                        const size_t cb = repeated_payload_bytes(f->type, rv.data + c * eb, e - c);
                        run.chunk_bytes.push_back((uint32_t)cb);
                        data += cb;
                    }
                    o = write_tag(o, f->number, WIRETYPE_LENGTH_DELIMITED);
                    o = write_varint(o, data);
                    run.dst = o;
                    run.bytes = data;
                    o += data;
                    sink->Take(std::move(run));
                } else if (f->packed) {
                    const size_t data = repeated_payload_bytes(f->type, rv.data, rv.n);
                    o = write_tag(o, f->number, WIRETYPE_LENGTH_DELIMITED);
                    o = write_varint(o, data);
                    for (size_t i = 0; i < rv.n; ++i) o = write_scalar(o, f->type, rv.data + i * eb);
                } else {
                    const WireType wt = wire_type_of(f->type);
                    for (size_t i = 0; i < rv.n; ++i) {
                        o = write_tag(o, f->number, wt);
                        o = write_scalar(o, f->type, rv.data + i * eb);
                    }
                }
            }
            }
            continue;
        }
        if (!field_present(*this, f)) continue;
        switch (f->cpp_type()) {
        case CppType::STRING: {
            const auto& s = cref<std::string>(*this, f);
            o = write_tag(o, f->number, WIRETYPE_LENGTH_DELIMITED);
            o = write_varint(o, s.size());
            memcpy(o, s.data(), s.size());
            o += s.size();
            break;
        }
        case CppType::MESSAGE: {
            const Message* sub = cref<Message*>(*this, f);
            o = write_tag(o, f->number, WIRETYPE_LENGTH_DELIMITED);
            o = write_varint(o, (uint64_t)sub->GetCachedSize());
            o = sub->SerializeWithCachedSizesToArray(o);
            break;
        }
        default:
            o = write_tag(o, f->number, wire_type_of(f->type));
            o = write_scalar(o, f->type, reinterpret_cast<const char*>(this) + f->offset);
        }
    }
    if (!_unknown.empty()) {
        memcpy(o, _unknown.data(), _unknown.size());
        o += _unknown.size();
    }
    return o;
}

bool Message::MergePartialFromCodedInput(CodedInput* in) {
    const Descriptor* d = GetDescriptor();
    for (;;) {
        const uint32_t tag = in->read_tag();
        if (tag == 0) return true;
        if (tag == 0xFFFFFFFFu || (tag >> 3) == 0) return false;
        if ((tag & 7) == WIRETYPE_END_GROUP) return false;
        const FieldDescriptor* f = d->FindFieldByNumber((int)(tag >> 3));
        if (!f) {
            if (!in->skip_field(tag, &_unknown)) return false;
            continue;
        }
        if (!parse_field(this, f, tag, in)) return false;
    }
}

static bool is_initialized_impl(const Message& m, std::string* missing, const std::string& prefix) {
    bool ok = true;
    const Descriptor* d = m.GetDescriptor();
    for (const FieldDescriptor& fd : d->fields) {
        const FieldDescriptor* f = &fd;
        if (f->is_required() && !field_present(m, f)) {
            ok = false;
            if (missing) {
                if (!missing->empty()) missing->append(", ");
                missing->append(prefix + f->name);
            } else {
                return false;
            }
        }
        if (f->cpp_type() == CppType::MESSAGE) {
            if (f->is_repeated()) {
                const auto& v = cref<RepeatedPtrBase>(m, f);
                for (int i = 0; i < v.size(); ++i) {
                    if (!is_initialized_impl(*v.Get(i), missing, prefix + f->name + "[" + std::to_string(i) + "].")) {
                        ok = false;
                        if (!missing) return false;
                    }
                }
            } else if (const Message* sub = cref<Message*>(m, f)) {
                if (!is_initialized_impl(*sub, missing, prefix + f->name + ".")) {
                    ok = false;
                    if (!missing) return false;
                }
            }
        }
    }
    return ok;
}

bool Message::IsInitialized() const { return is_initialized_impl(*this, nullptr, ""); }

std::string Message::InitializationErrorString() const {
    std::string s;
    is_initialized_impl(*this, &s, "");
    return s;
}

void Message::MergeFrom(const Message& from) {
    const Descriptor* d = GetDescriptor();
    CHECK(d == from.GetDescriptor() || d->full_name == from.GetDescriptor()->full_name)
        << "MergeFrom between different types";
    for (const FieldDescriptor& fd : d->fields) {
        const FieldDescriptor* f = &fd;
        if (f->is_repeated()) {
            const int n = Reflection::FieldSize(from, f);
            for (int i = 0; i < n; ++i) {
                switch (f->cpp_type()) {
                case CppType::INT32: Reflection::AddInt32(this, f, Reflection::GetRepeatedInt32(from, f, i)); break;
                case CppType::ENUM: Reflection::AddEnumValue(this, f, Reflection::GetRepeatedEnumValue(from, f, i)); break;
                case CppType::UINT32: Reflection::AddUInt32(this, f, Reflection::GetRepeatedUInt32(from, f, i)); break;
                case CppType::INT64: Reflection::AddInt64(this, f, Reflection::GetRepeatedInt64(from, f, i)); break;
                case CppType::UINT64: Reflection::AddUInt64(this, f, Reflection::GetRepeatedUInt64(from, f, i)); break;
                case CppType::FLOAT: Reflection::AddFloat(this, f, Reflection::GetRepeatedFloat(from, f, i)); break;
                case CppType::DOUBLE: Reflection::AddDouble(this, f, Reflection::GetRepeatedDouble(from, f, i)); break;
                case CppType::BOOL: Reflection::AddBool(this, f, Reflection::GetRepeatedBool(from, f, i)); break;
                case CppType::STRING: Reflection::AddString(this, f, Reflection::GetRepeatedString(from, f, i)); break;
                case CppType::MESSAGE: Reflection::AddMessage(this, f)->MergeFrom(Reflection::GetRepeatedMessage(from, f, i)); break;
                }
            }
            continue;
        }
        if (!field_present(from, f)) continue;
        switch (f->cpp_type()) {
        case CppType::MESSAGE: Reflection::MutableMessage(this, f)->MergeFrom(*cref<Message*>(from, f)); break;
        case CppType::STRING: Reflection::SetString(this, f, cref<std::string>(from, f)); break;
        default:
            memcpy(reinterpret_cast<char*>(this) + f->offset, reinterpret_cast<const char*>(&from) + f->offset,
                   CppTypeSize(f->cpp_type()));
            if (f->oneof_index >= 0) ClearOneofSiblings(this, f);
            set_has(this, f);
        }
    }
    _unknown.append(from._unknown);
}

void Message::CopyFrom(const Message& from) {
    if (&from == this) return;
    Clear();
    MergeFrom(from);
}

bool Message::SerializeToArray(void* data, int size) const {
    const size_t n = ByteSizeLong();
    if ((size_t)size < n) return false;
    SerializeWithCachedSizesToArray((uint8_t*)data);
    return true;
}

bool Message::AppendToString(std::string* out) const {
    const size_t n = ByteSizeLong();
    const size_t old = out->size();
    out->resize(old + n);
    uint8_t* e = SerializeWithCachedSizesToArray((uint8_t*)&(*out)[old]);
    return (size_t)(e - (uint8_t*)&(*out)[old]) == n;
}

bool Message::SerializeToString(std::string* out) const {
    out->clear();
    return AppendToString(out);
}

std::string Message::SerializeAsString() const {
    std::string s;
    SerializeToString(&s);
    return s;
}

bool Message::SerializeToBuf(Buf* out) const {
    const size_t n = ByteSizeLong();
    if (n == 0) return true;
    char* p = out->append_contiguous(n);
    if (!p) return false;
    uint8_t* e = SerializeWithCachedSizesToArray((uint8_t*)p);
    return (size_t)(e - (uint8_t*)p) == n;
}

bool Message::ParsePartialFromArray(const void* data, size_t size) {
    Clear();
    CodedInput in(data, size);
    return MergePartialFromCodedInput(&in);
}

bool Message::ParseFromArray(const void* data, size_t size) {
    return ParsePartialFromArray(data, size) && IsInitialized();
}

bool Message::MergeFromString(const std::string& s) {
    CodedInput in(s.data(), s.size());
    return MergePartialFromCodedInput(&in);
}

bool Message::ParseFromBuf(const Buf& in) {
    if (in.backing_block_num() == 1 && IsHostAccessible(in.ref_at(0).block->kind)) {
        return ParseFromArray(in.block_data(0), in.block_len(0));
    }
    if (in.empty()) return ParseFromArray("", 0);
    static thread_local std::string tmp;
    tmp.resize(in.size());
    in.copy_to(&tmp[0], in.size());
    return ParseFromArray(tmp.data(), tmp.size());
}

namespace {
template <typename T>
void append_elems(Message* m, const FieldDescriptor* f, const void* v, size_t n) {
    const T* p = static_cast<const T*>(v);
    auto& vec = ref<std::vector<T>>(m, f);
    vec.insert(vec.end(), p, p + n);
}
void append_decoded(Message* m, const FieldDescriptor* f, const void* v, size_t n) {
    switch (f->cpp_type()) {
    case CppType::BOOL: append_elems<uint8_t>(m, f, v, n); break;
    case CppType::INT32:
    case CppType::ENUM: append_elems<int32_t>(m, f, v, n); break;
    case CppType::UINT32: append_elems<uint32_t>(m, f, v, n); break;
    case CppType::INT64: append_elems<int64_t>(m, f, v, n); break;
    case CppType::UINT64: append_elems<uint64_t>(m, f, v, n); break;
    default: break;
    }
}
}  // namespace

bool Message::MergeFromFieldTable(const uint8_t* data, size_t size, const uint64_t* fields, int nfields,
                                  PackedRunDecoder* decoder) {
    const Descriptor* d = GetDescriptor();
    // large packed varint runs go to the decoder first, all in one call
    std::vector<PackedRunIn> runs;
    std::vector<int> run_of;  // field row -> runs index (or -1)
    if (decoder) {
        const size_t min = std::max<size_t>(1, decoder->min_bytes());
        for (int i = 0; i < nfields; ++i) {
            const uint64_t tag = fields[2 * i], v = fields[2 * i + 1];
            if ((tag & 7) != WIRETYPE_LENGTH_DELIMITED || (v & 0xFFFFFFFFu) < min) continue;
            const FieldDescriptor* f = d->FindFieldByNumber((int)(tag >> 3));
            if (!f || !f->is_repeated() || !f->is_packable() || !IsVarintFieldType(f->type)) continue;
            const size_t off = (size_t)(v >> 32), len = (size_t)(v & 0xFFFFFFFFu);
            if (off > size || len > size - off) return false;
            if (run_of.empty()) run_of.assign(nfields, -1);
            run_of[i] = (int)runs.size();
            PackedRunIn r;
            r.p = data + off;
            r.len = len;
            r.type = f->type;
            r.elem_bytes = elem_bytes(f->type);
            runs.push_back(r);
        }
        if (!runs.empty()) decoder->Decode(&runs);
    }
    for (int i = 0; i < nfields; ++i) {
        if (!run_of.empty() && run_of[i] >= 0 && runs[run_of[i]].values) {
            const PackedRunIn& r = runs[run_of[i]];
            append_decoded(this, d->FindFieldByNumber((int)(fields[2 * i] >> 3)), r.values, r.count);
            continue;
        }
        const uint64_t tag = fields[2 * i], v = fields[2 * i + 1];
        const WireType wt = (WireType)(tag & 7);
        const FieldDescriptor* f = d->FindFieldByNumber((int)(tag >> 3));
        if (!f || f->type == FieldType::GROUP) return false;
        if (wt != WIRETYPE_LENGTH_DELIMITED) {
            if (wt != wire_type_of(f->type)) return false;
            store_number(this, f, v);
            continue;
        }
        const size_t off = (size_t)(v >> 32), len = (size_t)(v & 0xFFFFFFFFu);
        if (off > size || len > size - off) return false;
        const uint8_t* p = data + off;
        if (f->is_repeated() && f->is_packable()) {
            if (!parse_packed(this, f, p, len)) return false;
            continue;
        }
        switch (f->cpp_type()) {
        case CppType::STRING:
            if (f->is_repeated()) {
                ref<std::vector<std::string>>(this, f).emplace_back((const char*)p, len);
            } else {
                if (f->oneof_index >= 0) ClearOneofSiblings(this, f);
                ref<std::string>(this, f).assign((const char*)p, len);
                set_has(this, f);
            }
            break;
        case CppType::MESSAGE: {
            Message* sub = f->is_repeated() ? Reflection::AddMessage(this, f) : Reflection::MutableMessage(this, f);
            CodedInput in(p, len);
            if (!parse_message(sub, &in) || !in.at_limit()) return false;
            break;
        }
        default:
            return false;  // a scalar field sent length-delimited but not packable
        }
    }
    return true;
}

// ---------------------------------------------------------------- text format
static void escape_bytes(const std::string& s, std::string* out) {
    for (unsigned char c : s) {
        switch (c) {
        case '\n': *out += "\\n"; break;
        case '\r': *out += "\\r"; break;
        case '\t': *out += "\\t"; break;
        case '"': *out += "\\\""; break;
        case '\\': *out += "\\\\"; break;
        default:
            if (c < 0x20 || c >= 0x7f) {
                char b[8];
                snprintf(b, sizeof(b), "\\%03o", c);
                *out += b;
            } else {
                out->push_back((char)c);
            }
        }
    }
}

static void scalar_text(const Message& m, const FieldDescriptor* f, int idx, std::string* out) {
    char b[64];
    const bool rep = idx >= 0;
    switch (f->cpp_type()) {
    case CppType::INT32: snprintf(b, sizeof(b), "%d", rep ? Reflection::GetRepeatedInt32(m, f, idx) : Reflection::GetInt32(m, f)); *out += b; break;
    case CppType::INT64: snprintf(b, sizeof(b), "%lld", (long long)(rep ? Reflection::GetRepeatedInt64(m, f, idx) : Reflection::GetInt64(m, f))); *out += b; break;
    case CppType::UINT32: snprintf(b, sizeof(b), "%u", rep ? Reflection::GetRepeatedUInt32(m, f, idx) : Reflection::GetUInt32(m, f)); *out += b; break;
    case CppType::UINT64: snprintf(b, sizeof(b), "%llu", (unsigned long long)(rep ? Reflection::GetRepeatedUInt64(m, f, idx) : Reflection::GetUInt64(m, f))); *out += b; break;
    case CppType::FLOAT: snprintf(b, sizeof(b), "%g", rep ? Reflection::GetRepeatedFloat(m, f, idx) : Reflection::GetFloat(m, f)); *out += b; break;
    case CppType::DOUBLE: snprintf(b, sizeof(b), "%.17g", rep ? Reflection::GetRepeatedDouble(m, f, idx) : Reflection::GetDouble(m, f)); *out += b; break;
    case CppType::BOOL: *out += (rep ? Reflection::GetRepeatedBool(m, f, idx) : Reflection::GetBool(m, f)) ? "true" : "false"; break;
    case CppType::ENUM: {
        int v = rep ? Reflection::GetRepeatedEnumValue(m, f, idx) : Reflection::GetEnumValue(m, f);
        const EnumValueDescriptor* ev = f->enum_type ? f->enum_type->FindValueByNumber(v) : nullptr;
        if (ev) *out += ev->name;
        else *out += std::to_string(v);
        break;
    }
    case CppType::STRING:
        *out += '"';
        escape_bytes(rep ? Reflection::GetRepeatedString(m, f, idx) : Reflection::GetString(m, f), out);
        *out += '"';
        break;
    case CppType::MESSAGE: break;
    }
}

static void debug_string_impl(const Message& m, int indent, bool single_line, std::string* out) {
    const Descriptor* d = m.GetDescriptor();
    const std::string pad = single_line ? "" : std::string(indent * 2, ' ');
    const char* nl = single_line ? " " : "\n";
    for (const FieldDescriptor& fd : d->fields) {
        const FieldDescriptor* f = &fd;
        int n = f->is_repeated() ? Reflection::FieldSize(m, f) : (Reflection::HasField(m, f) ? 1 : 0);
        for (int i = 0; i < n; ++i) {
            const int idx = f->is_repeated() ? i : -1;
            if (f->cpp_type() == CppType::MESSAGE) {
                *out += pad + f->name + " {" + nl;
                const Message& sub = idx >= 0 ? Reflection::GetRepeatedMessage(m, f, idx) : Reflection::GetMessage(m, f);
                debug_string_impl(sub, indent + 1, single_line, out);
                *out += pad + "}" + nl;
            } else {
                *out += pad + f->name + ": ";
                scalar_text(m, f, idx, out);
                *out += nl;
            }
        }
    }
}

std::string Message::DebugString() const {
    std::string s;
    debug_string_impl(*this, 0, false, &s);
    return s;
}

std::string Message::ShortDebugString() const {
    std::string s;
    debug_string_impl(*this, 0, true, &s);
    while (!s.empty() && s.back() == ' ') s.pop_back();
    return s;
}

// ---------------------------------------------------------------- Reflection

bool Reflection::HasField(const Message& m, const FieldDescriptor* f) {
    if (f->is_repeated()) return FieldSize(m, f) > 0;
    return field_present(m, f);
}

int Reflection::FieldSize(const Message& m, const FieldDescriptor* f) {
    if (!f->is_repeated()) return HasField(m, f) ? 1 : 0;
    switch (f->cpp_type()) {
    case CppType::STRING: return (int)cref<std::vector<std::string>>(m, f).size();
    case CppType::MESSAGE: return cref<RepeatedPtrBase>(m, f).size();
    default: return (int)raw_repeated(m, f).n;
    }
}

void Reflection::ClearField(Message* m, const FieldDescriptor* f) {
    if (f->is_repeated()) {
        clear_repeated(m, f);
        return;
    }
    if (f->cpp_type() == CppType::MESSAGE) {
        Message*& sub = ref<Message*>(m, f);
        delete sub;
        sub = nullptr;
    } else {
        set_scalar_default(m, f);
    }
    clear_has(m, f);
}

void Reflection::SetHasBit(Message* m, const FieldDescriptor* f) { set_has(m, f); }

void ClearOneofSiblings(Message* m, const FieldDescriptor* f) {
    const Descriptor* d = f->containing_type;
    for (const FieldDescriptor& o : d->fields) {
        if (&o != f && o.oneof_index == f->oneof_index && o.oneof_index >= 0) {
            if (field_present(*m, &o)) Reflection::ClearField(m, &o);
        }
    }
}

const Message& DefaultInstanceOf(const Descriptor* d) {
    CHECK(d->prototype) << "no prototype for " << d->full_name;
    return *d->prototype;
}

#define MRPC_SCALAR_REFL(Name, T, Storage)                                                        \
    T Reflection::Get##Name(const Message& m, const FieldDescriptor* f) { return (T)cref<Storage>(m, f); } \
    void Reflection::Set##Name(Message* m, const FieldDescriptor* f, T v) {                       \
        ref<Storage>(m, f) = (Storage)v;                                                          \
        if (f->oneof_index >= 0) ClearOneofSiblings(m, f);                                        \
        set_has(m, f);                                                                            \
    }                                                                                             \
    T Reflection::GetRepeated##Name(const Message& m, const FieldDescriptor* f, int i) {          \
        return (T)cref<std::vector<Storage>>(m, f)[i];                                            \
    }                                                                                             \
    void Reflection::Add##Name(Message* m, const FieldDescriptor* f, T v) { ref<std::vector<Storage>>(m, f).push_back((Storage)v); }

MRPC_SCALAR_REFL(Int32, int32_t, int32_t)
MRPC_SCALAR_REFL(Int64, int64_t, int64_t)
MRPC_SCALAR_REFL(UInt32, uint32_t, uint32_t)
MRPC_SCALAR_REFL(UInt64, uint64_t, uint64_t)
MRPC_SCALAR_REFL(Float, float, float)
MRPC_SCALAR_REFL(Double, double, double)
MRPC_SCALAR_REFL(EnumValue, int, int32_t)
#undef MRPC_SCALAR_REFL

bool Reflection::GetBool(const Message& m, const FieldDescriptor* f) { return cref<bool>(m, f); }
void Reflection::SetBool(Message* m, const FieldDescriptor* f, bool v) {
    ref<bool>(m, f) = v;
    if (f->oneof_index >= 0) ClearOneofSiblings(m, f);
    set_has(m, f);
}
bool Reflection::GetRepeatedBool(const Message& m, const FieldDescriptor* f, int i) {
    return cref<std::vector<uint8_t>>(m, f)[i] != 0;
}
void Reflection::AddBool(Message* m, const FieldDescriptor* f, bool v) { ref<std::vector<uint8_t>>(m, f).push_back(v ? 1 : 0); }

const std::string& Reflection::GetString(const Message& m, const FieldDescriptor* f) { return cref<std::string>(m, f); }
void Reflection::SetString(Message* m, const FieldDescriptor* f, const std::string& v) {
    ref<std::string>(m, f) = v;
    if (f->oneof_index >= 0) ClearOneofSiblings(m, f);
    set_has(m, f);
}
std::string* Reflection::MutableString(Message* m, const FieldDescriptor* f) {
    if (f->oneof_index >= 0) ClearOneofSiblings(m, f);
    set_has(m, f);
    return &ref<std::string>(m, f);
}
const std::string& Reflection::GetRepeatedString(const Message& m, const FieldDescriptor* f, int i) {
    return cref<std::vector<std::string>>(m, f)[i];
}
void Reflection::AddString(Message* m, const FieldDescriptor* f, const std::string& v) {
    ref<std::vector<std::string>>(m, f).push_back(v);
}

const Message& Reflection::GetMessage(const Message& m, const FieldDescriptor* f) {
    const Message* sub = cref<Message*>(m, f);
    return sub ? *sub : DefaultInstanceOf(f->message_type);
}
Message* Reflection::MutableMessage(Message* m, const FieldDescriptor* f) {
    Message*& sub = ref<Message*>(m, f);
    if (!sub) {
        if (f->oneof_index >= 0) ClearOneofSiblings(m, f);
        sub = f->message_type->NewMessage();
        set_has(m, f);
    }
    return sub;
}
const Message& Reflection::GetRepeatedMessage(const Message& m, const FieldDescriptor* f, int i) {
    return *cref<RepeatedPtrBase>(m, f).Get(i);
}
Message* Reflection::AddMessage(Message* m, const FieldDescriptor* f) {
    Message* sub = f->message_type->NewMessage();
    ref<RepeatedPtrBase>(m, f).AddAllocated(sub);
    return sub;
}

}  // namespace pb
}  // namespace mrpc
