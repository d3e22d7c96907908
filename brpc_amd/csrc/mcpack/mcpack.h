// mcpack v2 / compack codec and protobuf <-> mcpack conversion
// (role of the reference's src/mcpack2pb/: field_type.h, serializer.h,
// parser.h, mcpack2pb.h and the protoc-gen-mcpack plugin).
//
// Wire format (all integers little endian):
//   fixed head  | type u8 | name_size u8 |                     name | value (type & 0xF bytes)
//   short head  | type|0x80 u8 | name_size u8 | value_size u8 | name | value   (string/binary <= 255 B)
//   long head   | type u8 | name_size u8 | value_size u32     | name | value
// name_size counts the terminating NUL (0 = unnamed item). Objects and
// arrays are long-headed and their value starts with a u32 item count;
// an isomorphic array (compack) stores one item-type byte followed by raw
// primitive values. A message is an anonymous top-level object.
//
// Conversion is driven by the runtime descriptors every mrpc message
// carries (the same reflection json2pb uses); `idl_name` / `idl_type` field
// options are honoured as in the reference's idl_options.proto. Like the
// reference's protoc-gen-mcpack (src/mcpack2pb/generator.cpp), `mrpc_protoc
// --mcpack_out=DIR` emits specialised per-message serialize/parse functions
// (no reflection, no name hashing per field) that register themselves as the
// message's MessageHandler; the entry points below dispatch to them and fall
// back to the descriptor walk for messages without generated code. Both
// paths produce identical bytes (tests/legacy_protocols_unittest.cc).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace mrpc {
class Buf;
namespace pb {
class Descriptor;
class FieldDescriptor;
class Message;
}
namespace mcpack {

enum FieldType : uint8_t {
    FIELD_UNKNOWN = 0,
    FIELD_OBJECT = 0x10,
    FIELD_ARRAY = 0x20,
    FIELD_ISOARRAY = 0x30,
    FIELD_OBJECTISOARRAY = 0x40,
    FIELD_STRING = 0x50,
    FIELD_BINARY = 0x60,
    FIELD_INT8 = 0x11,
    FIELD_INT16 = 0x12,
    FIELD_INT32 = 0x14,
    FIELD_INT64 = 0x18,
    FIELD_UINT8 = 0x21,
    FIELD_UINT16 = 0x22,
    FIELD_UINT32 = 0x24,
    FIELD_UINT64 = 0x28,
    FIELD_BOOL = 0x31,
    FIELD_FLOAT = 0x44,
    FIELD_DOUBLE = 0x48,
    FIELD_DATE = 0x58,
    FIELD_NULL = 0x61,
};
static const uint8_t FIELD_SHORT_MASK = 0x80;
static const uint8_t FIELD_FIXED_MASK = 0x0f;
static const uint8_t FIELD_NON_DELETED_MASK = 0x70;

enum Format { FORMAT_COMPACK = 0, FORMAT_MCPACK_V2 = 1 };

const char* type2str(uint8_t type);
inline bool is_primitive(uint8_t t) { return (t & FIELD_FIXED_MASK) != 0; }
inline size_t primitive_size(uint8_t t) { return t & FIELD_FIXED_MASK; }
inline bool is_integral(uint8_t t) { return is_primitive(t) && (t & 0xF0) < 0x40; }
inline bool is_floating(uint8_t t) { return is_primitive(t) && (t & 0xF0) == 0x40; }

// Streaming writer. Groups (objects/arrays) are opened and closed in LIFO
// order; their heads are patched with sizes and counts when closed.
class Serializer {
public:
    explicit Serializer(std::string* out) : _out(out) {}
    bool good() const { return _good; }

    void begin_object(const std::string& name = std::string());
    void end_object();
    // Array of `item_type`. With FORMAT_COMPACK and a primitive item type the
    // array is isomorphic (raw values); otherwise every item has a head.
    void begin_array(const std::string& name, uint8_t item_type, Format fmt);
    void end_array();

    void add_int8(const std::string& n, int8_t v) { add_fixed(n, FIELD_INT8, &v, 1); }
    void add_int16(const std::string& n, int16_t v) { add_fixed(n, FIELD_INT16, &v, 2); }
    void add_int32(const std::string& n, int32_t v) { add_fixed(n, FIELD_INT32, &v, 4); }
    void add_int64(const std::string& n, int64_t v) { add_fixed(n, FIELD_INT64, &v, 8); }
    void add_uint8(const std::string& n, uint8_t v) { add_fixed(n, FIELD_UINT8, &v, 1); }
    void add_uint16(const std::string& n, uint16_t v) { add_fixed(n, FIELD_UINT16, &v, 2); }
    void add_uint32(const std::string& n, uint32_t v) { add_fixed(n, FIELD_UINT32, &v, 4); }
    void add_uint64(const std::string& n, uint64_t v) { add_fixed(n, FIELD_UINT64, &v, 8); }
    void add_bool(const std::string& n, bool v) {
        const uint8_t b = v ? 1 : 0;
        add_fixed(n, FIELD_BOOL, &b, 1);
    }
    void add_float(const std::string& n, float v) { add_fixed(n, FIELD_FLOAT, &v, 4); }
    void add_double(const std::string& n, double v) { add_fixed(n, FIELD_DOUBLE, &v, 8); }
    void add_string(const std::string& n, const std::string& v);
    void add_binary(const std::string& n, const void* data, size_t len);
    void add_null(const std::string& n);
    // Typed primitive add: value given as raw little-endian bytes.
    void add_fixed(const std::string& name, uint8_t type, const void* value, size_t size);

private:
    struct Group {
        uint8_t type;
        uint8_t item_type;
        bool iso;
        size_t head_pos;   // offset of the long head
        size_t value_pos;  // offset where the value starts (after name)
        uint32_t count;
    };
    bool named_ok(const std::string& name);
    void put_head(uint8_t type, const std::string& name, size_t value_size);
    std::string* _out;
    std::vector<Group> _stack;
    bool _good = true;
};

// A read-only view of one encoded field value (name excluded).
class Value {
public:
    Value() {}
    Value(uint8_t type, const char* data, size_t size) : _type(type), _data(data), _size(size) {}
    uint8_t type() const { return _type; }
    const char* data() const { return _data; }
    size_t size() const { return _size; }
    bool is_null() const { return _type == FIELD_NULL; }
    // Conversions (numeric types convert into each other; false on mismatch).
    bool to_int64(int64_t* v) const;
    bool to_uint64(uint64_t* v) const;
    bool to_double(double* v) const;
    bool to_bool(bool* v) const;
    bool to_string(std::string* v) const;  // string (NUL dropped) or binary
    std::string DebugString() const;

private:
    uint8_t _type = FIELD_UNKNOWN;
    const char* _data = nullptr;
    size_t _size = 0;
};

// Decodes one head+name+value at `p` (within `n` bytes). Returns the number
// of bytes consumed or 0 if malformed/truncated.
size_t DecodeField(const char* p, size_t n, std::string* name, Value* value);

// Items of an object / array / isoarray value.
struct Item {
    std::string name;  // empty for array items
    Value value;
};
bool ListItems(const Value& group, std::vector<Item>* items);

// Generated per-message codec (see the header comment).
struct MessageHandler {
    // fields of msg into the currently open object
    bool (*serialize_fields)(const pb::Message& msg, Format fmt, Serializer* sr);
    // msg from an object value
    bool (*parse_object)(const Value& obj, pb::Message* msg);
};
void RegisterMessageHandler(const pb::Descriptor* d, const MessageHandler* h);
const MessageHandler* FindMessageHandler(const pb::Descriptor* d);
// Process-wide switch (tests/benchmarks compare the two paths).
void SetGeneratedHandlersEnabled(bool on);

// Helpers of the generated code: a number written with a wire type other
// than its natural one (idl_type), and a repeated message field from an
// object isoarray ({a=[..],b=[..]} columns).
void AddConverted(Serializer* sr, const std::string& name, uint8_t wire_type, int64_t iv, uint64_t uv, double dv,
                  bool is_float_src, bool is_unsigned_src);
bool ParseObjectIsoArrayField(const Value& v, pb::Message* msg, const pb::FieldDescriptor* f);

// pb <-> mcpack. The output is a complete top-level object.
bool SerializeToString(const pb::Message& msg, Format fmt, std::string* out);
bool SerializeToBuf(const pb::Message& msg, Format fmt, Buf* out);
// Serializes msg's fields into the currently open object of `sr`.
bool SerializeFields(const pb::Message& msg, Format fmt, Serializer* sr);
bool ParseFromArray(const char* data, size_t n, pb::Message* msg);
bool ParseFromBuf(const Buf& buf, pb::Message* msg);
// Fills msg from an object value (e.g. a nested "params" object).
bool ParseFromObject(const Value& obj, pb::Message* msg);
// The descriptor walk only (ignores generated handlers).
bool SerializeFieldsByReflection(const pb::Message& msg, Format fmt, Serializer* sr);
bool ParseFromObjectByReflection(const Value& obj, pb::Message* msg);

}  // namespace mcpack
}  // namespace mrpc
