// Message/enum/service descriptors with storage layout (offsets + has-bits),
// shared by generated messages and runtime-built DynamicMessages. Role of
// google::protobuf::Descriptor* as used by the reference (service
// registration, json2pb, rpc_press's DynamicMessageFactory, /protobufs).
#pragma once

#include <atomic>

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace mrpc {
namespace pb {

class Message;
class Descriptor;
class EnumDescriptor;
class FileDescriptor;
class ServiceDescriptor;

enum class FieldType : uint8_t {
    DOUBLE = 1, FLOAT = 2, INT64 = 3, UINT64 = 4, INT32 = 5, FIXED64 = 6, FIXED32 = 7, BOOL = 8,
    STRING = 9, GROUP = 10, MESSAGE = 11, BYTES = 12, UINT32 = 13, ENUM = 14, SFIXED32 = 15,
    SFIXED64 = 16, SINT32 = 17, SINT64 = 18,
};
enum class Label : uint8_t { OPTIONAL = 1, REQUIRED = 2, REPEATED = 3 };
enum class CppType : uint8_t { INT32, INT64, UINT32, UINT64, DOUBLE, FLOAT, BOOL, ENUM, STRING, MESSAGE };

const char* FieldTypeName(FieldType t);
// inline: message.cc's reflective serialize / size / parse loops ask it per
// field (2.6% of the 32 B echo's host samples as an out-of-line call)
inline CppType CppTypeOf(FieldType t) {
    static constexpr CppType kMap[19] = {
        CppType::INT32,  CppType::DOUBLE, CppType::FLOAT,  CppType::INT64,   CppType::UINT64,
        CppType::INT32,  CppType::UINT64, CppType::UINT32, CppType::BOOL,    CppType::STRING,
        CppType::MESSAGE, CppType::MESSAGE, CppType::STRING, CppType::UINT32, CppType::ENUM,
        CppType::INT32,  CppType::INT64,  CppType::INT32,  CppType::INT64,
    };
    const unsigned i = (unsigned)t;
    return i < 19 ? kMap[i] : CppType::INT32;
}
size_t CppTypeSize(CppType t);   // storage size of a singular field
size_t CppTypeAlign(CppType t);

struct EnumValueDescriptor {
    std::string name;
    int number;
};

class EnumDescriptor {
public:
    std::string name;
    std::string full_name;
    const FileDescriptor* file = nullptr;
    std::vector<EnumValueDescriptor> values;
    const EnumValueDescriptor* FindValueByNumber(int n) const;
    const EnumValueDescriptor* FindValueByName(const std::string& s) const;
};

class FieldDescriptor {
public:
    std::string name;
    std::string json_name;
    int number = 0;
    FieldType type = FieldType::INT32;
    Label label = Label::OPTIONAL;
    bool packed = false;
    bool proto3_implicit = false;  // proto3 singular without `optional`: no has-bit
    std::string type_name;         // fully-qualified for MESSAGE/ENUM (".pkg.Msg")
    const Descriptor* message_type = nullptr;
    const EnumDescriptor* enum_type = nullptr;
    const Descriptor* containing_type = nullptr;
    int index = 0;
    int oneof_index = -1;
    // default value (proto2)
    bool has_default = false;
    std::string default_str;  // textual
    int64_t default_int = 0;
    uint64_t default_uint = 0;
    double default_double = 0;
    std::string default_string;
    // layout
    uint32_t offset = 0;
    int32_t has_bit = -1;
    std::map<std::string, std::string> options;

    bool is_repeated() const { return label == Label::REPEATED; }
    bool is_required() const { return label == Label::REQUIRED; }
    bool is_map() const;
    CppType cpp_type() const { return CppTypeOf(type); }
    bool is_packable() const { return cpp_type() != CppType::STRING && cpp_type() != CppType::MESSAGE; }
};

class Descriptor {
public:
    std::string name;
    std::string full_name;
    const FileDescriptor* file = nullptr;
    const Descriptor* containing_type = nullptr;
    std::vector<FieldDescriptor> fields;
    std::vector<std::string> oneof_names;
    std::vector<Descriptor*> nested_types;
    std::vector<EnumDescriptor*> enum_types;
    bool map_entry = false;
    bool proto3 = false;
    // layout
    uint32_t has_bits_offset = 0;
    uint32_t num_has_bits = 0;
    uint32_t object_size = 0;
    Message* (*factory)() = nullptr;  // generated messages
    const Message* prototype = nullptr;  // default instance (generated or dynamic)
    bool owns_prototype = false;         // dynamic prototypes die with their descriptor
    // Generated mcpack codec of this message (mcpack::MessageHandler*,
    // installed by `mrpc_protoc --mcpack_out` output at static init).
    std::atomic<const void*> mcpack_handler{nullptr};
    Descriptor() = default;
    Descriptor(const Descriptor&) = delete;
    Descriptor& operator=(const Descriptor&) = delete;
    ~Descriptor();

    int field_count() const { return (int)fields.size(); }
    const FieldDescriptor* field(int i) const { return &fields[i]; }
    const FieldDescriptor* FindFieldByNumber(int n) const;
    const FieldDescriptor* FindFieldByName(const std::string& s) const;
    const FieldDescriptor* FindFieldByJsonName(const std::string& s) const;
    void BuildIndex();  // call once fields are final
    Message* NewMessage() const;

private:
    std::vector<int> _by_number;  // number -> index+1 (dense for small numbers)
    std::map<int, int> _by_number_sparse;
    std::map<std::string, int> _by_name;
};

class MethodDescriptor {
public:
    std::string name;
    std::string full_name;
    const ServiceDescriptor* service = nullptr;
    const Descriptor* input_type = nullptr;
    const Descriptor* output_type = nullptr;
    std::string input_type_name;
    std::string output_type_name;
    int index = 0;
    bool client_streaming = false;
    bool server_streaming = false;
    std::map<std::string, std::string> options;  // e.g. "(brpc.method_timeout)"
};

class ServiceDescriptor {
public:
    std::string name;
    std::string full_name;
    const FileDescriptor* file = nullptr;
    std::vector<MethodDescriptor> methods;
    std::map<std::string, std::string> options;
    int method_count() const { return (int)methods.size(); }
    const MethodDescriptor* method(int i) const { return &methods[i]; }
    const MethodDescriptor* FindMethodByName(const std::string& n) const;
};

class FileDescriptor {
public:
    std::string name;  // relative path, e.g. "echo.proto"
    std::string package;
    std::string syntax = "proto2";
    std::vector<std::string> dependencies;
    std::vector<Descriptor*> message_types;
    std::vector<EnumDescriptor*> enum_types;
    std::vector<ServiceDescriptor*> services;
    std::map<std::string, std::string> options;
    std::string source;  // original .proto text, for /protobufs
    // Storage of descriptors parsed at run time (the lists above only point
    // into it; generated files keep theirs in static registries instead).
    std::vector<std::unique_ptr<Descriptor>> owned_messages;
    std::vector<std::unique_ptr<EnumDescriptor>> owned_enums;
    std::vector<std::unique_ptr<ServiceDescriptor>> owned_services;
};

// Global registry of all known descriptors (generated pool + runtime pools).
class DescriptorPool {
public:
    static DescriptorPool* generated_pool();
    void AddFile(FileDescriptor* f);  // takes ownership, registers all symbols
    const FileDescriptor* FindFileByName(const std::string& n) const;
    const Descriptor* FindMessageTypeByName(const std::string& full_name) const;
    const EnumDescriptor* FindEnumTypeByName(const std::string& full_name) const;
    const ServiceDescriptor* FindServiceByName(const std::string& full_name) const;
    const MethodDescriptor* FindMethodByName(const std::string& full_name) const;
    std::vector<const FileDescriptor*> files() const;
    std::vector<const ServiceDescriptor*> services() const;

private:
    void add_message(Descriptor* d);
    mutable std::mutex _mu;
    std::vector<std::unique_ptr<FileDescriptor>> _files;
    std::map<std::string, const FileDescriptor*> _file_by_name;
    std::map<std::string, const Descriptor*> _messages;
    std::map<std::string, const EnumDescriptor*> _enums;
    std::map<std::string, const ServiceDescriptor*> _services;
};

std::string ToJsonName(const std::string& field_name);

}  // namespace pb
}  // namespace mrpc
