// Framed thrift over TBinaryProtocol without the Apache thrift library
// (role of the reference's src/brpc/thrift_message.h, thrift_service.h and
// policy/thrift_protocol.cpp, which wrap generated thrift classes).
//
// Messages are handled as dynamic value trees (ThriftValue) encoded with
// the strict binary protocol:
//   frame   | length i32 BE | message |
//   message | 0x8001 | 0x00 | type u8 | name (i32 len + bytes) | seqid i32 | struct |
//   struct  | { field-type u8 | field-id i16 | value }* | STOP(0) |
// A call's struct holds the arguments; a reply's struct holds field 0
// (success) or declared exceptions (ids >= 1); an EXCEPTION message holds a
// TApplicationException {1: message, 2: type}.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "base/buf.h"
#include "pb/message.h"
#include "pb/service.h"

namespace mrpc {

class Controller;
class Server;

namespace thrift {

enum TType : uint8_t {
    T_STOP = 0, T_VOID = 1, T_BOOL = 2, T_BYTE = 3, T_DOUBLE = 4, T_I16 = 6, T_I32 = 8, T_I64 = 10,
    T_STRING = 11, T_STRUCT = 12, T_MAP = 13, T_SET = 14, T_LIST = 15,
};
enum MessageType : uint8_t { T_CALL = 1, T_REPLY = 2, T_EXCEPTION = 3, T_ONEWAY = 4 };

// TApplicationException types.
enum AppExceptionType {
    TAPP_UNKNOWN = 0, TAPP_UNKNOWN_METHOD = 1, TAPP_INVALID_MESSAGE_TYPE = 2, TAPP_WRONG_METHOD_NAME = 3,
    TAPP_BAD_SEQUENCE_ID = 4, TAPP_MISSING_RESULT = 5, TAPP_INTERNAL_ERROR = 6, TAPP_PROTOCOL_ERROR = 7,
};

class Value {
public:
    Value() : _type(T_VOID) {}
    static Value Bool(bool v) { Value x(T_BOOL); x._i = v; return x; }
    static Value Byte(int8_t v) { Value x(T_BYTE); x._i = v; return x; }
    static Value I16(int16_t v) { Value x(T_I16); x._i = v; return x; }
    static Value I32(int32_t v) { Value x(T_I32); x._i = v; return x; }
    static Value I64(int64_t v) { Value x(T_I64); x._i = v; return x; }
    static Value Double(double v) { Value x(T_DOUBLE); x._d = v; return x; }
    static Value String(const std::string& v) { Value x(T_STRING); x._s = v; return x; }
    static Value Struct() { return Value(T_STRUCT); }
    static Value List(TType elem) { Value x(T_LIST); x._elem = elem; return x; }
    static Value Set(TType elem) { Value x(T_SET); x._elem = elem; return x; }
    static Value Map(TType key, TType val) { Value x(T_MAP); x._key = key; x._elem = val; return x; }

    TType type() const { return _type; }
    bool is_void() const { return _type == T_VOID; }
    int64_t as_int() const { return _i; }
    bool as_bool() const { return _i != 0; }
    double as_double() const { return _d; }
    const std::string& as_string() const { return _s; }

    // struct
    Value& field(int16_t id) { return _fields[id]; }
    const Value* find(int16_t id) const {
        auto it = _fields.find(id);
        return it == _fields.end() ? nullptr : &it->second;
    }
    const std::map<int16_t, Value>& fields() const { return _fields; }
    // list / set
    TType elem_type() const { return _elem; }
    std::vector<Value>& elems() { return _elems; }
    const std::vector<Value>& elems() const { return _elems; }
    // map
    TType key_type() const { return _key; }
    std::vector<std::pair<Value, Value>>& pairs() { return _pairs; }
    const std::vector<std::pair<Value, Value>>& pairs() const { return _pairs; }

    bool operator==(const Value& o) const;
    bool operator!=(const Value& o) const { return !(*this == o); }
    std::string DebugString() const;

private:
    explicit Value(TType t) : _type(t) {}
    TType _type;
    TType _elem = T_STOP, _key = T_STOP;
    int64_t _i = 0;
    double _d = 0;
    std::string _s;
    std::map<int16_t, Value> _fields;
    std::vector<Value> _elems;
    std::vector<std::pair<Value, Value>> _pairs;
};

// TBinaryProtocol codec.
void WriteValue(std::string* out, const Value& v);
void WriteStruct(std::string* out, const Value& s);  // fields + STOP
// Returns bytes consumed, 0 on malformed/truncated input.
size_t ReadValue(const char* p, size_t n, TType type, Value* v, int depth = 0);

struct MessageHeader {
    std::string name;
    MessageType type = T_CALL;
    int32_t seqid = 0;
};
void WriteMessage(std::string* out, const MessageHeader& h, const Value& body);
// Parses a (unframed) message; false if malformed.
bool ReadMessage(const char* p, size_t n, MessageHeader* h, Value* body);

}  // namespace thrift

// Request/response of framed-thrift calls (Channel protocol "thrift").
//  client: set method_name + body (the args struct) on the request; the
//          response's body is the result struct (field 0 = success).
//  server: ThriftService sees the args struct and fills the result struct.
class ThriftFramedMessage : public pb::Message {
public:
    std::string method_name;
    int32_t seq_id = 0;
    thrift::Value body = thrift::Value::Struct();
    const pb::Descriptor* GetDescriptor() const override { return OpaqueDescriptor("mrpc.ThriftFramedMessage"); }
    pb::Message* New() const override { return new ThriftFramedMessage; }
    void Clear() override {
        method_name.clear();
        seq_id = 0;
        body = thrift::Value::Struct();
    }
    // result helpers
    const thrift::Value* success() const { return body.find(0); }
};

class ThriftService {
public:
    ThriftService();
    virtual ~ThriftService();
    // Fill response->body (result struct). Failing cntl sends a
    // TApplicationException carrying the error text.
    virtual void ProcessThriftFramedRequest(Controller* cntl, ThriftFramedMessage* request,
                                            ThriftFramedMessage* response, Closure* done) = 0;
    class MethodStatus* status() const { return _status.get(); }

private:
    std::unique_ptr<class MethodStatus> _status;
};

}  // namespace mrpc
