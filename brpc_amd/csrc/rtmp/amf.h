// AMF0 codec for RTMP commands and metadata (role of the reference's
// src/brpc/amf.h/.cpp). Values form a small dynamic tree:
// number, boolean, string (short/long), object, ecma-array, strict-array,
// null, undefined, date.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

namespace mrpc {
namespace rtmp {

enum AMFType : uint8_t {
    AMF_NUMBER = 0x00,
    AMF_BOOLEAN = 0x01,
    AMF_STRING = 0x02,
    AMF_OBJECT = 0x03,
    AMF_NULL = 0x05,
    AMF_UNDEFINED = 0x06,
    AMF_ECMA_ARRAY = 0x08,
    AMF_OBJECT_END = 0x09,
    AMF_STRICT_ARRAY = 0x0A,
    AMF_DATE = 0x0B,
    AMF_LONG_STRING = 0x0C,
};

class AMFValue {
public:
    AMFValue() : _type(AMF_UNDEFINED) {}
    static AMFValue Number(double v) { AMFValue x(AMF_NUMBER); x._num = v; return x; }
    static AMFValue Bool(bool v) { AMFValue x(AMF_BOOLEAN); x._num = v ? 1 : 0; return x; }
    static AMFValue String(const std::string& s) { AMFValue x(AMF_STRING); x._str = s; return x; }
    static AMFValue Null() { return AMFValue(AMF_NULL); }
    static AMFValue Undefined() { return AMFValue(AMF_UNDEFINED); }
    static AMFValue Object() { return AMFValue(AMF_OBJECT); }
    static AMFValue EcmaArray() { return AMFValue(AMF_ECMA_ARRAY); }
    static AMFValue StrictArray() { return AMFValue(AMF_STRICT_ARRAY); }
    static AMFValue Date(double ms) { AMFValue x(AMF_DATE); x._num = ms; return x; }

    AMFType type() const { return _type; }
    bool is_null() const { return _type == AMF_NULL || _type == AMF_UNDEFINED; }
    double number() const { return _num; }
    bool boolean() const { return _num != 0; }
    const std::string& str() const { return _str; }

    // object / ecma array (insertion ordered)
    AMFValue& Set(const std::string& key, const AMFValue& v);
    const AMFValue* Find(const std::string& key) const;
    const std::vector<std::pair<std::string, AMFValue>>& props() const { return _props; }
    // strict array
    std::vector<AMFValue>& items() { return _items; }
    const std::vector<AMFValue>& items() const { return _items; }

    std::string DebugString() const;

private:
    explicit AMFValue(AMFType t) : _type(t) {}
    AMFType _type;
    double _num = 0;
    std::string _str;
    std::vector<std::pair<std::string, AMFValue>> _props;
    std::vector<AMFValue> _items;
};

void WriteAMF(std::string* out, const AMFValue& v);
// Returns bytes consumed (0 when malformed/truncated).
size_t ReadAMF(const char* p, size_t n, AMFValue* v, int depth = 0);
// A sequence of values (a command: name, transaction id, args...).
bool ReadAMFList(const char* p, size_t n, std::vector<AMFValue>* out);

}  // namespace rtmp
}  // namespace mrpc
