// Message base class + table-driven (descriptor/offset based) codec and
// reflection. Generated classes (mrpc_protoc) and DynamicMessage share the
// same storage conventions so one codec serves both:
//   int32/sint32/sfixed32/enum -> int32_t     int64/sint64/sfixed64 -> int64_t
//   uint32/fixed32 -> uint32_t                uint64/fixed64 -> uint64_t
//   float, double, bool                        string/bytes -> std::string
//   message -> Message* (nullptr = unset)
//   repeated scalar T -> std::vector<T> (bool -> std::vector<uint8_t>)
//   repeated string -> std::vector<std::string>
//   repeated message -> RepeatedPtrBase (std::vector<Message*>)
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "pb/descriptor.h"
#include "pb/wire.h"

namespace mrpc {
class Buf;
namespace pb {

class Message {
public:
    Message() : _cached_size(0) {}
    virtual ~Message();
    virtual const Descriptor* GetDescriptor() const = 0;
    virtual Message* New() const = 0;

    virtual void Clear();
    virtual size_t ByteSizeLong() const;
    virtual uint8_t* SerializeWithCachedSizesToArray(uint8_t* target) const;
    virtual bool MergePartialFromCodedInput(CodedInput* in);

    int ByteSize() const { return (int)ByteSizeLong(); }
    int GetCachedSize() const { return _cached_size; }
    void SetCachedSize(int s) const { _cached_size = s; }

    bool IsInitialized() const;
    std::string InitializationErrorString() const;
    void CopyFrom(const Message& from);
    void MergeFrom(const Message& from);

    bool SerializeToString(std::string* out) const;
    std::string SerializeAsString() const;
    bool SerializeToArray(void* data, int size) const;
    bool AppendToString(std::string* out) const;
    bool SerializeToBuf(Buf* out) const;
    bool ParseFromArray(const void* data, size_t size);
    bool ParsePartialFromArray(const void* data, size_t size);
    bool ParseFromString(const std::string& s) { return ParseFromArray(s.data(), s.size()); }
    bool MergeFromString(const std::string& s);
    bool ParseFromBuf(const Buf& in);
    // Merges the top-level fields listed in a wire-scan table (the GPU
    // pb_scan layout: {tag, value} pairs, value = the number for wires
    // 0/1/5, (offset << 32) | length into `data` for wire 2) instead of
    // walking the bytes; nested messages and packed runs are parsed from
    // their ranges. False for anything the table cannot express (unknown
    // fields, mismatched wire types, groups, ranges outside data): the
    // caller then parses the bytes normally.
    bool MergeFromFieldTable(const uint8_t* data, size_t size, const uint64_t* fields, int nfields,
                             class PackedRunDecoder* decoder = nullptr);
    std::string DebugString() const;
    std::string ShortDebugString() const;
    std::string GetTypeName() const { return GetDescriptor()->full_name; }

    const std::string& unknown_fields() const { return _unknown; }
    std::string* mutable_unknown_fields() { return &_unknown; }

protected:
    mutable int _cached_size;
    std::string _unknown;
};

class RepeatedPtrBase {
public:
    RepeatedPtrBase() {}
    ~RepeatedPtrBase() { Clear(); }
    RepeatedPtrBase(const RepeatedPtrBase&) = delete;
    RepeatedPtrBase& operator=(const RepeatedPtrBase&) = delete;
    int size() const { return (int)_v.size(); }
    bool empty() const { return _v.empty(); }
    void Clear() {
        for (Message* m : _v) delete m;
        _v.clear();
    }
    Message* AddMessage(const Message* prototype) {
        Message* m = prototype->New();
        _v.push_back(m);
        return m;
    }
    void AddAllocated(Message* m) { _v.push_back(m); }
    Message* Get(int i) const { return _v[i]; }
    void RemoveLast() {
        delete _v.back();
        _v.pop_back();
    }
    void SwapElements(int a, int b) { std::swap(_v[a], _v[b]); }
    std::vector<Message*>& raw() { return _v; }
    const std::vector<Message*>& raw() const { return _v; }

protected:
    std::vector<Message*> _v;
};

template <typename T>
class RepeatedPtrField : public RepeatedPtrBase {
public:
    T* Add() {
        T* t = new T;
        _v.push_back(t);
        return t;
    }
    const T& Get(int i) const { return *static_cast<const T*>(_v[i]); }
    T* Mutable(int i) { return static_cast<T*>(_v[i]); }
    const T& operator[](int i) const { return Get(i); }
    class const_iterator {
    public:
        explicit const_iterator(std::vector<Message*>::const_iterator it) : _it(it) {}
        const T& operator*() const { return *static_cast<const T*>(*_it); }
        const T* operator->() const { return static_cast<const T*>(*_it); }
        const_iterator& operator++() { ++_it; return *this; }
        bool operator!=(const const_iterator& o) const { return _it != o._it; }
    private:
        std::vector<Message*>::const_iterator _it;
    };
    const_iterator begin() const { return const_iterator(_v.begin()); }
    const_iterator end() const { return const_iterator(_v.end()); }
};

// Descriptor-driven reflection over any Message (generated or dynamic).
class Reflection {
public:
    static bool HasField(const Message& m, const FieldDescriptor* f);
    static int FieldSize(const Message& m, const FieldDescriptor* f);
    static void ClearField(Message* m, const FieldDescriptor* f);
    static void SetHasBit(Message* m, const FieldDescriptor* f);

    static int32_t GetInt32(const Message& m, const FieldDescriptor* f);
    static int64_t GetInt64(const Message& m, const FieldDescriptor* f);
    static uint32_t GetUInt32(const Message& m, const FieldDescriptor* f);
    static uint64_t GetUInt64(const Message& m, const FieldDescriptor* f);
    static float GetFloat(const Message& m, const FieldDescriptor* f);
    static double GetDouble(const Message& m, const FieldDescriptor* f);
    static bool GetBool(const Message& m, const FieldDescriptor* f);
    static int GetEnumValue(const Message& m, const FieldDescriptor* f);
    static const std::string& GetString(const Message& m, const FieldDescriptor* f);
    static const Message& GetMessage(const Message& m, const FieldDescriptor* f);

    static void SetInt32(Message* m, const FieldDescriptor* f, int32_t v);
    static void SetInt64(Message* m, const FieldDescriptor* f, int64_t v);
    static void SetUInt32(Message* m, const FieldDescriptor* f, uint32_t v);
    static void SetUInt64(Message* m, const FieldDescriptor* f, uint64_t v);
    static void SetFloat(Message* m, const FieldDescriptor* f, float v);
    static void SetDouble(Message* m, const FieldDescriptor* f, double v);
    static void SetBool(Message* m, const FieldDescriptor* f, bool v);
    static void SetEnumValue(Message* m, const FieldDescriptor* f, int v);
    static void SetString(Message* m, const FieldDescriptor* f, const std::string& v);
    static std::string* MutableString(Message* m, const FieldDescriptor* f);
    static Message* MutableMessage(Message* m, const FieldDescriptor* f);

    static int32_t GetRepeatedInt32(const Message& m, const FieldDescriptor* f, int i);
    static int64_t GetRepeatedInt64(const Message& m, const FieldDescriptor* f, int i);
    static uint32_t GetRepeatedUInt32(const Message& m, const FieldDescriptor* f, int i);
    static uint64_t GetRepeatedUInt64(const Message& m, const FieldDescriptor* f, int i);
    static float GetRepeatedFloat(const Message& m, const FieldDescriptor* f, int i);
    static double GetRepeatedDouble(const Message& m, const FieldDescriptor* f, int i);
    static bool GetRepeatedBool(const Message& m, const FieldDescriptor* f, int i);
    static int GetRepeatedEnumValue(const Message& m, const FieldDescriptor* f, int i);
    static const std::string& GetRepeatedString(const Message& m, const FieldDescriptor* f, int i);
    static const Message& GetRepeatedMessage(const Message& m, const FieldDescriptor* f, int i);
    // The element array of a repeated scalar field (its std::vector's data;
    // *elem_bytes 1/4/8) and its size; nullptr for strings and messages.
    static const void* RepeatedScalarData(const Message& m, const FieldDescriptor* f, size_t* n, size_t* elem_bytes);

    static void AddInt32(Message* m, const FieldDescriptor* f, int32_t v);
    static void AddInt64(Message* m, const FieldDescriptor* f, int64_t v);
    static void AddUInt32(Message* m, const FieldDescriptor* f, uint32_t v);
    static void AddUInt64(Message* m, const FieldDescriptor* f, uint64_t v);
    static void AddFloat(Message* m, const FieldDescriptor* f, float v);
    static void AddDouble(Message* m, const FieldDescriptor* f, double v);
    static void AddBool(Message* m, const FieldDescriptor* f, bool v);
    static void AddEnumValue(Message* m, const FieldDescriptor* f, int v);
    static void AddString(Message* m, const FieldDescriptor* f, const std::string& v);
    static Message* AddMessage(Message* m, const FieldDescriptor* f);
};

// Free helpers used by generated code.
void ClearOneofSiblings(Message* m, const FieldDescriptor* f);

// Device encoding of large packed varint runs (the body-encode
// half of the batched device codec). While a sink is installed on the
// calling thread, SerializeWithCachedSizesToArray writes the tag and the
// length of every packed varint-typed field with >= min_elems() elements,
// skips its payload and hands the run to the sink, which must fill
// [dst, dst + bytes) before the output is used (gpu/snappy_offload.cc does
// it in the codec batch, ahead of the compress kernel reading the body).
// Element layout is the field's vector: 1 (bool), 4 (32-bit) or 8 bytes.
constexpr size_t kPackedRunChunkElems = 2048;  // = gpu kPbRunChunkElems
struct PackedRun {
    uint8_t* dst = nullptr;
    const void* values = nullptr;
    size_t n = 0;
    size_t elem_bytes = 0;
    FieldType type = FieldType::INT32;
    size_t bytes = 0;
    std::vector<uint32_t> chunk_bytes;  // output bytes of each kPackedRunChunkElems elements
};
class PackedRunSink {
public:
    virtual ~PackedRunSink() {}
    virtual size_t min_elems() const = 0;
    virtual void Take(PackedRun&& run) = 0;
};
// The parse half: MergeFromFieldTable hands the top-level packed varint
// runs of >= min_bytes() bytes to a decoder in one call (one device round
// trip per message) and appends the decoded elements; a run it did not
// decode (values == nullptr) is parsed on the host.
struct PackedRunIn {
    const uint8_t* p = nullptr;  // the run's bytes (inside the decoded body)
    size_t len = 0;
    FieldType type = FieldType::INT32;
    size_t elem_bytes = 0;
    const void* values = nullptr;  // out: decoded elements in the field's vector layout
    size_t count = 0;              // out
};
class PackedRunDecoder {
public:
    virtual ~PackedRunDecoder() {}
    virtual size_t min_bytes() const = 0;
    // decoded arrays stay valid until the decoder is destroyed
    virtual void Decode(std::vector<PackedRunIn>* runs) = 0;
};
// Installs `sink` for this thread (nullptr: none); returns the previous one.
PackedRunSink* SetThreadPackedRunSink(PackedRunSink* sink);
// The host encoding of a run (what the serializer would have written):
// the fallback when the device could not encode it.
void EncodePackedRunOnHost(const PackedRun& run);
bool IsVarintFieldType(FieldType t);
}  // namespace pb
// Field-less descriptor for hand-written opaque messages (redis, memcache,
// nshead, thrift...): such messages carry their own wire encoding.
const pb::Descriptor* OpaqueDescriptor(const char* full_name);
namespace pb {
const Message& DefaultInstanceOf(const Descriptor* d);

}  // namespace pb
}  // namespace mrpc
