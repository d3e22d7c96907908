// Small JSON DOM: parse / serialize (rapidjson is not available; the
// reference's json2pb builds on rapidjson, src/json2pb). Used by json2pb,
// naming services and builtin pages.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace mrpc {
namespace json {

class Value {
public:
    // RAW: pre-rendered JSON text written verbatim (an array of numbers
    // printed by the device, json2pb's SetPb2JsonArrayOffload)
    enum Type { NUL, BOOL, INT, UINT, DOUBLE, STRING, ARRAY, OBJECT, RAW };
    Value() : _type(NUL) {}
    // copies never share the packed view (it is rebuilt on demand), so a
    // copy never reads _view non-atomically while a reader publishes it
    Value(const Value& o)
        : _type(o._type), _b(o._b), _i(o._i), _u(o._u), _d(o._d), _s(o._s), _arr(o._arr), _ints(o._ints),
          _obj(o._obj) {}
    Value(Value&&) = default;
    Value& operator=(const Value& o) {
        if (this != &o) *this = Value(o);
        return *this;
    }
    Value& operator=(Value&&) = default;
    explicit Value(bool b) : _type(BOOL), _b(b) {}
    explicit Value(int64_t i) : _type(INT), _i(i) {}
    explicit Value(uint64_t u) : _type(UINT), _u(u) {}
    explicit Value(int i) : _type(INT), _i(i) {}
    explicit Value(double d) : _type(DOUBLE), _d(d) {}
    explicit Value(const std::string& s) : _type(STRING), _s(s) {}
    explicit Value(const char* s) : _type(STRING), _s(s) {}
    static Value Array() { Value v; v._type = ARRAY; return v; }
    static Value Object() { Value v; v._type = OBJECT; return v; }
    static Value Raw(std::string text) { Value v; v._type = RAW; v._s = std::move(text); return v; }

    Type type() const { return _type; }
    bool is_null() const { return _type == NUL; }
    bool is_bool() const { return _type == BOOL; }
    bool is_number() const { return _type == INT || _type == UINT || _type == DOUBLE; }
    bool is_int() const { return _type == INT || _type == UINT; }
    bool is_string() const { return _type == STRING; }
    bool is_array() const { return _type == ARRAY; }
    bool is_object() const { return _type == OBJECT; }

    bool as_bool() const { return _type == BOOL ? _b : (is_number() && as_double() != 0); }
    int64_t as_int() const;
    uint64_t as_uint() const;
    double as_double() const;
    const std::string& as_string() const { return _s; }
    std::string& mutable_string() { return _s; }
    bool uint_overflows_int() const { return _type == UINT && _u > (uint64_t)INT64_MAX; }

    // arrays. An array of integers parsed in bulk (the device parser of
    // SetIntArrayOffload) keeps them packed; packed_ints() lets json2pb take
    // them as they are. The const array() of a packed array builds a Value
    // view once (published atomically, so concurrent readers of one parsed
    // Value are safe; the packed form itself never changes); the mutating
    // accessors convert the array to Values in place.
    static Value PackedInts(std::vector<int64_t> v) {
        Value a;
        a._type = ARRAY;
        a._ints = std::move(v);
        return a;
    }
    const std::vector<int64_t>* packed_ints() const { return _ints.empty() ? nullptr : &_ints; }
    const std::vector<Value>& array() const {
        if (_ints.empty()) return _arr;
        return packed_view();
    }
    std::vector<Value>& mutable_array() {
        materialize();
        _type = ARRAY;
        return _arr;
    }
    Value& push_back(Value v) {
        materialize();
        _type = ARRAY;
        _arr.push_back(std::move(v));
        return _arr.back();
    }
    size_t size() const { return _type == ARRAY ? (_ints.empty() ? _arr.size() : _ints.size()) : _obj.size(); }

    // objects (insertion ordered)
    const std::vector<std::pair<std::string, Value>>& members() const { return _obj; }
    const Value* find(const std::string& key) const;
    Value* find(const std::string& key);
    Value& set(const std::string& key, Value v);
    Value& operator[](const std::string& key);

    std::string ToString(bool pretty = false) const;

private:
    void write(std::string* out, bool pretty, int indent) const;
    void materialize() {
        if (_ints.empty()) return;
        _arr.reserve(_ints.size());
        for (int64_t x : _ints) _arr.emplace_back(x);
        _ints.clear();
        _view.reset();
    }
    const std::vector<Value>& packed_view() const;
    Type _type;
    bool _b = false;
    int64_t _i = 0;
    uint64_t _u = 0;
    double _d = 0;
    std::string _s;
    std::vector<Value> _arr;
    std::vector<int64_t> _ints;
    // Values of a packed array for const readers (std::atomic_load/store)
    mutable std::shared_ptr<const std::vector<Value>> _view;
    std::vector<std::pair<std::string, Value>> _obj;
};

// Bulk parse of a large integer array (gpu/json_offload.cc): the
// reader, when it has a structural index, hands an array whose index shows
// only ',' between its brackets (no strings, objects or nested arrays) and
// at least min_elems elements to `fn` with the text base and the n + 1
// separator offsets; fn returns false unless every element is an int64,
// and the reader then parses the array itself.
typedef bool (*IntArrayOffload)(const char* base, const uint32_t* seps, size_t nseps, std::vector<int64_t>* out);
void SetIntArrayOffload(IntArrayOffload fn, size_t min_elems);

// Returns false and sets *error on malformed input.
bool Parse(const std::string& text, Value* out, std::string* error = nullptr);
bool Parse(const char* data, size_t n, Value* out, std::string* error = nullptr);
// Same result as Parse, with a structural index of `data` (ascending
// offsets of every unescaped quote and every {}[]:, outside strings, as
// gpu::LaunchJsonIndex produces): strings are cut at indexed quotes instead
// of scanned. A wrong index only costs speed, never correctness.
bool ParseWithIndex(const char* data, size_t n, const uint32_t* index, size_t nindex, Value* out,
                    std::string* error = nullptr);
void EscapeString(const std::string& s, std::string* out);
// Shortest round-tripping form of d in the reference rapidjson layout ("2.0", "0.1", "1e22").
void AppendShortestDouble(double d, std::string* out);

}  // namespace json
}  // namespace mrpc
