#include "json/json.h"

#include <charconv>

#include <atomic>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace mrpc {
namespace json {

const std::vector<Value>& Value::packed_view() const {
    std::shared_ptr<const std::vector<Value>> v = std::atomic_load(&_view);
    if (v) return *v;
    auto built = std::make_shared<std::vector<Value>>();
    built->reserve(_ints.size());
    for (int64_t x : _ints) built->emplace_back(x);
    std::shared_ptr<const std::vector<Value>> want = built;
    // first publisher wins; a loser's copy is dropped, every reader gets the
    // published one
    std::shared_ptr<const std::vector<Value>> expected;
    if (std::atomic_compare_exchange_strong(&_view, &expected, want)) return *want;
    return *expected;
}


int64_t Value::as_int() const {
    switch (_type) {
    case INT: return _i;
    case UINT: return (int64_t)_u;
    case DOUBLE: return (int64_t)_d;
    case BOOL: return _b;
    case STRING: return strtoll(_s.c_str(), nullptr, 10);
    default: return 0;
    }
}

uint64_t Value::as_uint() const {
    switch (_type) {
    case INT: return (uint64_t)_i;
    case UINT: return _u;
    case DOUBLE: return (uint64_t)_d;
    case BOOL: return _b;
    case STRING: return strtoull(_s.c_str(), nullptr, 10);
    default: return 0;
    }
}

double Value::as_double() const {
    switch (_type) {
    case INT: return (double)_i;
    case UINT: return (double)_u;
    case DOUBLE: return _d;
    case BOOL: return _b;
    case STRING: return strtod(_s.c_str(), nullptr);
    default: return 0;
    }
}

const Value* Value::find(const std::string& key) const {
    if (_type != OBJECT) return nullptr;
    for (auto& kv : _obj) {
        if (kv.first == key) return &kv.second;
    }
    return nullptr;
}

Value* Value::find(const std::string& key) {
    if (_type != OBJECT) return nullptr;
    for (auto& kv : _obj) {
        if (kv.first == key) return &kv.second;
    }
    return nullptr;
}

Value& Value::set(const std::string& key, Value v) {
    _type = OBJECT;
    Value* e = find(key);
    if (e) {
        *e = std::move(v);
        return *e;
    }
    _obj.emplace_back(key, std::move(v));
    return _obj.back().second;
}

Value& Value::operator[](const std::string& key) {
    _type = OBJECT;
    Value* e = find(key);
    if (e) return *e;
    _obj.emplace_back(key, Value());
    return _obj.back().second;
}

namespace {
// Bytes that need no escape are copied in runs: a word at a time while no
// byte of it is a control character, '"' or '\\' (per-byte push_back was
// 43% of an http echo of a 32 KiB string field).
inline bool word_is_plain(uint64_t w) {
    const uint64_t ones = 0x0101010101010101ull, highs = 0x8080808080808080ull;
    const uint64_t lt20 = (w - ones * 0x20) & ~w & highs;  // a byte < 0x20 (bytes >= 0x80 are plain)
    const uint64_t q = w ^ (ones * '"'), b = w ^ (ones * '\\');
    const uint64_t zq = (q - ones) & ~q & highs, zb = (b - ones) & ~b & highs;
    return (lt20 | zq | zb) == 0;
}
inline bool byte_is_plain(unsigned char c) { return c >= 0x20 && c != '"' && c != '\\'; }
}  // namespace

void EscapeString(const std::string& s, std::string* out) {
    out->reserve(out->size() + s.size() + 2);
    out->push_back('"');
    const char* p = s.data();
    const char* const end = p + s.size();
    while (p < end) {
        const char* run = p;
        while (end - p >= 8) {
            uint64_t w;
            memcpy(&w, p, 8);
            if (!word_is_plain(w)) break;
            p += 8;
        }
        while (p < end && byte_is_plain((unsigned char)*p)) ++p;
        out->append(run, (size_t)(p - run));
        if (p >= end) break;
        const unsigned char c = (unsigned char)*p++;
        switch (c) {
        case '"': *out += "\\\""; break;
        case '\\': *out += "\\\\"; break;
        case '\n': *out += "\\n"; break;
        case '\r': *out += "\\r"; break;
        case '\t': *out += "\\t"; break;
        case '\b': *out += "\\b"; break;
        case '\f': *out += "\\f"; break;
        default: {
            char b[8];
            snprintf(b, sizeof(b), "\\u%04x", c);
            *out += b;
        }
        }
    }
    out->push_back('"');
}

// Shortest round-tripping decimal form of a double, laid out the way the
// reference's rapidjson Writer does (Grisu digits + Prettify): integral
// values keep a ".0" ("2.0"), plain decimals up to 21 integer digits,
// "0.000ddd" down to 1e-6, exponent form otherwise ("1e22", "1.5e-7").
// Matches the expected strings of test/brpc_protobuf_json_unittest.cpp.
void AppendShortestDouble(double d, std::string* out) {
    if (d == 0) {
        *out += std::signbit(d) ? "-0.0" : "0.0";
        return;
    }
    char buf[40];
    int prec = 1;
    for (; prec <= 17; ++prec) {
        snprintf(buf, sizeof(buf), "%.*e", prec - 1, d);
        if (strtod(buf, nullptr) == d) break;
    }
    // buf: [-]d[.ddd]e(+|-)XX
    const char* p = buf;
    if (*p == '-') {
        out->push_back('-');
        ++p;
    }
    std::string digits;
    for (; *p && *p != 'e'; ++p)
        if (*p != '.') digits.push_back(*p);
    const int e10 = atoi(p + 1);
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    const int length = (int)digits.size();
    const int kk = e10 + 1;      // position of the decimal point
    const int k = kk - length;   // zeros after the digits
    if (k >= 0 && kk <= 21) {
        *out += digits;
        out->append((size_t)k, '0');
        *out += ".0";
    } else if (kk > 0 && kk <= 21) {
        out->append(digits, 0, (size_t)kk);
        out->push_back('.');
        out->append(digits, (size_t)kk, std::string::npos);
    } else if (kk > -6 && kk <= 0) {
        *out += "0.";
        out->append((size_t)(-kk), '0');
        *out += digits;
    } else {
        out->push_back(digits[0]);
        if (length > 1) {
            out->push_back('.');
            out->append(digits, 1, std::string::npos);
        }
        out->push_back('e');
        *out += std::to_string(kk - 1);
    }
}

void Value::write(std::string* out, bool pretty, int indent) const {
    char buf[64];
    auto nl = [&](int ind) {
        if (!pretty) return;
        out->push_back('\n');
        out->append(ind * 2, ' ');
    };
    switch (_type) {
    case NUL: *out += "null"; break;
    case BOOL: *out += _b ? "true" : "false"; break;
    case INT: snprintf(buf, sizeof(buf), "%lld", (long long)_i); *out += buf; break;
    case UINT: snprintf(buf, sizeof(buf), "%llu", (unsigned long long)_u); *out += buf; break;
    case DOUBLE:
        if (std::isnan(_d) || std::isinf(_d)) {
            *out += std::isnan(_d) ? "\"NaN\"" : (_d > 0 ? "\"Infinity\"" : "\"-Infinity\"");
        } else {
            AppendShortestDouble(_d, out);
        }
        break;
    case STRING: EscapeString(_s, out); break;
    case RAW: *out += _s; break;
    case ARRAY:
        if (!_ints.empty()) {
            out->push_back('[');
            for (size_t i = 0; i < _ints.size(); ++i) {
                if (i) out->push_back(',');
                nl(indent + 1);
                snprintf(buf, sizeof(buf), "%lld", (long long)_ints[i]);
                *out += buf;
            }
            nl(indent);
            out->push_back(']');
            break;
        }
        out->push_back('[');
        for (size_t i = 0; i < _arr.size(); ++i) {
            if (i) out->push_back(',');
            nl(indent + 1);
            _arr[i].write(out, pretty, indent + 1);
        }
        if (!_arr.empty()) nl(indent);
        out->push_back(']');
        break;
    case OBJECT:
        out->push_back('{');
        for (size_t i = 0; i < _obj.size(); ++i) {
            if (i) out->push_back(',');
            nl(indent + 1);
            EscapeString(_obj[i].first, out);
            out->push_back(':');
            if (pretty) out->push_back(' ');
            _obj[i].second.write(out, pretty, indent + 1);
        }
        if (!_obj.empty()) nl(indent);
        out->push_back('}');
        break;
    }
}

std::string Value::ToString(bool pretty) const {
    std::string s;
    write(&s, pretty, 0);
    return s;
}

namespace {
std::atomic<IntArrayOffload> g_int_array_offload{nullptr};
std::atomic<size_t> g_int_array_min{(size_t)-1};
}  // namespace

void SetIntArrayOffload(IntArrayOffload fn, size_t min_elems) {
    g_int_array_min.store(fn ? (min_elems ? min_elems : 1) : (size_t)-1, std::memory_order_relaxed);
    g_int_array_offload.store(fn, std::memory_order_release);
}

namespace {
class Reader {
public:
    Reader(const char* p, size_t n) : _p(p), _end(p + n), _begin(p) {}
    // A structural index (offsets of unescaped quotes and of {}[]:, outside
    // strings, ascending — gpu/json_kernels.hip): strings end at the next
    // indexed quote instead of a byte scan. An index that disagrees with the
    // text is ignored from that point on.
    void set_index(const uint32_t* idx, size_t n) {
        _idx = idx;
        _nidx = n;
        _k = 0;
    }
    bool parse(Value* v, std::string* err) {
        skip();
        if (!value(v, 0)) {
            if (err) *err = "invalid json at offset " + std::to_string(_p - _begin) + ": " + _err;
            return false;
        }
        skip();
        if (_p != _end) {
            if (err) *err = "trailing characters at offset " + std::to_string(_p - _begin);
            return false;
        }
        return true;
    }

private:
    void skip() {
        while (_p < _end && (*_p == ' ' || *_p == '\t' || *_p == '\n' || *_p == '\r')) ++_p;
    }
    bool fail(const char* m) {
        _err = m;
        return false;
    }
    bool value(Value* v, int depth) {
        if (depth > 200) return fail("nesting too deep");
        if (_p >= _end) return fail("unexpected end");
        switch (*_p) {
        case '{': return object(v, depth);
        case '[': return array(v, depth);
        case '"': {
            std::string s;
            if (!string(&s)) return false;
            *v = Value(s);
            return true;
        }
        case 't':
            if (_end - _p >= 4 && memcmp(_p, "true", 4) == 0) {
                _p += 4;
                *v = Value(true);
                return true;
            }
            return fail("bad literal");
        case 'f':
            if (_end - _p >= 5 && memcmp(_p, "false", 5) == 0) {
                _p += 5;
                *v = Value(false);
                return true;
            }
            return fail("bad literal");
        case 'n':
            if (_end - _p >= 4 && memcmp(_p, "null", 4) == 0) {
                _p += 4;
                *v = Value();
                return true;
            }
            return fail("bad literal");
        default: return number(v);
        }
    }
    // Numbers are converted in place from the text (std::from_chars): no
    // std::string per number, no errno/strtoll round trip.
    bool number(Value* v) {
        const char* b = _p;
        if (_p < _end && *_p == '-') ++_p;
        if (_p >= _end || !isdigit((unsigned char)*_p)) return fail("bad number");
        bool is_float = false;
        while (_p < _end && (isdigit((unsigned char)*_p) || *_p == '.' || *_p == 'e' || *_p == 'E' ||
                             ((*_p == '+' || *_p == '-') && (_p[-1] == 'e' || _p[-1] == 'E')))) {
            if (*_p == '.' || *_p == 'e' || *_p == 'E') is_float = true;
            ++_p;
        }
        if (!is_float) {
            int64_t x;
            if (parse_int64(b, _p, &x) == _p) {
                *v = Value(x);
                return true;
            }
            if (*b != '-') {
                uint64_t x;
                auto r = std::from_chars(b, _p, x);
                if (r.ec == std::errc() && r.ptr == _p) {
                    if (x <= (uint64_t)INT64_MAX) *v = Value((int64_t)x);
                    else *v = Value(x);
                    return true;
                }
            }
        }
        double d = 0;
        auto r = std::from_chars(b, _p, d);
        if (r.ec == std::errc::result_out_of_range) {
            d = strtod(std::string(b, _p - b).c_str(), nullptr);  // +-inf / denormal edge, as before
        } else if (r.ec != std::errc() || r.ptr != _p) {
            return fail("bad number");
        }
        *v = Value(d);
        return true;
    }
    // A decimal int64 literal at [p, end): the end of its digits, or nullptr
    // (no digits, more than 19 digits, or out of int64 range: the caller
    // takes the general path). Up to 19 digits cannot overflow a uint64, so
    // the loop has no per-digit overflow check.
    static const char* parse_int64(const char* p, const char* end, int64_t* out) {
        const bool neg = p < end && *p == '-';
        if (neg) ++p;
        const char* b = p;
        const char* lim = end - p > 19 ? p + 19 : end;
        uint64_t v = 0;
        while (p < lim && (unsigned)(*p - '0') < 10u) v = v * 10 + (unsigned)(*p++ - '0');
        if (p == b || (p < end && (unsigned)(*p - '0') < 10u)) return nullptr;
        if (neg) {
            if (v > (uint64_t)INT64_MAX + 1) return nullptr;
            *out = (int64_t)(0 - v);
        } else {
            if (v > (uint64_t)INT64_MAX) return nullptr;
            *out = (int64_t)v;
        }
        return p;
    }
    // An integer element of an int array, converted in place: true with *x
    // when the next value is a plain int64 literal followed by ',' or ']'
    // (after spaces); false (nothing consumed) otherwise.
    bool int_element(int64_t* x) {
        const char* e = parse_int64(_p, _end, x);
        if (!e) return false;
        if (e < _end && (*e == '.' || *e == 'e' || *e == 'E')) return false;
        _p = e;
        return true;
    }
    static void put_utf8(std::string* s, uint32_t cp) {
        if (cp < 0x80) {
            s->push_back((char)cp);
        } else if (cp < 0x800) {
            s->push_back((char)(0xC0 | (cp >> 6)));
            s->push_back((char)(0x80 | (cp & 0x3F)));
        } else if (cp < 0x10000) {
            s->push_back((char)(0xE0 | (cp >> 12)));
            s->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            s->push_back((char)(0x80 | (cp & 0x3F)));
        } else {
            s->push_back((char)(0xF0 | (cp >> 18)));
            s->push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
            s->push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            s->push_back((char)(0x80 | (cp & 0x3F)));
        }
    }
    bool hex4(uint32_t* out) {
        if (_end - _p < 4) return fail("bad unicode escape");
        uint32_t v = 0;
        for (int i = 0; i < 4; ++i) {
            char c = _p[i];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else return fail("bad unicode escape");
        }
        _p += 4;
        *out = v;
        return true;
    }
    // Closing quote of the string opening at _p from the index, or nullptr.
    const char* indexed_close() {
        if (!_idx) return nullptr;
        const size_t at = (size_t)(_p - _begin);
        while (_k < _nidx && _idx[_k] < at) ++_k;
        if (_k + 1 >= _nidx || _idx[_k] != at || _idx[_k + 1] >= (size_t)(_end - _begin) ||
            _begin[_idx[_k + 1]] != '"') {
            _idx = nullptr;  // stale or foreign index: scan from here on
            return nullptr;
        }
        const char* close = _begin + _idx[_k + 1];
        _k += 2;
        return close;
    }
    bool string(std::string* s) {
        if (const char* close = indexed_close()) {
            const char* b = _p + 1;
            // only trusted when the range holds no quote or backslash: then
            // `close` is certainly this string's end
            if (!memchr(b, '\\', (size_t)(close - b)) && !memchr(b, '"', (size_t)(close - b))) {
                s->append(b, (size_t)(close - b));
                _p = close + 1;
                return true;
            }
        }
        ++_p;  // opening quote
        for (;;) {  // runs without escapes or quotes go in one append
            const char* q = _p;
            // the closing quote, then any backslash before it (both memchr)
            const char* quote = (const char*)memchr(q, '"', (size_t)(_end - q));
            if (!quote) quote = _end;
            const char* bs = (const char*)memchr(q, '\\', (size_t)(quote - q));
            q = bs ? bs : quote;
            s->append(_p, (size_t)(q - _p));
            _p = q;
            if (_p >= _end || *_p == '"') break;
            ++_p;  // backslash
            if (_p >= _end) return fail("bad escape");
            if (!escape(s)) return false;
        }
        if (_p >= _end) return fail("unterminated string");
        ++_p;
        return true;
    }
    bool escape(std::string* s) {
        char e = *_p++;
        switch (e) {
        case '"': s->push_back('"'); break;
        case '\\': s->push_back('\\'); break;
        case '/': s->push_back('/'); break;
        case 'b': s->push_back('\b'); break;
        case 'f': s->push_back('\f'); break;
        case 'n': s->push_back('\n'); break;
        case 'r': s->push_back('\r'); break;
        case 't': s->push_back('\t'); break;
        case 'u': {
            uint32_t cp;
            if (!hex4(&cp)) return false;
            if (cp >= 0xD800 && cp < 0xDC00 && _end - _p >= 6 && _p[0] == '\\' && _p[1] == 'u') {
                _p += 2;
                uint32_t lo;
                if (!hex4(&lo)) return false;
                cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            put_utf8(s, cp);
            break;
        }
        default: return fail("bad escape");
        }
        return true;
    }
    // The index shows an array of >= the offload's minimum plain elements
    // (only ',' between the brackets): one bulk parse instead of a Value
    // per element; false leaves the array to the element-wise path.
    bool bulk_int_array(Value* v) {
        IntArrayOffload fn = g_int_array_offload.load(std::memory_order_acquire);
        if (!fn || !_idx) return false;
        const size_t at = (size_t)(_p - _begin);
        while (_k < _nidx && _idx[_k] < at) ++_k;
        if (_k >= _nidx || _idx[_k] != at) return false;
        size_t j = _k + 1;
        const size_t len = (size_t)(_end - _begin);
        while (j < _nidx && _idx[j] < len && _begin[_idx[j]] == ',') ++j;
        if (j >= _nidx || _idx[j] >= len || _begin[_idx[j]] != ']') return false;
        if (j - _k < g_int_array_min.load(std::memory_order_relaxed)) return false;
        std::vector<int64_t> ints;
        if (!fn(_begin, _idx + _k, j - _k + 1, &ints) || ints.size() != j - _k) return false;
        *v = Value::PackedInts(std::move(ints));
        _p = _begin + _idx[j] + 1;
        _k = j + 1;
        return true;
    }
    bool array(Value* v, int depth) {
        if (bulk_int_array(v)) return true;
        ++_p;
        *v = Value::Array();
        skip();
        if (_p < _end && *_p == ']') {
            ++_p;
            return true;
        }
        // Integer arrays stay packed (one int64 per element, no Value per
        // element; json2pb takes them in bulk, the way rapidjson's in-situ
        // numbers feed the reference's json_to_pb.cpp). The first element
        // that is not a plain int64 turns the array into Values.
        std::vector<int64_t> ints;
        for (;;) {
            int64_t x;
            skip();
            if (!int_element(&x)) break;
            ints.push_back(x);
            skip();
            if (_p < _end && *_p == ',') {
                ++_p;
                continue;
            }
            if (_p < _end && *_p == ']') {
                ++_p;
                *v = Value::PackedInts(std::move(ints));
                return true;
            }
            return fail("expected , or ]");
        }
        for (int64_t x : ints) v->push_back(Value(x));
        for (;;) {
            Value e;
            skip();
            if (!value(&e, depth + 1)) return false;
            v->push_back(std::move(e));
            skip();
            if (_p < _end && *_p == ',') {
                ++_p;
                continue;
            }
            if (_p < _end && *_p == ']') {
                ++_p;
                return true;
            }
            return fail("expected , or ]");
        }
    }
    bool object(Value* v, int depth) {
        ++_p;
        *v = Value::Object();
        skip();
        if (_p < _end && *_p == '}') {
            ++_p;
            return true;
        }
        for (;;) {
            skip();
            if (_p >= _end || *_p != '"') return fail("expected key");
            std::string key;
            if (!string(&key)) return false;
            skip();
            if (_p >= _end || *_p != ':') return fail("expected :");
            ++_p;
            skip();
            Value e;
            if (!value(&e, depth + 1)) return false;
            v->set(key, std::move(e));
            skip();
            if (_p < _end && *_p == ',') {
                ++_p;
                continue;
            }
            if (_p < _end && *_p == '}') {
                ++_p;
                return true;
            }
            return fail("expected , or }");
        }
    }
    const char* _p;
    const char* _end;
    const char* _begin;
    std::string _err;
    const uint32_t* _idx = nullptr;
    size_t _nidx = 0, _k = 0;
};
}  // namespace

bool Parse(const char* data, size_t n, Value* out, std::string* error) {
    Reader r(data, n);
    return r.parse(out, error);
}

bool ParseWithIndex(const char* data, size_t n, const uint32_t* index, size_t nindex, Value* out,
                    std::string* error) {
    Reader r(data, n);
    r.set_index(index, nindex);
    return r.parse(out, error);
}

bool Parse(const std::string& text, Value* out, std::string* error) { return Parse(text.data(), text.size(), out, error); }

}  // namespace json
}  // namespace mrpc
