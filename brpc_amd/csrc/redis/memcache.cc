#include "redis/memcache.h"

#include <cstring>

#include "base/util.h"

namespace mrpc {

const pb::Descriptor* OpaqueDescriptor(const char* full_name);  // redis.cc

namespace {
enum : uint8_t {
    OP_GET = 0x00,
    OP_SET = 0x01,
    OP_ADD = 0x02,
    OP_REPLACE = 0x03,
    OP_DELETE = 0x04,
    OP_INCREMENT = 0x05,
    OP_DECREMENT = 0x06,
    OP_FLUSH = 0x08,
    OP_VERSION = 0x0b,
    OP_APPEND = 0x0e,
    OP_PREPEND = 0x0f,
    OP_TOUCH = 0x1c,
};

void put16(std::string* s, uint16_t v) {
    s->push_back((char)(v >> 8));
    s->push_back((char)v);
}
void put32(std::string* s, uint32_t v) {
    for (int i = 3; i >= 0; --i) s->push_back((char)(v >> (8 * i)));
}
void put64(std::string* s, uint64_t v) {
    for (int i = 7; i >= 0; --i) s->push_back((char)(v >> (8 * i)));
}
uint64_t get_be(const unsigned char* p, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 8) | p[i];
    return v;
}

void header(std::string* s, uint8_t op, size_t keylen, size_t extlen, size_t bodylen, uint64_t cas) {
    s->push_back((char)0x80);
    s->push_back((char)op);
    put16(s, (uint16_t)keylen);
    s->push_back((char)extlen);
    s->push_back(0);      // data type
    put16(s, 0);          // vbucket
    put32(s, (uint32_t)bodylen);
    put32(s, 0);          // opaque
    put64(s, cas);
}
}  // namespace

const pb::Descriptor* MemcacheRequest::GetDescriptor() const { return OpaqueDescriptor("mrpc.MemcacheRequest"); }
const pb::Descriptor* MemcacheResponse::GetDescriptor() const { return OpaqueDescriptor("mrpc.MemcacheResponse"); }

void MemcacheRequest::Clear() {
    _buf.clear();
    _nop = 0;
}

// memcached rejects keys above 250 bytes; the header's body length is 32-bit
static bool valid_op(const std::string& key, size_t value_size = 0) {
    return key.size() <= 250 && value_size <= 0xFFFFFFFFull - 300;
}

bool MemcacheRequest::Get(const std::string& key) {
    if (!valid_op(key)) return false;
    std::string s;
    header(&s, OP_GET, key.size(), 0, key.size(), 0);
    s += key;
    _buf.append(s);
    ++_nop;
    return true;
}

bool MemcacheRequest::store(uint8_t op, const std::string& key, const std::string& value, uint32_t flags,
                            uint32_t exptime, uint64_t cas) {
    if (!valid_op(key, value.size())) return false;
    const bool extras = op == OP_SET || op == OP_ADD || op == OP_REPLACE;
    std::string s;
    const size_t ext = extras ? 8 : 0;
    header(&s, op, key.size(), ext, ext + key.size() + value.size(), cas);
    if (extras) {
        put32(&s, flags);
        put32(&s, exptime);
    }
    s += key;
    s += value;
    _buf.append(s);
    ++_nop;
    return true;
}

bool MemcacheRequest::Set(const std::string& k, const std::string& v, uint32_t f, uint32_t e, uint64_t c) {
    return store(OP_SET, k, v, f, e, c);
}
bool MemcacheRequest::Add(const std::string& k, const std::string& v, uint32_t f, uint32_t e, uint64_t c) {
    return store(OP_ADD, k, v, f, e, c);
}
bool MemcacheRequest::Replace(const std::string& k, const std::string& v, uint32_t f, uint32_t e, uint64_t c) {
    return store(OP_REPLACE, k, v, f, e, c);
}
bool MemcacheRequest::Append(const std::string& k, const std::string& v, uint32_t f, uint32_t e, uint64_t c) {
    return store(OP_APPEND, k, v, f, e, c);
}
bool MemcacheRequest::Prepend(const std::string& k, const std::string& v, uint32_t f, uint32_t e, uint64_t c) {
    return store(OP_PREPEND, k, v, f, e, c);
}

bool MemcacheRequest::Delete(const std::string& key) {
    if (!valid_op(key)) return false;
    std::string s;
    header(&s, OP_DELETE, key.size(), 0, key.size(), 0);
    s += key;
    _buf.append(s);
    ++_nop;
    return true;
}

bool MemcacheRequest::Flush(uint32_t timeout) {
    std::string s;
    header(&s, OP_FLUSH, 0, 4, 4, 0);
    put32(&s, timeout);
    _buf.append(s);
    ++_nop;
    return true;
}

bool MemcacheRequest::counter(uint8_t op, const std::string& key, uint64_t delta, uint64_t initial, uint32_t exptime) {
    if (!valid_op(key)) return false;
    std::string s;
    header(&s, op, key.size(), 20, 20 + key.size(), 0);
    put64(&s, delta);
    put64(&s, initial);
    put32(&s, exptime);
    s += key;
    _buf.append(s);
    ++_nop;
    return true;
}

bool MemcacheRequest::Increment(const std::string& k, uint64_t d, uint64_t i, uint32_t e) {
    return counter(OP_INCREMENT, k, d, i, e);
}
bool MemcacheRequest::Decrement(const std::string& k, uint64_t d, uint64_t i, uint32_t e) {
    return counter(OP_DECREMENT, k, d, i, e);
}

bool MemcacheRequest::Touch(const std::string& key, uint32_t exptime) {
    if (!valid_op(key)) return false;
    std::string s;
    header(&s, OP_TOUCH, key.size(), 4, 4 + key.size(), 0);
    put32(&s, exptime);
    s += key;
    _buf.append(s);
    ++_nop;
    return true;
}

bool MemcacheRequest::Version() {
    std::string s;
    header(&s, OP_VERSION, 0, 0, 0, 0);
    _buf.append(s);
    ++_nop;
    return true;
}

// ------------------------------------------------------------------ response
int MemcacheResponse::ConsumePartial(Buf* in, int count) {
    while ((int)_results.size() < count) {
        unsigned char h[24];
        if (in->size() < 24) return 0;
        in->copy_to(h, 24);
        if (h[0] != 0x81) return -1;
        const uint16_t keylen = (uint16_t)get_be(h + 2, 2);
        const uint8_t extlen = h[4];
        const uint32_t body = (uint32_t)get_be(h + 8, 4);
        if (body < (uint32_t)keylen + extlen) return -1;
        if (in->size() < 24 + (size_t)body) return 0;
        Result r;
        r.opcode = h[1];
        r.status = (uint16_t)get_be(h + 6, 2);
        r.cas = get_be(h + 16, 8);
        in->pop_front(24);
        std::string ext, key, value;
        in->cutn(&ext, extlen);
        in->cutn(&key, keylen);
        in->cutn(&value, body - keylen - extlen);
        if (extlen >= 4) r.flags = (uint32_t)get_be((const unsigned char*)ext.data(), 4);
        r.key = key;
        if ((r.opcode == OP_INCREMENT || r.opcode == OP_DECREMENT) && r.status == 0 && value.size() == 8) {
            r.counter = get_be((const unsigned char*)value.data(), 8);
        }
        r.value = value;
        _results.push_back(std::move(r));
    }
    return 1;
}

bool MemcacheResponse::pop(uint8_t op, Result* r) {
    if (_next >= _results.size()) {
        _err = "no more results";
        return false;
    }
    *r = _results[_next++];
    if (r->opcode != op) {
        _err = "result opcode " + std::to_string(r->opcode) + " does not match the popped operation";
        return false;
    }
    if (r->status != MC_STATUS_SUCCESS) {
        _err = "status " + std::to_string(r->status) + ": " + r->value;
        return false;
    }
    return true;
}

bool MemcacheResponse::PopGet(std::string* value, uint32_t* flags, uint64_t* cas) {
    Result r;
    if (!pop(OP_GET, &r)) return false;
    if (value) *value = r.value;
    if (flags) *flags = r.flags;
    if (cas) *cas = r.cas;
    return true;
}

#define MC_POP_CAS(NAME, OP)                 \
    bool MemcacheResponse::NAME(uint64_t* cas) { \
        Result r;                            \
        if (!pop(OP, &r)) return false;      \
        if (cas) *cas = r.cas;               \
        return true;                         \
    }
MC_POP_CAS(PopSet, OP_SET)
MC_POP_CAS(PopAdd, OP_ADD)
MC_POP_CAS(PopReplace, OP_REPLACE)
MC_POP_CAS(PopAppend, OP_APPEND)
MC_POP_CAS(PopPrepend, OP_PREPEND)
#undef MC_POP_CAS

bool MemcacheResponse::PopDelete() {
    Result r;
    return pop(OP_DELETE, &r);
}
bool MemcacheResponse::PopFlush() {
    Result r;
    return pop(OP_FLUSH, &r);
}
bool MemcacheResponse::PopTouch() {
    Result r;
    return pop(OP_TOUCH, &r);
}

bool MemcacheResponse::PopIncrement(uint64_t* v, uint64_t* cas) {
    Result r;
    if (!pop(OP_INCREMENT, &r)) return false;
    if (v) *v = r.counter;
    if (cas) *cas = r.cas;
    return true;
}

bool MemcacheResponse::PopDecrement(uint64_t* v, uint64_t* cas) {
    Result r;
    if (!pop(OP_DECREMENT, &r)) return false;
    if (v) *v = r.counter;
    if (cas) *cas = r.cas;
    return true;
}

bool MemcacheResponse::PopVersion(std::string* version) {
    Result r;
    if (!pop(OP_VERSION, &r)) return false;
    if (version) *version = r.value;
    return true;
}

}  // namespace mrpc
