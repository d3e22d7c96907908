// Memcache binary-protocol client (role of the reference's
// src/brpc/memcache.h and policy/memcache_binary_protocol.cpp). A request
// batches operations; the channel pipelines them on one connection and the
// response pops results in the same order.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "base/buf.h"
#include "pb/message.h"

namespace mrpc {

enum MemcacheStatus {
    MC_STATUS_SUCCESS = 0x00,
    MC_STATUS_KEY_ENOENT = 0x01,
    MC_STATUS_KEY_EEXISTS = 0x02,
    MC_STATUS_E2BIG = 0x03,
    MC_STATUS_EINVAL = 0x04,
    MC_STATUS_NOT_STORED = 0x05,
    MC_STATUS_DELTA_BADVAL = 0x06,
    MC_STATUS_AUTH_ERROR = 0x20,
    MC_STATUS_UNKNOWN_COMMAND = 0x81,
    MC_STATUS_ENOMEM = 0x82,
};

class MemcacheRequest : public pb::Message {
public:
    bool Get(const std::string& key);
    bool Set(const std::string& key, const std::string& value, uint32_t flags, uint32_t exptime, uint64_t cas_value);
    bool Add(const std::string& key, const std::string& value, uint32_t flags, uint32_t exptime, uint64_t cas_value);
    bool Replace(const std::string& key, const std::string& value, uint32_t flags, uint32_t exptime,
                 uint64_t cas_value);
    bool Append(const std::string& key, const std::string& value, uint32_t flags, uint32_t exptime,
                uint64_t cas_value);
    bool Prepend(const std::string& key, const std::string& value, uint32_t flags, uint32_t exptime,
                 uint64_t cas_value);
    bool Delete(const std::string& key);
    bool Flush(uint32_t timeout);
    bool Increment(const std::string& key, uint64_t delta, uint64_t initial_value, uint32_t exptime);
    bool Decrement(const std::string& key, uint64_t delta, uint64_t initial_value, uint32_t exptime);
    bool Touch(const std::string& key, uint32_t exptime);
    bool Version();
    int op_count() const { return _nop; }
    void Clear() override;
    const pb::Descriptor* GetDescriptor() const override;
    pb::Message* New() const override { return new MemcacheRequest; }
    const Buf& raw() const { return _buf; }

private:
    bool store(uint8_t op, const std::string& key, const std::string& value, uint32_t flags, uint32_t exptime,
               uint64_t cas);
    bool counter(uint8_t op, const std::string& key, uint64_t delta, uint64_t initial, uint32_t exptime);
    Buf _buf;
    int _nop = 0;
};

class MemcacheResponse : public pb::Message {
public:
    struct Result {
        uint8_t opcode = 0;
        uint16_t status = 0;
        uint64_t cas = 0;
        uint32_t flags = 0;
        std::string key, value;
        uint64_t counter = 0;
    };
    // Pop the next result in request order; false with *err on failure.
    bool PopGet(std::string* value, uint32_t* flags, uint64_t* cas);
    bool PopSet(uint64_t* cas);
    bool PopAdd(uint64_t* cas);
    bool PopReplace(uint64_t* cas);
    bool PopAppend(uint64_t* cas);
    bool PopPrepend(uint64_t* cas);
    bool PopDelete();
    bool PopFlush();
    bool PopIncrement(uint64_t* new_value, uint64_t* cas);
    bool PopDecrement(uint64_t* new_value, uint64_t* cas);
    bool PopTouch();
    bool PopVersion(std::string* version);
    const std::string& LastError() const { return _err; }
    int result_count() const { return (int)(_results.size() - _next); }
    void Clear() override {
        _results.clear();
        _next = 0;
        _err.clear();
    }
    const pb::Descriptor* GetDescriptor() const override;
    pb::Message* New() const override { return new MemcacheResponse; }
    // protocol: parse up to `count` responses; 1 done, 0 more, -1 bad
    int ConsumePartial(Buf* in, int count);

private:
    bool pop(uint8_t op, Result* r);
    std::vector<Result> _results;
    size_t _next = 0;
    std::string _err;
};

}  // namespace mrpc
