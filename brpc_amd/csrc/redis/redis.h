// Redis (RESP2) client and server (role of the reference's src/brpc/redis.h,
// redis_reply.h, redis_command.h, policy/redis_protocol.cpp).
//
// Client: RedisRequest holds any number of commands; Channel (protocol
// "redis") pipelines them on one connection and RedisResponse receives one
// reply per command, in order. Server: a RedisService maps command names
// to RedisCommandHandler objects; commands of a connection are executed in
// arrival order inside the connection's reader fiber so replies keep RESP
// ordering.
#pragma once

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "base/buf.h"
#include "pb/message.h"

namespace mrpc {

enum RedisReplyType {
    REDIS_REPLY_STRING = 1,   // bulk string
    REDIS_REPLY_ARRAY = 2,
    REDIS_REPLY_INTEGER = 3,
    REDIS_REPLY_NIL = 4,
    REDIS_REPLY_STATUS = 5,   // simple string
    REDIS_REPLY_ERROR = 6,
};
const char* RedisReplyTypeToString(RedisReplyType t);

class RedisReply {
public:
    RedisReply() : _type(REDIS_REPLY_NIL), _integer(0) {}
    RedisReplyType type() const { return _type; }
    bool is_nil() const { return _type == REDIS_REPLY_NIL; }
    bool is_error() const { return _type == REDIS_REPLY_ERROR; }
    bool is_integer() const { return _type == REDIS_REPLY_INTEGER; }
    bool is_string() const { return _type == REDIS_REPLY_STRING || _type == REDIS_REPLY_STATUS; }
    bool is_array() const { return _type == REDIS_REPLY_ARRAY; }
    int64_t integer() const { return _integer; }
    const std::string& data() const { return _str; }  // string / status / error text
    const std::string& error_message() const { return _str; }
    size_t size() const { return _array.size(); }
    const RedisReply& operator[](size_t i) const { return _array[i]; }
    RedisReply& operator[](size_t i) { return _array[i]; }

    void SetNil() { reset(REDIS_REPLY_NIL); }
    void SetStatus(const std::string& s) { reset(REDIS_REPLY_STATUS); _str = s; }
    void SetError(const std::string& s) { reset(REDIS_REPLY_ERROR); _str = s; }
    void SetString(const std::string& s) { reset(REDIS_REPLY_STRING); _str = s; }
    void SetInteger(int64_t v) { reset(REDIS_REPLY_INTEGER); _integer = v; }
    void SetArray(size_t n) { reset(REDIS_REPLY_ARRAY); _array.resize(n); }

    // RESP serialization / incremental parsing. ConsumePartial returns
    // 1 (reply complete, bytes consumed), 0 (need more), -1 (malformed).
    void SerializeTo(Buf* out) const;
    int ConsumePartial(Buf* in);
    std::string ToString() const;  // human readable

private:
    void reset(RedisReplyType t) {
        _type = t;
        _integer = 0;
        _str.clear();
        _array.clear();
    }
    RedisReplyType _type;
    int64_t _integer;
    std::string _str;
    std::vector<RedisReply> _array;
};

// Non-protobuf payload classes still go through Channel::CallMethod, so
// they are pb::Messages with an opaque (field-less) descriptor.
class RedisRequest : public pb::Message {
public:
    RedisRequest() {}
    // printf-like: "SET %s %d"; %s arguments may contain spaces/binary.
    bool AddCommand(const char* fmt, ...);
    // Pre-split arguments.
    bool AddCommandByComponents(const std::vector<std::string>& args);
    int command_size() const { return _ncommand; }
    bool has_error() const { return _has_error; }
    void Clear() override;
    const pb::Descriptor* GetDescriptor() const override;
    pb::Message* New() const override { return new RedisRequest; }
    bool SerializeTo(Buf* out) const;
    std::string ToString() const;

private:
    Buf _buf;
    int _ncommand = 0;
    bool _has_error = false;
};

class RedisResponse : public pb::Message {
public:
    int reply_size() const { return (int)_replies.size(); }
    const RedisReply& reply(int i) const { return _replies[i]; }
    void Clear() override { _replies.clear(); }
    const pb::Descriptor* GetDescriptor() const override;
    pb::Message* New() const override { return new RedisResponse; }
    // Parse up to `count` replies; 1 when all arrived, 0 need more, -1 bad.
    int ConsumePartial(Buf* in, int count);

private:
    std::vector<RedisReply> _replies;
};

// Server side
class RedisCommandHandler {
public:
    enum Result { OK = 0, CONTINUE = 1, BATCHED = 2 };
    virtual ~RedisCommandHandler() {}
    // args[0] is the command name (lower-cased).
    virtual Result Run(const std::vector<std::string>& args, RedisReply* output, bool flush_batched) = 0;
    // MULTI support: return a handler that receives the queued commands.
    virtual RedisCommandHandler* NewTransactionHandler() { return nullptr; }
};

class RedisService {
public:
    virtual ~RedisService() {}
    bool AddCommandHandler(const std::string& name, RedisCommandHandler* handler);
    RedisCommandHandler* FindCommandHandler(const std::string& name) const;

private:
    std::map<std::string, RedisCommandHandler*> _handlers;
};

}  // namespace mrpc
