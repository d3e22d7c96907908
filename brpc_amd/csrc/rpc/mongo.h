// Server-side mongo adaptor (role of the reference's
// src/brpc/mongo_service_adaptor.h): a server whose
// ServerOptions.mongo_service_adaptor is set speaks the mongo wire protocol;
// every message is dispatched to the registered
// mrpc.policy.MongoService.default_method (see proto/mongo.proto).
#pragma once

#include <memory>

#include "base/buf.h"

namespace mrpc {

// Per-connection state created on the first mongo message of a socket and
// destroyed with it; reachable from handlers via
// Controller::mongo_session_data().
class MongoContext {
public:
    virtual ~MongoContext() {}
};

class MongoServiceAdaptor {
public:
    virtual ~MongoServiceAdaptor() {}
    // A failed call must still answer the client: write an error reply to
    // request `response_to` into out.
    virtual void SerializeError(int response_to, Buf* out) const = 0;
    virtual MongoContext* CreateSocketContext() const = 0;
};

#pragma pack(push, 1)
struct mongo_head_t {
    int32_t message_length;  // including this head
    int32_t request_id;
    int32_t response_to;
    int32_t op_code;
};
#pragma pack(pop)
static_assert(sizeof(mongo_head_t) == 16, "mongo head is 16 bytes");

}  // namespace mrpc
