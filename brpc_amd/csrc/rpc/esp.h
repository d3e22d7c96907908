// ESP client messages (role of the reference's src/brpc/esp_head.h,
// esp_message.h): a packed 32-byte little-endian head followed by
// body_len bytes. ESP has no magic number and no correlation id; the client
// maps responses to calls through the socket's pipelined-info queue.
#pragma once

#include <cstdint>
#include <cstring>

#include "base/buf.h"
#include "pb/message.h"

namespace mrpc {

#pragma pack(push, 1)
union EspAddress {
    uint64_t addr;
    struct {
        uint16_t stub;
        uint16_t port;
        uint32_t ip;
    };
};

struct EspHead {
    EspAddress from;
    EspAddress to;
    uint32_t msg;
    uint64_t msg_id;
    int32_t body_len;
};
#pragma pack(pop)
static_assert(sizeof(EspHead) == 32, "EspHead must be 32 bytes");

class EspMessage : public pb::Message {
public:
    EspMessage() { Clear(); }
    EspHead head;
    Buf body;
    const pb::Descriptor* GetDescriptor() const override { return OpaqueDescriptor("mrpc.EspMessage"); }
    pb::Message* New() const override { return new EspMessage; }
    void Clear() override {
        memset(&head, 0, sizeof(head));
        body.clear();
    }
    size_t ByteSizeLong() const override { return sizeof(EspHead) + body.size(); }
};

}  // namespace mrpc
