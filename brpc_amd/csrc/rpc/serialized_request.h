// A request whose body is already serialized (and possibly compressed):
// sent as-is by pb protocols instead of being re-encoded. Used for
// proxying and by rpc_replay to resend dumped requests byte-for-byte
// (role of the reference's src/brpc/serialized_request.h).
#pragma once

#include "base/buf.h"
#include "pb/message.h"

namespace mrpc {

class SerializedRequest : public pb::Message {
public:
    const pb::Descriptor* GetDescriptor() const override { return OpaqueDescriptor("mrpc.SerializedRequest"); }
    pb::Message* New() const override { return new SerializedRequest; }
    void Clear() override { _data.clear(); }
    size_t ByteSizeLong() const override { return _data.size(); }
    const Buf& serialized_data() const { return _data; }
    Buf& serialized_data() { return _data; }

private:
    Buf _data;
};

}  // namespace mrpc
