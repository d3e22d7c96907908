// DynamicMessage: messages whose layout is computed at runtime from a
// descriptor (role of google::protobuf::DynamicMessageFactory used by the
// reference's rpc_press/rpc_replay to load .proto files without codegen).
#pragma once

#include "pb/descriptor.h"
#include "pb/message.h"

namespace mrpc {
namespace pb {

class DynamicMessage : public Message {
public:
    static DynamicMessage* Create(const Descriptor* d);
    ~DynamicMessage() override;
    const Descriptor* GetDescriptor() const override { return _desc; }
    Message* New() const override { return Create(_desc); }
    static void operator delete(void* p) { ::free(p); }

private:
    explicit DynamicMessage(const Descriptor* d) : _desc(d) {}
    const Descriptor* _desc;
};

// Computes offsets/has-bits/object_size for a descriptor tree to be used by
// DynamicMessage (no-op for descriptors with a generated factory), and
// installs dynamic prototypes. Must be called after type resolution.
void PrepareDynamicLayout(Descriptor* d);

// Parses proto2 default value text into the typed default fields.
void ResolveDefaultValue(FieldDescriptor* f);

}  // namespace pb
}  // namespace mrpc
