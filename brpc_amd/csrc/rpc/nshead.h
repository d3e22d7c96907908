// nshead: the 36-byte little-endian head of Baidu's legacy protocols, the
// raw NsheadMessage, the NsheadService a server hands nshead requests to,
// and the adaptors that map nshead requests onto protobuf services:
//   NsheadPbServiceAdaptor  generic (subclass decides meta / body codec)
//   NovaServiceAdaptor      nova_pbrpc: head.reserved = method index, snappy flag in head.version
//   PublicPbrpcServiceAdaptor  public_pbrpc: body is PublicPbrpcRequest
//   NsheadMcpackAdaptor     nshead_mcpack: body is the mcpack of the request
// (roles of the reference's src/brpc/nshead.h, nshead_message.h,
// nshead_service.h, nshead_pb_service_adaptor.h and the NovaServiceAdaptor /
// PublicPbrpcServiceAdaptor / NsheadMcpackAdaptor in src/brpc/policy/).
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "base/buf.h"
#include "pb/message.h"
#include "pb/service.h"
#include "rpc/ordered_response.h"

namespace mrpc {

class Server;
class Controller;
class MethodStatus;
namespace policy {
class NsheadMeta;
}

static const uint32_t NSHEAD_MAGICNUM = 0xfb709394;

#pragma pack(push, 1)
struct nshead_t {
    uint16_t id;
    uint16_t version;
    uint32_t log_id;
    char provider[16];
    uint32_t magic_num;
    uint32_t reserved;
    uint32_t body_len;
};
#pragma pack(pop)
static_assert(sizeof(nshead_t) == 36, "nshead_t must be 36 bytes");

// Raw nshead request/response: usable as the request/response of a
// Channel whose protocol is "nshead", and what NsheadService sees.
class NsheadMessage : public pb::Message {
public:
    NsheadMessage() { Clear(); }
    nshead_t head;
    Buf body;
    const pb::Descriptor* GetDescriptor() const override;
    pb::Message* New() const override { return new NsheadMessage; }
    void Clear() override {
        memset(&head, 0, sizeof(head));
        body.clear();
    }
    size_t ByteSizeLong() const override { return sizeof(nshead_t) + body.size(); }
};

// Completion of one nshead request: Run() writes response.head+body back
// (the response head defaults to the request head with magic/body_len
// fixed up) unless the controller asked to close the connection.
class NsheadClosure : public Closure {
public:
    Controller* controller() { return _cntl.get(); }
    const NsheadMessage& request() const { return _request; }
    NsheadMessage* response() { return &_response; }
    int64_t received_us() const { return _received_us; }
    // Skip writing a response (one-way requests).
    void DoNotRespond() { _do_respond = false; }
    void Run() override;

    // ---- internal (set by the nshead protocol)
    NsheadClosure();
    ~NsheadClosure() override;
    std::unique_ptr<Controller> _cntl;
    NsheadMessage _request;
    NsheadMessage _response;
    Server* _server = nullptr;
    int64_t _received_us = 0;
    bool _do_respond = true;
    bool _added_concurrency = false;
    // nshead carries no correlation id: responses of one connection must
    // leave in request order even when handlers finish out of order.
    uint64_t _seq = 0;
    std::shared_ptr<OrderedResponseWriter> _sequencer;
};



class NsheadService {
public:
    NsheadService();
    virtual ~NsheadService();
    // Called for every nshead request. `done->Run()` sends the response.
    virtual void ProcessNsheadRequest(const Server& server, Controller* cntl, const NsheadMessage& request,
                                      NsheadMessage* response, NsheadClosure* done) = 0;
    MethodStatus* status() const { return _status.get(); }
    void Expose(const std::string& prefix);

private:
    std::unique_ptr<MethodStatus> _status;
};

class NsheadPbServiceAdaptor : public NsheadService {
public:
    // Extract full_method_name etc. from the raw request (fail cntl on error).
    virtual void ParseNsheadMeta(const Server& server, const NsheadMessage& request, Controller* cntl,
                                 policy::NsheadMeta* out_meta) const = 0;
    virtual void ParseRequestFromBuf(const policy::NsheadMeta& meta, const NsheadMessage& raw_req, Controller* cntl,
                                     pb::Message* pb_req) const = 0;
    // Also called when cntl->Failed(): encode the error in the protocol's way.
    virtual void SerializeResponseToBuf(const policy::NsheadMeta& meta, Controller* cntl, const pb::Message* pb_res,
                                        NsheadMessage* raw_res) const = 0;
    void ProcessNsheadRequest(const Server& server, Controller* cntl, const NsheadMessage& request,
                              NsheadMessage* response, NsheadClosure* done) final;
};

class NovaServiceAdaptor : public NsheadPbServiceAdaptor {
public:
    void ParseNsheadMeta(const Server& server, const NsheadMessage& request, Controller* cntl,
                         policy::NsheadMeta* out_meta) const override;
    void ParseRequestFromBuf(const policy::NsheadMeta& meta, const NsheadMessage& raw_req, Controller* cntl,
                             pb::Message* pb_req) const override;
    void SerializeResponseToBuf(const policy::NsheadMeta& meta, Controller* cntl, const pb::Message* pb_res,
                                NsheadMessage* raw_res) const override;
};

class PublicPbrpcServiceAdaptor : public NsheadPbServiceAdaptor {
public:
    void ParseNsheadMeta(const Server& server, const NsheadMessage& request, Controller* cntl,
                         policy::NsheadMeta* out_meta) const override;
    void ParseRequestFromBuf(const policy::NsheadMeta& meta, const NsheadMessage& raw_req, Controller* cntl,
                             pb::Message* pb_req) const override;
    void SerializeResponseToBuf(const policy::NsheadMeta& meta, Controller* cntl, const pb::Message* pb_res,
                                NsheadMessage* raw_res) const override;
};

// nshead_mcpack: the single service method is chosen by `full_method_name`
// given at construction (or the first method of the first service).
class NsheadMcpackAdaptor : public NsheadPbServiceAdaptor {
public:
    explicit NsheadMcpackAdaptor(const std::string& full_method_name = std::string()) : _method(full_method_name) {}
    void ParseNsheadMeta(const Server& server, const NsheadMessage& request, Controller* cntl,
                         policy::NsheadMeta* out_meta) const override;
    void ParseRequestFromBuf(const policy::NsheadMeta& meta, const NsheadMessage& raw_req, Controller* cntl,
                             pb::Message* pb_req) const override;
    void SerializeResponseToBuf(const policy::NsheadMeta& meta, Controller* cntl, const pb::Message* pb_res,
                                NsheadMessage* raw_res) const override;

private:
    std::string _method;
};

// Packs head+body (magic/body_len filled in).
void PackNsheadFrame(Buf* out, const nshead_t& head, const Buf& body);
static const uint16_t NOVA_SNAPPY_COMPRESS_FLAG = 0x1;

}  // namespace mrpc
