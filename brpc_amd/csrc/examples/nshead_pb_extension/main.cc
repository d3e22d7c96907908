// nshead + protobuf extension (reference example/nshead_pb_extension_c++):
// a legacy nshead wire format carrying a protobuf body is mapped onto an
// ordinary protobuf service by an NsheadPbServiceAdaptor — the adaptor
// names the method, parses the request and encodes the response (and
// errors) the legacy way, and the pb service stays unaware of nshead.
// Here the legacy format is: nshead.reserved = method index (0 = Echo),
// body = serialized EchoRequest; responses set nshead.reserved to the
// error code and carry the EchoResponse or the error text.
#include <memory>

#include "examples/common.h"
#include "mrpc/proto/legacy_meta.pb.h"
#include "rpc/nshead.h"

namespace {

class LegacyEchoAdaptor : public mrpc::NsheadPbServiceAdaptor {
public:
    void ParseNsheadMeta(const mrpc::Server&, const mrpc::NsheadMessage& req, mrpc::Controller* cntl,
                         mrpc::policy::NsheadMeta* meta) const override {
        if (req.head.reserved != 0) {
            cntl->SetFailed(mrpc::ENOMETHOD, "no method #%u", req.head.reserved);
            return;
        }
        meta->set_full_method_name("example.EchoService.Echo");
        meta->set_log_id(req.head.log_id);
    }
    void ParseRequestFromBuf(const mrpc::policy::NsheadMeta&, const mrpc::NsheadMessage& raw, mrpc::Controller* cntl,
                             mrpc::pb::Message* pb_req) const override {
        if (!pb_req->ParseFromBuf(raw.body)) cntl->SetFailed(mrpc::EREQUEST, "bad EchoRequest body");
    }
    void SerializeResponseToBuf(const mrpc::policy::NsheadMeta&, mrpc::Controller* cntl,
                                const mrpc::pb::Message* pb_res, mrpc::NsheadMessage* raw) const override {
        if (cntl->Failed()) {
            raw->head.reserved = (uint32_t)cntl->ErrorCode();
            raw->body.append(cntl->ErrorText());
            return;
        }
        raw->head.reserved = 0;
        pb_res->SerializeToBuf(&raw->body);
    }
};

bool Call(mrpc::Channel& ch, uint32_t method, const std::string& msg, example::EchoResponse* res, uint32_t* code) {
    mrpc::NsheadMessage req, raw_res;
    req.head.reserved = method;
    req.head.log_id = 42;
    example::EchoRequest pb;
    pb.set_message(msg);
    pb.SerializeToBuf(&req.body);
    mrpc::Controller cntl;
    ch.CallMethod(nullptr, &cntl, &req, &raw_res, nullptr);
    if (cntl.Failed()) return false;
    *code = raw_res.head.reserved;
    return *code != 0 || res->ParseFromBuf(raw_res.body);
}

}  // namespace

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    demo::TaggedEcho echo("pb");
    LegacyEchoAdaptor adaptor;
    mrpc::Server server;
    server.AddService(&echo, mrpc::SERVER_DOESNT_OWN_SERVICE);
    mrpc::ServerOptions so;
    so.nshead_service = &adaptor;
    if (server.Start("127.0.0.1:0", &so) != 0) return 1;
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.protocol = "nshead";
    opt.timeout_ms = 2000;
    if (ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &opt) != 0) return 1;
    bool ok = true;
    for (int i = 0; i < 10 && ok; ++i) {
        example::EchoResponse res;
        uint32_t code = 1;
        ok = Call(ch, 0, "legacy " + std::to_string(i), &res, &code) && code == 0 &&
             res.message() == "legacy " + std::to_string(i) + "@pb";
    }
    example::EchoResponse res;
    uint32_t code = 0;
    const bool routed_error = Call(ch, 9, "x", &res, &code) && code == (uint32_t)mrpc::ENOMETHOD;
    printf("10 nshead+pb echoes through the adaptor; unknown method -> error code %u\n", code);
    server.Stop(0);
    server.Join();
    return demo::Check(ok && routed_error, "nshead_pb adaptor");
}
