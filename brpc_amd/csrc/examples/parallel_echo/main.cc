// Parallel echo (reference example/parallel_echo_c++): one call fans out to
// -servers sub-channels concurrently (the data-parallel broadcast shape:
// one direct link per peer); a CallMapper tags each sub-request and a
// ResponseMerger concatenates the answers.
#include <memory>
#include <vector>

#include "examples/common.h"
#include "rpc/combo_channels.h"

DEFINE_int32(servers, 7, "sub channels (e.g. the 7 xGMI peers of a GPU)");

namespace {
class Mapper : public mrpc::CallMapper {
public:
    mrpc::SubCall Map(int i, int n, const mrpc::pb::MethodDescriptor* m, const mrpc::pb::Message* req,
                      mrpc::pb::Message* res) override {
        auto* r = new example::EchoRequest(*static_cast<const example::EchoRequest*>(req));
        r->set_message(r->message() + "/" + std::to_string(i));
        return mrpc::SubCall(m, r, res->New(), mrpc::SubCall::DELETE_REQUEST | mrpc::SubCall::DELETE_RESPONSE);
    }
};
class Merger : public mrpc::ResponseMerger {
public:
    Result Merge(mrpc::pb::Message* response, const mrpc::pb::Message* sub) override {
        auto* r = static_cast<example::EchoResponse*>(response);
        auto* s = static_cast<const example::EchoResponse*>(sub);
        r->set_message(r->message().empty() ? s->message() : r->message() + " " + s->message());
        return MERGED;
    }
};
}  // namespace

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    std::vector<std::unique_ptr<demo::LocalServer>> servers;
    mrpc::ParallelChannel pc;
    mrpc::ParallelChannelOptions po;
    po.timeout_ms = 2000;
    pc.Init(&po);
    auto mapper = std::make_shared<Mapper>();
    auto merger = std::make_shared<Merger>();
    for (int i = 0; i < FLAGS_servers; ++i) {
        servers.emplace_back(new demo::LocalServer("peer" + std::to_string(i)));
        auto* ch = new mrpc::Channel;
        mrpc::ChannelOptions o;
        o.timeout_ms = 2000;
        if (ch->Init(servers.back()->addr().c_str(), &o) != 0) return 1;
        pc.AddChannel(ch, mrpc::OWNS_CHANNEL, mapper, merger);
    }
    example::EchoService_Stub stub(&pc);
    mrpc::Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("fan");
    stub.Echo(&cntl, &req, &res, nullptr);
    printf("merged: %s\n", res.message().c_str());
    int parts = 1;
    for (char c : res.message()) parts += c == ' ';
    return demo::Check(!cntl.Failed() && parts == FLAGS_servers, "scatter/gather over sub channels");
}
