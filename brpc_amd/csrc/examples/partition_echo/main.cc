// Partition echo (reference example/partition_echo_c++): servers announce
// "index/count" tags in the naming service; a PartitionChannel sends one
// sub-call per partition (shard), each partition load-balanced on its own.
#include <memory>
#include <vector>

#include "examples/common.h"
#include "rpc/combo_channels.h"

namespace {
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
    // 3 partitions; partition 1 has two replicas
    demo::LocalServer p0("p0"), p1a("p1a"), p1b("p1b"), p2("p2");
    const std::string url = "list://" + p0.addr() + " 0/3," + p1a.addr() + " 1/3," + p1b.addr() + " 1/3," +
                            p2.addr() + " 2/3";
    mrpc::PartitionParser parser;
    mrpc::PartitionChannelOptions opt;
    opt.timeout_ms = 2000;
    opt.response_merger = std::make_shared<Merger>();
    mrpc::PartitionChannel pch;
    if (pch.Init(3, &parser, url.c_str(), "rr", &opt) != 0) return 1;
    example::EchoService_Stub stub(&pch);
    bool ok = true;
    for (int i = 0; i < 4; ++i) {
        mrpc::Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("shard");
        stub.Echo(&cntl, &req, &res, nullptr);
        printf("call %d: %s\n", i, res.message().c_str());
        ok = ok && !cntl.Failed() && res.message().find("@p0") != std::string::npos &&
             res.message().find("@p2") != std::string::npos && res.message().find("@p1") != std::string::npos;
    }
    return demo::Check(ok, "one sub-call per partition");
}
