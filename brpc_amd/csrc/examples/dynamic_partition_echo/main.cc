// Dynamic partition echo (reference example/dynamic_partition_echo_c++):
// the naming service lists servers of two partitioning schemes at once —
// 3 partitions ("i/3" tags) and 4 partitions ("i/4") — as happens while a
// sharded service is being re-partitioned. A DynamicPartitionChannel groups
// them by scheme, sends each call to ONE complete scheme (one sub-call per
// partition of it) and follows the server list file as the migration
// finishes and the 3-way scheme disappears.
#include <cstdio>
#include <fstream>
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

int count_of(const std::string& s, const std::string& what) {
    int n = 0;
    for (size_t p = s.find(what); p != std::string::npos; p = s.find(what, p + 1)) ++n;
    return n;
}
}  // namespace

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    std::vector<std::unique_ptr<demo::LocalServer>> s3, s4;
    for (int i = 0; i < 3; ++i) s3.emplace_back(new demo::LocalServer("3way-" + std::to_string(i)));
    for (int i = 0; i < 4; ++i) s4.emplace_back(new demo::LocalServer("4way-" + std::to_string(i)));
    char path[] = "/tmp/mrpc_dynpart_XXXXXX";
    const int fd = mkstemp(path);
    if (fd < 0) return 1;
    close(fd);
    auto write_list = [&](bool with_3way) {
        std::ofstream f(path);
        if (with_3way) {
            for (int i = 0; i < 3; ++i) f << s3[i]->addr() << " " << i << "/3\n";
        }
        for (int i = 0; i < 4; ++i) f << s4[i]->addr() << " " << i << "/4\n";
    };
    write_list(true);

    mrpc::PartitionParser parser;  // "index/count" tags
    mrpc::PartitionChannelOptions opt;
    opt.timeout_ms = 2000;
    opt.response_merger = std::make_shared<Merger>();
    mrpc::DynamicPartitionChannel ch;
    if (ch.Init(&parser, (std::string("file://") + path).c_str(), "rr", &opt) != 0) return 1;
    example::EchoService_Stub stub(&ch);
    printf("schemes served: %d\n", ch.scheme_count());
    bool ok = ch.scheme_count() == 2;
    int by3 = 0, by4 = 0;
    for (int i = 0; i < 200 && ok; ++i) {
        mrpc::Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("q");
        stub.Echo(&cntl, &req, &res, nullptr);
        if (cntl.Failed()) {
            ok = false;
            break;
        }
        // every call is answered by exactly one complete scheme
        const int n3 = count_of(res.message(), "@3way-"), n4 = count_of(res.message(), "@4way-");
        if (n3 == 3 && n4 == 0) ++by3;
        else if (n4 == 4 && n3 == 0) ++by4;
        else ok = false;
    }
    printf("calls served by the 3-way scheme: %d, by the 4-way scheme: %d\n", by3, by4);
    ok = ok && by3 > 0 && by4 > 0;

    // migration done: the 3-way servers leave the list
    write_list(false);
    ch.Refresh();
    printf("schemes served after the migration: %d\n", ch.scheme_count());
    ok = ok && ch.scheme_count() == 1;
    for (int i = 0; i < 50 && ok; ++i) {
        mrpc::Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("q");
        stub.Echo(&cntl, &req, &res, nullptr);
        ok = !cntl.Failed() && count_of(res.message(), "@4way-") == 4 && count_of(res.message(), "@3way-") == 0;
    }
    unlink(path);
    return demo::Check(ok, "calls follow the partition schemes");
}
