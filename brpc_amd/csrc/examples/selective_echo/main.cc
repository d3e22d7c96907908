// Selective echo (reference example/selective_echo_c++): a SelectiveChannel
// load-balances over whole sub-channels (replica groups); when one group is
// down, calls fail over to the others.
#include <memory>
#include <set>

#include "examples/common.h"
#include "rpc/combo_channels.h"

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    demo::LocalServer a("groupA"), b("groupB");
    mrpc::SelectiveChannel sc;
    mrpc::ChannelOptions so;
    so.timeout_ms = 1000;
    so.max_retry = 2;
    if (sc.Init("rr", &so) != 0) return 1;
    for (const std::string& addr : {a.addr(), b.addr(), std::string("127.0.0.1:1")}) {  // last group is dead
        auto* ch = new mrpc::Channel;
        mrpc::ChannelOptions o;
        o.timeout_ms = 500;
        o.max_retry = 0;
        ch->Init(addr.c_str(), &o);
        sc.AddChannel(ch, mrpc::OWNS_CHANNEL);
    }
    example::EchoService_Stub stub(&sc);
    std::set<std::string> seen;
    int fails = 0;
    for (int i = 0; i < 30; ++i) {
        mrpc::Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("s");
        stub.Echo(&cntl, &req, &res, nullptr);
        if (cntl.Failed()) ++fails;
        else seen.insert(res.message());
    }
    printf("answered by %zu groups, %d failures\n", seen.size(), fails);
    return demo::Check(fails == 0 && seen.size() == 2, "replica groups with failover");
}
