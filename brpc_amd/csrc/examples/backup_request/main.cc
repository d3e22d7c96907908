// Backup request (reference example/backup_request_c++): two replicas, the
// first one slow; with backup_request_ms the channel sends a duplicate to the
// other replica after 2 ms and the first response wins.
#include "base/time.h"
#include "examples/common.h"

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    demo::LocalServer slow("slow", 50000), fast("fast");
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.timeout_ms = 2000;
    opt.backup_request_ms = 2;
    const std::string url = "list://" + slow.addr() + "," + fast.addr();
    if (ch.Init(url.c_str(), "rr", &opt) != 0) return 1;
    example::EchoService_Stub stub(&ch);
    int via_backup = 0, fails = 0;
    for (int i = 0; i < 20; ++i) {
        mrpc::Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("b");
        cntl.set_log_id(i);
        stub.Echo(&cntl, &req, &res, nullptr);
        if (cntl.Failed()) ++fails;
        if (res.message() == "b@fast" && cntl.has_backup_request()) ++via_backup;
    }
    printf("%d calls answered by the backup replica, %d failed\n", via_backup, fails);
    return demo::Check(fails == 0 && via_backup >= 5, "backup requests");
}
