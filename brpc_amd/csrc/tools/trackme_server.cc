// trackme_server: collects TrackMe reports from servers started with
// -trackme_server=<this address> (role of the reference's
// tools/trackme_server). Reporters are listed at /TrackMeService and on
// stdout; -bug_file lists version ranges with a severity and a message that
// is sent back to the reporting servers:
//     <min_version> <max_version> <warning|fatal> <text...>
#include <unistd.h>

#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "mrpc/proto/tools.pb.h"
#include "rpc/controller.h"
#include "rpc/server.h"

DEFINE_int32(port, 8877, "listening port");
DEFINE_string(bug_file, "", "version ranges reported back as warning/fatal");
DEFINE_int32(reporting_interval, 0, "if >0, tell reporters to use this interval (seconds)");

using namespace mrpc;

namespace {

struct Bug {
    int64_t lo, hi;
    tools::TrackMeSeverity sev;
    std::string text;
};

std::vector<Bug> LoadBugs(const std::string& path) {
    std::vector<Bug> out;
    if (path.empty()) return out;
    std::ifstream f(path);
    std::string line;
    while (std::getline(f, line)) {
        if (line.empty() || line[0] == '#') continue;
        std::istringstream is(line);
        Bug b;
        std::string sev;
        if (!(is >> b.lo >> b.hi >> sev)) continue;
        std::getline(is, b.text);
        if (!b.text.empty() && b.text[0] == ' ') b.text.erase(0, 1);
        b.sev = sev == "fatal" ? tools::TrackMeFatal : tools::TrackMeWarning;
        out.push_back(b);
    }
    return out;
}

class TrackMeServiceImpl : public tools::TrackMeService {
public:
    explicit TrackMeServiceImpl(std::vector<Bug> bugs) : _bugs(std::move(bugs)) {}
    void TrackMe(RpcController* c, const tools::TrackMeRequest* req, tools::TrackMeResponse* res,
                 Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = static_cast<Controller*>(c);
        const std::string who = req->server_addr().empty() ? cntl->remote_side().to_string() : req->server_addr();
        {
            std::lock_guard<std::mutex> lk(_mu);
            const bool first = _seen.find(who) == _seen.end();
            _seen[who] = std::make_pair(req->rpc_version(), realtime_us());
            if (first) LOG(INFO) << "new reporter " << who << " version=" << req->rpc_version();
        }
        res->set_severity(tools::TrackMeOK);
        for (const Bug& b : _bugs) {
            if (req->rpc_version() >= b.lo && req->rpc_version() <= b.hi) {
                res->set_severity(b.sev);
                res->set_error_text(b.text);
                if (b.sev == tools::TrackMeFatal) break;
            }
        }
        if (FLAGS_reporting_interval > 0) res->set_new_interval(FLAGS_reporting_interval);
    }
    size_t reporters() {
        std::lock_guard<std::mutex> lk(_mu);
        return _seen.size();
    }

private:
    std::vector<Bug> _bugs;
    std::mutex _mu;
    std::map<std::string, std::pair<int64_t, int64_t>> _seen;
};

}  // namespace

int main(int argc, char** argv) {
    ParseCommandLineFlags(&argc, &argv);
    TrackMeServiceImpl svc(LoadBugs(FLAGS_bug_file));
    Server server;
    if (server.AddService(&svc, SERVER_DOESNT_OWN_SERVICE) != 0) return 1;
    if (server.Start(FLAGS_port, nullptr) != 0) {
        LOG(ERROR) << "Fail to start trackme_server on port " << FLAGS_port;
        return 1;
    }
    server.RunUntilAskedToQuit();
    LOG(INFO) << "reporters seen: " << svc.reporters();
    return 0;
}
