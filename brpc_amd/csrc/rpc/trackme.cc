#include "rpc/trackme.h"

#include <atomic>
#include <mutex>

#include "base/flags.h"
#include "base/logging.h"
#include "fiber/fiber.h"
#include "mrpc/proto/tools.pb.h"
#include "rpc/channel.h"
#include "rpc/controller.h"

DEFINE_string(trackme_server, "", "ip:port (or naming service url) that collects server versions; empty = off");
DEFINE_int32(trackme_interval, 60, "seconds between two trackme reports");

namespace mrpc {

namespace {
std::mutex g_mu;
EndPoint g_addr;
bool g_started = false;
std::atomic<int64_t> g_sent{0};
std::atomic<int> g_interval{0};

void* TrackMeLoop(void*) {
    Channel ch;
    ChannelOptions opt;
    opt.timeout_ms = 1000;
    opt.max_retry = 0;
    std::string inited_for;
    for (;;) {
        const std::string target = FLAGS_trackme_server;
        if (target.empty()) {
            fiber::usleep(1000000);
            continue;
        }
        if (inited_for != target) {
            const bool is_ns = target.find("://") != std::string::npos;
            if ((is_ns ? ch.Init(target.c_str(), "rr", &opt) : ch.Init(target.c_str(), &opt)) != 0) {
                LOG(WARNING) << "trackme: fail to init channel to " << target;
                fiber::usleep(1000000 * (uint64_t)std::max(1, FLAGS_trackme_interval));
                continue;
            }
            inited_for = target;
        }
        tools::TrackMeRequest req;
        tools::TrackMeResponse res;
        req.set_rpc_version(RpcVersionNumber());
        {
            std::lock_guard<std::mutex> g(g_mu);
            req.set_server_addr(g_addr.to_string());
        }
        Controller cntl;
        tools::TrackMeService_Stub stub(&ch);
        stub.TrackMe(&cntl, &req, &res, nullptr);
        g_sent.fetch_add(1);
        if (!cntl.Failed()) {
            if (res.severity() == tools::TrackMeFatal) {
                LOG(ERROR) << "trackme: this version is reported FATAL: " << res.error_text();
            } else if (res.severity() == tools::TrackMeWarning) {
                LOG(WARNING) << "trackme: " << res.error_text();
            }
            if (res.has_new_interval() && res.new_interval() > 0) g_interval.store(res.new_interval());
        }
        const int iv = g_interval.load() > 0 ? g_interval.load() : FLAGS_trackme_interval;
        fiber::usleep(1000000ull * (uint64_t)std::max(1, iv));
    }
    return nullptr;
}
}  // namespace

int64_t RpcVersionNumber() { return 1 * 10000 + 4 * 100 + 0; }

int64_t TrackMeReportsSent() { return g_sent.load(); }

void SetTrackMeAddress(const EndPoint& ep) {
    if (FLAGS_trackme_server.empty()) return;
    std::lock_guard<std::mutex> g(g_mu);
    g_addr = ep;
    if (g_started) return;
    g_started = true;
    fiber::fiber_t th;
    fiber::start_background(&th, &fiber::ATTR_NORMAL, TrackMeLoop, nullptr);
}

}  // namespace mrpc
