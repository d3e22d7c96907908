// rpc_replay: resend requests captured by -rpc_dump (role of the
// reference's tools/rpc_replay). Requests are sent byte-for-byte
// (SerializedRequest) with their recorded protocol, method, compression and
// attachment, at -qps (0: as fast as -thread_num closed-loop senders go),
// -times passes over the dump; the latency table matches rpc_press.
#include <unistd.h>

#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "base/flags.h"
#include "base/recordio.h"
#include "base/time.h"
#include "fiber/fiber.h"
#include "mrpc/proto/rpc_dump.pb.h"
#include "pb/descriptor.h"
#include "rpc/channel.h"
#include "rpc/protocol.h"
#include "rpc/rpc_dump.h"
#include "rpc/serialized_request.h"
#include "rpc/server.h"
#include "var/percentile.h"

DEFINE_string(dir, "./rpc_data/rpc_dump", "directory of rpc_dump files (or one file)");
DEFINE_string(server, "127.0.0.1:8002", "ip:port, or a naming service url with -lb_policy");
DEFINE_string(lb_policy, "", "load balancer when -server is a naming service url");
DEFINE_string(protocol, "", "override the recorded protocol");
DEFINE_int32(thread_num, 1, "concurrent senders");
DEFINE_double(qps, 0, "target qps (0: closed loop)");
DEFINE_int32(times, 1, "passes over the dumped requests");
DEFINE_int32(timeout_ms, 1000, "RPC timeout");
DEFINE_int32(max_retry, 0, "max retries");
DEFINE_int32(dummy_port, -1, "builtin-service dummy server port (-1: off)");

using namespace mrpc;

namespace {

struct Sample {
    RpcDumpMeta meta;
    Buf body, attachment;
    const pb::MethodDescriptor* method = nullptr;
};

// Runtime descriptors for recorded "service.method" names.
const pb::MethodDescriptor* MethodFor(const RpcDumpMeta& m) {
    static std::mutex mu;
    static std::map<std::string, std::unique_ptr<pb::ServiceDescriptor>> services;
    std::lock_guard<std::mutex> g(mu);
    std::unique_ptr<pb::ServiceDescriptor>& sd = services[m.service_name()];
    if (!sd) {
        sd.reset(new pb::ServiceDescriptor);
        sd->full_name = m.service_name();
        const size_t dot = sd->full_name.rfind('.');
        sd->name = dot == std::string::npos ? sd->full_name : sd->full_name.substr(dot + 1);
        sd->methods.reserve(256);  // stable addresses
    }
    for (auto& md : sd->methods) {
        if (md.name == m.method_name()) return &md;
    }
    if (sd->methods.size() >= 256) return nullptr;
    pb::MethodDescriptor md;
    md.name = m.method_name();
    md.full_name = sd->full_name + "." + md.name;
    md.service = sd.get();
    md.index = m.has_method_index() ? m.method_index() : (int)sd->methods.size();
    sd->methods.push_back(md);
    return &sd->methods.back();
}

bool LoadSamples(std::vector<Sample>* out) {
    std::vector<std::string> files;
    if (access((FLAGS_dir + "/.").c_str(), F_OK) == 0) {
        for (const std::string& f : ListRpcDumpFiles(FLAGS_dir)) files.push_back(FLAGS_dir + "/" + f);
    } else {
        files.push_back(FLAGS_dir);
    }
    for (const std::string& path : files) {
        RecordReader rd(path);
        if (!rd.ok()) continue;
        Record r;
        while (rd.ReadNext(&r)) {
            const Buf* mb = r.Meta("meta");
            Sample s;
            if (!mb || !s.meta.ParseFromBuf(*mb)) continue;
            Buf payload = r.Payload();
            const size_t att = (size_t)std::max(0, s.meta.attachment_size());
            if (att > payload.size()) continue;
            payload.cutn(&s.body, payload.size() - att);
            s.attachment.swap(payload);
            s.method = MethodFor(s.meta);
            if (s.method) out->push_back(std::move(s));
        }
    }
    return !out->empty();
}

}  // namespace

int main(int argc, char** argv) {
    ParseCommandLineFlags(&argc, &argv);
    GlobalInitializeOrDie();
    if (FLAGS_dummy_port >= 0) StartDummyServerAt(FLAGS_dummy_port);
    std::vector<Sample> samples;
    if (!LoadSamples(&samples)) {
        fprintf(stderr, "rpc_replay: no request found in %s\n", FLAGS_dir.c_str());
        return 1;
    }
    // one channel per protocol
    std::map<std::string, std::unique_ptr<Channel>> channels;
    for (const Sample& s : samples) {
        const std::string proto =
            !FLAGS_protocol.empty() ? FLAGS_protocol : ProtocolTypeToString(s.meta.protocol_type());
        if (channels.count(proto)) continue;
        ChannelOptions opt;
        opt.protocol = proto;
        opt.timeout_ms = FLAGS_timeout_ms;
        opt.max_retry = FLAGS_max_retry;
        std::unique_ptr<Channel> ch(new Channel);
        const int rc = FLAGS_lb_policy.empty() ? ch->Init(FLAGS_server.c_str(), &opt)
                                               : ch->Init(FLAGS_server.c_str(), FLAGS_lb_policy.c_str(), &opt);
        if (rc != 0) {
            fprintf(stderr, "rpc_replay: cannot init %s channel to %s\n", proto.c_str(), FLAGS_server.c_str());
            return 1;
        }
        channels[proto] = std::move(ch);
    }
    const int64_t total = (int64_t)samples.size() * std::max(1, FLAGS_times);
    std::atomic<int64_t> next{0}, ok{0}, fail{0};
    std::mutex hist_mu;
    var::LatencyHistogram hist;
    const int64_t pace_us = FLAGS_qps > 0 ? (int64_t)(1e6 * FLAGS_thread_num / FLAGS_qps) : 0;
    const int64_t t0 = monotonic_us();
    auto sender = [&]() {
        var::LatencyHistogram local;
        int64_t due = monotonic_us();
        for (;;) {
            const int64_t i = next.fetch_add(1);
            if (i >= total) break;
            if (pace_us) {
                const int64_t now = monotonic_us();
                if (due > now) fiber::usleep(due - now);
                due += pace_us;
            }
            const Sample& s = samples[(size_t)(i % (int64_t)samples.size())];
            const std::string proto =
                !FLAGS_protocol.empty() ? FLAGS_protocol : ProtocolTypeToString(s.meta.protocol_type());
            Controller cntl;
            SerializedRequest req;
            SerializedRequest res;  // keeps the raw response bytes
            req.serialized_data() = s.body;
            cntl.request_attachment() = s.attachment;
            cntl.set_request_compress_type(s.meta.compress_type());
            const int64_t b = monotonic_us();
            channels[proto]->CallMethod(s.method, &cntl, &req, &res, nullptr);
            local.add(monotonic_us() - b);
            (cntl.Failed() ? fail : ok).fetch_add(1);
            if (cntl.Failed() && fail.load() <= 5) fprintf(stderr, "rpc_replay: %s\n", cntl.ErrorText().c_str());
        }
        std::lock_guard<std::mutex> g(hist_mu);
        hist.merge(local);
    };
    std::vector<fiber::fiber_t> tids(std::max(1, FLAGS_thread_num));
    struct Arg {
        std::function<void()> fn;
    } arg{sender};
    for (auto& t : tids) {
        fiber::start_background(&t, nullptr, [](void* a) -> void* {
            static_cast<Arg*>(a)->fn();
            return nullptr;
        }, &arg);
    }
    for (auto t : tids) fiber::join(t);
    const double secs = (monotonic_us() - t0) / 1e6;
    printf("[Summary] replayed:%lld success:%lld error:%lld elapsed:%.2fs qps:%.0f\n", (long long)total,
           (long long)ok.load(), (long long)fail.load(), secs, secs > 0 ? total / secs : 0.0);
    printf("[Latency]\n  avg %10.0f us\n  50%% %10lld us\n  90%% %10lld us\n  99%% %10lld us\n  99.9%% %8lld us\n"
           "  max %10lld us\n",
           hist.mean(), (long long)hist.percentile(0.5), (long long)hist.percentile(0.9),
           (long long)hist.percentile(0.99), (long long)hist.percentile(0.999), (long long)hist.max());
    return fail.load() == 0 ? 0 : 2;
}
