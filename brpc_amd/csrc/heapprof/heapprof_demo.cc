// Heap profiler demo + self-check: this executable links heapprof.cc, keeps
// ~48 MiB live from one known function and churns ~200 MiB through another,
// then reads /hotspots/heap, /hotspots/growth and /pprof/heap from its own
// builtin services and checks the sampled estimates name the right code.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "base/flags.h"
#include "http/http_header.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/server.h"

std::vector<void*> g_keep;
void* volatile g_sink;  // keeps the compiler from eliding malloc/free pairs

__attribute__((noinline)) void KeepLiveBuffers() {
    for (int i = 0; i < 3072; ++i) {
        void* p = malloc(16384);
        memset(p, 1, 64);
        g_keep.push_back(p);
    }
}

__attribute__((noinline)) void ChurnTemporaryBuffers() {
    for (int i = 0; i < 3200; ++i) {
        char* p = static_cast<char*>(malloc(65536));
        p[0] = 1;
        g_sink = p;
        free(g_sink);
    }
}

std::string Get(mrpc::Channel& ch, const char* path) {
    mrpc::Controller cntl;
    cntl.http_request().uri().set_path(path);
    ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    if (cntl.Failed()) return "FAILED: " + cntl.ErrorText();
    return cntl.response_attachment().to_string();
}

long long BytesOf(const std::string& report, const char* fn) {
    long long total = 0;
    size_t b = 0;
    while (b < report.size()) {
        size_t e = report.find('\n', b);
        if (e == std::string::npos) e = report.size();
        const std::string line = report.substr(b, e - b);
        const size_t first_sym = line.find(' ', line.find(' ') + 1);
        // attribute a row to fn if fn is among its first frames
        if (!line.empty() && line[0] != '#' && line.find(fn) != std::string::npos && first_sym != std::string::npos &&
            line.find(fn) < first_sym + 200) {
            total += atoll(line.c_str());
        }
        b = e + 1;
    }
    return total;
}

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    mrpc::Server server;
    if (server.Start("127.0.0.1:0", nullptr) != 0) return 1;
    KeepLiveBuffers();
    ChurnTemporaryBuffers();
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.protocol = "http";
    opt.timeout_ms = 5000;
    if (ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &opt) != 0) return 1;
    const std::string heap = Get(ch, "/hotspots/heap");
    const std::string growth = Get(ch, "/hotspots/growth");
    const std::string raw = Get(ch, "/pprof/heap");
    const long long live_keep = BytesOf(heap, "KeepLiveBuffers");
    const long long live_churn = BytesOf(heap, "ChurnTemporaryBuffers");
    const long long grow_churn = BytesOf(growth, "ChurnTemporaryBuffers");
    printf("%s\n", heap.substr(0, 600).c_str());
    printf("in-use KeepLiveBuffers ~%lld MiB (true 48), in-use Churn ~%lld MiB (true 0), growth Churn ~%lld MiB "
           "(true 200)\n",
           live_keep >> 20, live_churn >> 20, grow_churn >> 20);
    const bool ok = raw.compare(0, 14, "heap profile: ") == 0 && raw.find("MAPPED_LIBRARIES:") != std::string::npos &&
                    live_keep > (24ll << 20) && live_keep < (96ll << 20) && live_churn < (8ll << 20) &&
                    grow_churn > (100ll << 20) && grow_churn < (400ll << 20);
    printf("%-48s %s\n", "sampling heap profiler", ok ? "OK" : "FAILED");
    return ok ? 0 : 1;
}
