#include "builtin/cpu_profiler.h"

#include <cxxabi.h>
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <vector>

#include "fiber/fiber.h"

namespace mrpc {
namespace profiler {

namespace {

const int kMaxDepth = 48;
const size_t kMaxSamples = 1 << 16;

struct Sample {
    int depth;
    void* pc[kMaxDepth];
};

Sample* g_samples = nullptr;
std::atomic<size_t> g_nsample{0};
std::atomic<bool> g_running{false};
std::mutex g_mu;

void on_sigprof(int, siginfo_t*, void*) {
    const int saved_errno = errno;
    const size_t i = g_nsample.fetch_add(1, std::memory_order_relaxed);
    if (i < kMaxSamples) {
        Sample& s = g_samples[i];
        s.depth = backtrace(s.pc, kMaxDepth);
    }
    errno = saved_errno;
}

std::string demangle(const char* name) {
    int status = 0;
    char* d = abi::__cxa_demangle(name, nullptr, nullptr, &status);
    if (status == 0 && d) {
        std::string r = d;
        free(d);
        return r;
    }
    return name;
}

}  // namespace

std::string Symbolize(uintptr_t addr) {
    Dl_info info;
    if (dladdr(reinterpret_cast<void*>(addr), &info) && info.dli_sname) {
        return demangle(info.dli_sname);
    }
    if (dladdr(reinterpret_cast<void*>(addr), &info) && info.dli_fname) {
        const char* base = strrchr(info.dli_fname, '/');
        char buf[64];
        snprintf(buf, sizeof(buf), "+0x%lx", (unsigned long)(addr - (uintptr_t)info.dli_fbase));
        return std::string(base ? base + 1 : info.dli_fname) + buf;
    }
    char buf[32];
    snprintf(buf, sizeof(buf), "0x%lx", (unsigned long)addr);
    return buf;
}

bool IsCpuProfilerRunning() { return g_running.load(); }

bool ProfileCpu(double seconds, int frequency_hz, std::string* folded, std::string* pprof_binary, int64_t* nsamples) {
    std::unique_lock<std::mutex> lk(g_mu, std::try_to_lock);
    if (!lk.owns_lock() || g_running.exchange(true)) return false;
    if (frequency_hz <= 0 || frequency_hz > 4000) frequency_hz = 100;
    if (!g_samples) g_samples = new Sample[kMaxSamples];
    {
        void* warm[4];
        backtrace(warm, 4);  // first call loads libgcc outside the handler
    }
    g_nsample.store(0);
    struct sigaction sa, old_sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = on_sigprof;
    sa.sa_flags = SA_RESTART | SA_SIGINFO;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGPROF, &sa, &old_sa);
    const long period_us = 1000000L / frequency_hz;
    itimerval tv;
    tv.it_interval.tv_sec = period_us / 1000000;
    tv.it_interval.tv_usec = period_us % 1000000;
    tv.it_value = tv.it_interval;
    setitimer(ITIMER_PROF, &tv, nullptr);
    const int64_t us = (int64_t)(seconds * 1e6);
    if (fiber::worker_index() >= 0) {
        fiber::usleep(us);
    } else {
        usleep(us);
    }
    itimerval zero;
    memset(&zero, 0, sizeof(zero));
    setitimer(ITIMER_PROF, &zero, nullptr);
    sigaction(SIGPROF, &old_sa, nullptr);
    const size_t n = std::min(g_nsample.load(), kMaxSamples);
    if (nsamples) *nsamples = (int64_t)n;

    // aggregate identical stacks (skip the handler + signal trampoline frames)
    std::map<std::vector<void*>, int64_t> stacks;
    for (size_t i = 0; i < n; ++i) {
        const Sample& s = g_samples[i];
        const int skip = std::min(2, s.depth);
        std::vector<void*> st(s.pc + skip, s.pc + s.depth);
        ++stacks[st];
    }
    if (folded) {
        std::map<void*, std::string> names;
        std::vector<std::pair<int64_t, std::string>> lines;
        for (auto& kv : stacks) {
            std::string line;
            for (auto it = kv.first.rbegin(); it != kv.first.rend(); ++it) {
                auto f = names.find(*it);
                if (f == names.end()) f = names.emplace(*it, Symbolize((uintptr_t)*it)).first;
                if (!line.empty()) line += ";";
                std::string nm = f->second;
                std::replace(nm.begin(), nm.end(), ';', ':');
                std::replace(nm.begin(), nm.end(), ' ', '_');
                line += nm;
            }
            lines.emplace_back(kv.second, line);
        }
        std::sort(lines.begin(), lines.end(), [](auto& a, auto& b) { return a.first > b.first; });
        std::ostringstream os;
        for (auto& l : lines) os << l.second << " " << l.first << "\n";
        *folded = os.str();
    }
    if (pprof_binary) {
        // gperftools legacy CPU profile: header, samples, trailer, maps
        std::vector<uintptr_t> w = {0, 3, 0, (uintptr_t)period_us, 0};
        for (auto& kv : stacks) {
            w.push_back((uintptr_t)kv.second);
            w.push_back(kv.first.size());
            for (void* pc : kv.first) w.push_back((uintptr_t)pc);
        }
        w.push_back(0);
        w.push_back(1);
        w.push_back(0);
        pprof_binary->assign(reinterpret_cast<const char*>(w.data()), w.size() * sizeof(uintptr_t));
        std::ifstream maps("/proc/self/maps");
        std::stringstream ss;
        ss << maps.rdbuf();
        pprof_binary->append(ss.str());
    }
    g_running.store(false);
    return true;
}

}  // namespace profiler
}  // namespace mrpc
