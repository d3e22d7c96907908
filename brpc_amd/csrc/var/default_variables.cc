// Process-level variables from /proc (role of bvar/default_variables.cpp).
#include <dirent.h>
#include <sys/resource.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <mutex>

#include "base/time.h"
#include "var/recorder.h"

namespace mrpc {
namespace var {

namespace {
int64_t g_start_us = realtime_us();

struct ProcStat {
    int64_t utime = 0, stime = 0, nthreads = 0, vsize = 0, rss_pages = 0;
};

bool read_proc_stat(ProcStat* st) {
    FILE* f = fopen("/proc/self/stat", "r");
    if (!f) return false;
    char buf[2048];
    size_t n = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[n] = 0;
    const char* p = strrchr(buf, ')');
    if (!p) return false;
    // fields after comm: state(3) ppid ... utime(14) stime(15) ... num_threads(20) ... vsize(23) rss(24)
    long long vals[30] = {0};
    int idx = 3;
    const char* s = p + 2;
    char state;
    if (sscanf(s, "%c", &state) != 1) return false;
    s += 2;
    while (*s && idx < 25) {
        ++idx;
        vals[idx] = strtoll(s, (char**)&s, 10);
        while (*s == ' ') ++s;
    }
    st->utime = vals[14];
    st->stime = vals[15];
    st->nthreads = vals[20];
    st->vsize = vals[23];
    st->rss_pages = vals[24];
    return true;
}

double cpu_usage() {
    static std::mutex mu;
    static int64_t last_ticks = -1, last_us = 0;
    std::lock_guard<std::mutex> g(mu);
    ProcStat st;
    if (!read_proc_stat(&st)) return 0;
    int64_t ticks = st.utime + st.stime;
    int64_t now = monotonic_us();
    double r = 0;
    if (last_ticks >= 0 && now > last_us) {
        r = (double)(ticks - last_ticks) / sysconf(_SC_CLK_TCK) / ((now - last_us) / 1e6);
    }
    last_ticks = ticks;
    last_us = now;
    return r;
}

int64_t fd_count() {
    DIR* d = opendir("/proc/self/fd");
    if (!d) return 0;
    int64_t n = 0;
    while (readdir(d)) ++n;
    closedir(d);
    return n > 2 ? n - 2 : 0;
}

double loadavg(int i) {
    double l[3] = {0, 0, 0};
    if (getloadavg(l, 3) < 0) return 0;
    return l[i];
}
}  // namespace

void ExposeDefaultVariables() {
    static std::once_flag once;
    std::call_once(once, [] {
        new PassiveStatus<double>("process_cpu_usage", [] { return cpu_usage(); });
        new PassiveStatus<int64_t>("process_memory_resident", [] {
            ProcStat st;
            read_proc_stat(&st);
            return st.rss_pages * (int64_t)sysconf(_SC_PAGESIZE);
        });
        new PassiveStatus<int64_t>("process_memory_virtual", [] {
            ProcStat st;
            read_proc_stat(&st);
            return st.vsize;
        });
        new PassiveStatus<int64_t>("process_thread_count", [] {
            ProcStat st;
            read_proc_stat(&st);
            return st.nthreads;
        });
        new PassiveStatus<int64_t>("process_fd_count", [] { return fd_count(); });
        new PassiveStatus<double>("process_uptime", [] { return (realtime_us() - g_start_us) / 1e6; });
        new PassiveStatus<int64_t>("process_pid", [] { return (int64_t)getpid(); });
        new PassiveStatus<double>("system_loadavg_1m", [] { return loadavg(0); });
        new PassiveStatus<double>("system_loadavg_5m", [] { return loadavg(1); });
        new PassiveStatus<int64_t>("system_core_count", [] { return (int64_t)sysconf(_SC_NPROCESSORS_ONLN); });
        new PassiveStatus<int64_t>("process_max_fds", [] {
            rlimit r;
            getrlimit(RLIMIT_NOFILE, &r);
            return (int64_t)r.rlim_cur;
        });
    });
}

}  // namespace var
}  // namespace mrpc
