#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdlib>

#include "base/flags.h"
#include "base/time.h"
#include "tests/test.h"

namespace mtest {
std::vector<TestCase>& registry() {
    static std::vector<TestCase>* r = new std::vector<TestCase>;
    return *r;
}
int g_failures_in_current = 0;
void report_failure(const char* file, int line, const std::string& msg) {
    fprintf(stderr, "  FAILURE %s:%d: %s\n", file, line, msg.c_str());
    ++g_failures_in_current;
}
}  // namespace mtest

static bool match(const std::string& full, const std::string& filters) {
    if (filters.empty()) return true;
    size_t b = 0;
    while (b <= filters.size()) {
        size_t e = filters.find(',', b);
        if (e == std::string::npos) e = filters.size();
        std::string f = filters.substr(b, e - b);
        if (!f.empty()) {
            if (f.back() == '*') {
                if (full.compare(0, f.size() - 1, f, 0, f.size() - 1) == 0) return true;
            } else if (full == f || full.find(f) != std::string::npos) {
                return true;
            }
        }
        b = e + 1;
    }
    return false;
}

static void crash_handler(int sig) {
    void* frames[64];
    int n = backtrace(frames, 64);
    fprintf(stderr, "*** signal %d, backtrace:\n", sig);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int main(int argc, char** argv) {
    signal(SIGPIPE, SIG_IGN);
    signal(SIGSEGV, crash_handler);
    signal(SIGABRT, crash_handler);
    signal(SIGBUS, crash_handler);
    std::string filter;
    bool list = false;
    std::vector<char*> rest;
    for (int i = 0; i < argc; ++i) {
        if (strncmp(argv[i], "--filter=", 9) == 0) filter = argv[i] + 9;
        else if (strcmp(argv[i], "--list") == 0) list = true;
        else rest.push_back(argv[i]);
    }
    int rc_argc = (int)rest.size();
    char** rc_argv = rest.data();
    mrpc::ParseCommandLineFlags(&rc_argc, &rc_argv);
    int failed = 0, passed = 0;
    for (auto& tc : mtest::registry()) {
        std::string full = std::string(tc.suite) + "." + tc.name;
        if (!match(full, filter)) continue;
        if (list) {
            printf("%s\n", full.c_str());
            continue;
        }
        printf("[ RUN      ] %s\n", full.c_str());
        fflush(stdout);
        mtest::g_failures_in_current = 0;
        int64_t t0 = mrpc::monotonic_us();
        tc.fn();
        int64_t dt = mrpc::monotonic_us() - t0;
        if (mtest::g_failures_in_current) {
            ++failed;
            printf("[  FAILED  ] %s (%ld us)\n", full.c_str(), (long)dt);
        } else {
            ++passed;
            printf("[       OK ] %s (%ld us)\n", full.c_str(), (long)dt);
        }
        fflush(stdout);
    }
    if (!list) printf("[==========] %d passed, %d failed\n", passed, failed);
    fflush(stdout);
    _exit(failed ? 1 : 0);
}
