#include "base/logging.h"

#include <pthread.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <mutex>

#include "base/time.h"

namespace mrpc {

static std::atomic<LogSink*> g_sink{nullptr};
static std::atomic<int> g_min_level{LOG_INFO};
static std::atomic<int> g_verbose{0};

LogSink* SetLogSink(LogSink* sink) { return g_sink.exchange(sink); }
void SetMinLogLevel(int level) { g_min_level.store(level, std::memory_order_relaxed); }
int GetMinLogLevel() { return g_min_level.load(std::memory_order_relaxed); }
void SetVerboseLevel(int v) { g_verbose.store(v, std::memory_order_relaxed); }
int GetVerboseLevel() { return g_verbose.load(std::memory_order_relaxed); }

std::string ErrnoString(int err) {
    char buf[128];
    // GNU strerror_r returns char*
    const char* s = strerror_r(err, buf, sizeof(buf));
    return s ? std::string(s) : std::string("Unknown error");
}

bool LogEverySecondAllowed(std::atomic<int64_t>* last_ns) {
    int64_t now = monotonic_ns();
    int64_t last = last_ns->load(std::memory_order_relaxed);
    if (now - last < 1000000000LL) return false;
    return last_ns->compare_exchange_strong(last, now, std::memory_order_relaxed);
}

LogMessage::LogMessage(const char* file, int line, int severity, bool with_errno)
    : _file(file), _line(line), _severity(severity), _saved_errno(errno), _with_errno(with_errno) {}

static const char* kSevChar = "VINWEF";

LogMessage::~LogMessage() {
    if (_with_errno) {
        _os << ": " << ErrnoString(_saved_errno) << " [" << _saved_errno << "]";
    }
    std::string content = _os.str();
    LogSink* sink = g_sink.load(std::memory_order_acquire);
    bool consumed = sink && sink->OnLogMessage(_severity, _file, _line, content);
    if (!consumed) {
        const char* base = strrchr(_file, '/');
        base = base ? base + 1 : _file;
        int64_t us = realtime_us();
        time_t sec = us / 1000000;
        struct tm tmv;
        localtime_r(&sec, &tmv);
        char head[96];
        int n = snprintf(head, sizeof(head), "%c%02d%02d %02d:%02d:%02d.%06d %5d %s:%d] ",
                         kSevChar[_severity + 1], tmv.tm_mon + 1, tmv.tm_mday, tmv.tm_hour, tmv.tm_min,
                         tmv.tm_sec, (int)(us % 1000000), (int)syscall(SYS_gettid), base, _line);
        std::string line(head, n);
        line += content;
        line += '\n';
        fwrite(line.data(), 1, line.size(), stderr);
    }
    errno = _saved_errno;
    if (_severity == LOG_FATAL) {
        fflush(stderr);
        abort();
    }
}

}  // namespace mrpc
