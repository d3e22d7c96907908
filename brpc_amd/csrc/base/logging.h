// Streaming logger: LOG(INFO) << ..., PLOG, CHECK*, VLOG(n), LOG_EVERY_SECOND,
// LOG_ONCE. Capability parity with butil/logging.h (reference
// docs/en/streaming_log.md:148); sinks are pluggable and the minimum level and
// verbose level are runtime flags (see /vlog, /flags).
#pragma once

#include <atomic>
#include <cstring>
#include <sstream>
#include <string>

#include "base/macros.h"

namespace mrpc {

enum LogSeverity { LOG_VERBOSE = -1, LOG_INFO = 0, LOG_NOTICE = 1, LOG_WARNING = 2, LOG_ERROR = 3, LOG_FATAL = 4 };

class LogSink {
public:
    virtual ~LogSink() {}
    // Returns true if the message was consumed (default sink is skipped).
    virtual bool OnLogMessage(int severity, const char* file, int line, const std::string& content) = 0;
};

// Replace the sink, returns the old one. NULL restores stderr logging.
LogSink* SetLogSink(LogSink* sink);
void SetMinLogLevel(int level);
int GetMinLogLevel();
void SetVerboseLevel(int v);
int GetVerboseLevel();
std::string ErrnoString(int err);

class LogMessage {
public:
    LogMessage(const char* file, int line, int severity, bool with_errno = false);
    ~LogMessage();
    std::ostream& stream() { return _os; }
private:
    const char* _file;
    int _line;
    int _severity;
    int _saved_errno;
    bool _with_errno;
    std::ostringstream _os;
};

struct LogVoidify {
    void operator&(std::ostream&) {}
};

bool LogEverySecondAllowed(std::atomic<int64_t>* last_ns);

}  // namespace mrpc

#define MRPC_SEV_INFO ::mrpc::LOG_INFO
#define MRPC_SEV_NOTICE ::mrpc::LOG_NOTICE
#define MRPC_SEV_WARNING ::mrpc::LOG_WARNING
#define MRPC_SEV_ERROR ::mrpc::LOG_ERROR
#define MRPC_SEV_FATAL ::mrpc::LOG_FATAL

#define LOG_IS_ON(sev) (MRPC_SEV_##sev >= ::mrpc::GetMinLogLevel())
#define LOG(sev) \
    !LOG_IS_ON(sev) ? (void)0 : ::mrpc::LogVoidify() & ::mrpc::LogMessage(__FILE__, __LINE__, MRPC_SEV_##sev).stream()
#define PLOG(sev) \
    !LOG_IS_ON(sev) ? (void)0 : ::mrpc::LogVoidify() & ::mrpc::LogMessage(__FILE__, __LINE__, MRPC_SEV_##sev, true).stream()
#define LOG_IF(sev, cond) \
    !((cond) && LOG_IS_ON(sev)) ? (void)0 : ::mrpc::LogVoidify() & ::mrpc::LogMessage(__FILE__, __LINE__, MRPC_SEV_##sev).stream()
#define VLOG_IS_ON(n) ((n) <= ::mrpc::GetVerboseLevel())
#define VLOG(n) \
    !VLOG_IS_ON(n) ? (void)0 : ::mrpc::LogVoidify() & ::mrpc::LogMessage(__FILE__, __LINE__, ::mrpc::LOG_VERBOSE).stream()

#define LOG_EVERY_SECOND(sev)                                                          \
    static std::atomic<int64_t> MRPC_CONCAT(_mrpc_les_, __LINE__){0};                 \
    !(LOG_IS_ON(sev) && ::mrpc::LogEverySecondAllowed(&MRPC_CONCAT(_mrpc_les_, __LINE__))) \
        ? (void)0                                                                      \
        : ::mrpc::LogVoidify() & ::mrpc::LogMessage(__FILE__, __LINE__, MRPC_SEV_##sev).stream()

#define LOG_ONCE(sev)                                                     \
    static std::atomic<bool> MRPC_CONCAT(_mrpc_lonce_, __LINE__){false}; \
    !(LOG_IS_ON(sev) && !MRPC_CONCAT(_mrpc_lonce_, __LINE__).exchange(true)) \
        ? (void)0                                                         \
        : ::mrpc::LogVoidify() & ::mrpc::LogMessage(__FILE__, __LINE__, MRPC_SEV_##sev).stream()

#define CHECK(cond) \
    LOG_IF(FATAL, MRPC_UNLIKELY(!(cond))) << "Check failed: " #cond ". "
#define MRPC_CHECK_OP(a, b, op) \
    LOG_IF(FATAL, MRPC_UNLIKELY(!((a)op(b)))) << "Check failed: " #a " " #op " " #b " (" << (a) << " vs " << (b) << "). "
#define CHECK_EQ(a, b) MRPC_CHECK_OP(a, b, ==)
#define CHECK_NE(a, b) MRPC_CHECK_OP(a, b, !=)
#define CHECK_LT(a, b) MRPC_CHECK_OP(a, b, <)
#define CHECK_LE(a, b) MRPC_CHECK_OP(a, b, <=)
#define CHECK_GT(a, b) MRPC_CHECK_OP(a, b, >)
#define CHECK_GE(a, b) MRPC_CHECK_OP(a, b, >=)
#ifdef NDEBUG
#define DCHECK(cond) while (false) CHECK(cond)
#define DCHECK_EQ(a, b) while (false) CHECK_EQ(a, b)
#define DCHECK_LT(a, b) while (false) CHECK_LT(a, b)
#define DCHECK_GE(a, b) while (false) CHECK_GE(a, b)
#else
#define DCHECK(cond) CHECK(cond)
#define DCHECK_EQ(a, b) CHECK_EQ(a, b)
#define DCHECK_LT(a, b) CHECK_LT(a, b)
#define DCHECK_GE(a, b) CHECK_GE(a, b)
#endif
