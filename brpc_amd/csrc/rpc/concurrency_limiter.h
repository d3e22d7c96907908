// Server-side admission control (role of src/brpc/concurrency_limiter.h,
// adaptive_max_concurrency.h, policy/{constant,auto,timeout}_concurrency_limiter).
#pragma once

#include <cstdint>
#include <string>

namespace mrpc {

class Controller;

// "unlimited" (0), an integer, "auto" or "timeout".
class AdaptiveMaxConcurrency {
public:
    AdaptiveMaxConcurrency() : _value("unlimited"), _max(0) {}
    AdaptiveMaxConcurrency(int v);  // NOLINT
    AdaptiveMaxConcurrency(const std::string& s);  // NOLINT
    AdaptiveMaxConcurrency(const char* s) : AdaptiveMaxConcurrency(std::string(s)) {}  // NOLINT
    const std::string& type() const;  // "constant", "unlimited", "auto", "timeout"
    const std::string& value() const { return _value; }
    int max_concurrency() const { return _max; }
    bool operator==(const AdaptiveMaxConcurrency& o) const { return _value == o._value; }

private:
    std::string _value;
    int _max;
};

class ConcurrencyLimiter {
public:
    virtual ~ConcurrencyLimiter() {}
    // false => reject with ELIMIT.
    virtual bool OnRequested(int current_concurrency, Controller* cntl) = 0;
    virtual void OnResponded(int error_code, int64_t latency_us) = 0;
    virtual int MaxConcurrency() = 0;
    virtual ConcurrencyLimiter* New(const AdaptiveMaxConcurrency& amc) const = 0;
};

// nullptr for "unlimited".
ConcurrencyLimiter* CreateConcurrencyLimiter(const AdaptiveMaxConcurrency& amc);
void RegisterConcurrencyLimiter(const std::string& name, const ConcurrencyLimiter* prototype);
void RegisterBuiltinConcurrencyLimiters();

}  // namespace mrpc
