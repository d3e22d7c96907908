// Admission control and breaker units, after the reference's
// test/brpc_adaptive_max_concurrency_unittest.cpp,
// brpc_auto_concurrency_limiter_unittest.cpp,
// brpc_timeout_concurrency_limiter_unittest.cpp and
// brpc_circuit_breaker_unittest.cpp: the max_concurrency spellings, each
// built-in limiter's accept/reject rule and what its feedback changes, a
// user-registered limiter, and breaker reset / isolation bookkeeping.
#include <memory>
#include <string>

#include "base/flags.h"
#include "base/time.h"
#include "cluster/circuit_breaker.h"
#include "net/socket.h"
#include "rpc/concurrency_limiter.h"
#include "rpc/errno.h"
#include "tests/test.h"

DECLARE_int32(auto_cl_initial_max_concurrency);
DECLARE_int32(auto_cl_min_sample_count);
DECLARE_int32(auto_cl_max_sample_count);
DECLARE_int32(timeout_cl_max_concurrency);
DECLARE_int32(timeout_cl_default_timeout_ms);
DECLARE_int32(timeout_cl_initial_avg_latency_us);
DECLARE_int32(circuit_breaker_min_isolation_duration_ms);
DECLARE_int32(circuit_breaker_max_isolation_duration_ms);

using namespace mrpc;

namespace {

struct FlagScope {
    int32_t* p;
    int32_t old;
    FlagScope(int32_t* flag, int32_t v) : p(flag), old(*flag) { *p = v; }
    ~FlagScope() { *p = old; }
};

class CountingLimiter : public ConcurrencyLimiter {
public:
    explicit CountingLimiter(int every = 0) : _every(every) {}
    bool OnRequested(int, Controller*) override { return _every == 0 || (++_n % _every) != 0; }
    void OnResponded(int, int64_t) override {}
    int MaxConcurrency() override { return -7; }
    ConcurrencyLimiter* New(const AdaptiveMaxConcurrency&) const override { return new CountingLimiter(3); }

private:
    int _every;
    int _n = 0;
};

}  // namespace

TEST(LimiterUnit, max_concurrency_spellings) {
    EXPECT_EQ(AdaptiveMaxConcurrency().type(), std::string("unlimited"));
    EXPECT_EQ(AdaptiveMaxConcurrency("").type(), std::string("unlimited"));
    EXPECT_EQ(AdaptiveMaxConcurrency("0").type(), std::string("unlimited"));
    EXPECT_EQ(AdaptiveMaxConcurrency("unlimited").type(), std::string("unlimited"));
    EXPECT_EQ(AdaptiveMaxConcurrency("128").type(), std::string("constant"));
    EXPECT_EQ(AdaptiveMaxConcurrency("128").max_concurrency(), 128);
    EXPECT_EQ(AdaptiveMaxConcurrency(3).value(), std::string("3"));
    EXPECT_EQ(AdaptiveMaxConcurrency("auto").max_concurrency(), 0);
    EXPECT_EQ(AdaptiveMaxConcurrency("timeout").type(), std::string("timeout"));
}

TEST(LimiterUnit, equality_compares_the_spelling) {
    EXPECT_TRUE(AdaptiveMaxConcurrency(10) == AdaptiveMaxConcurrency("10"));
    EXPECT_TRUE(AdaptiveMaxConcurrency("auto") == AdaptiveMaxConcurrency(std::string("auto")));
    EXPECT_FALSE(AdaptiveMaxConcurrency(10) == AdaptiveMaxConcurrency(11));
    EXPECT_FALSE(AdaptiveMaxConcurrency("auto") == AdaptiveMaxConcurrency("timeout"));
}

TEST(LimiterUnit, constant_limiter_admits_up_to_its_max) {
    std::unique_ptr<ConcurrencyLimiter> l(CreateConcurrencyLimiter(AdaptiveMaxConcurrency(3)));
    ASSERT_TRUE(l != nullptr);
    EXPECT_EQ(l->MaxConcurrency(), 3);
    EXPECT_TRUE(l->OnRequested(1, nullptr));
    EXPECT_TRUE(l->OnRequested(3, nullptr));
    EXPECT_FALSE(l->OnRequested(4, nullptr));
    l->OnResponded(0, 1000000);  // feedback changes nothing
    EXPECT_EQ(l->MaxConcurrency(), 3);
}

TEST(LimiterUnit, auto_limiter_starts_from_the_initial_flag) {
    FlagScope f(&FLAGS_auto_cl_initial_max_concurrency, 17);
    std::unique_ptr<ConcurrencyLimiter> l(CreateConcurrencyLimiter(AdaptiveMaxConcurrency("auto")));
    ASSERT_TRUE(l != nullptr);
    EXPECT_EQ(l->MaxConcurrency(), 17);
    EXPECT_TRUE(l->OnRequested(17, nullptr));
    EXPECT_FALSE(l->OnRequested(18, nullptr));
}

TEST(LimiterUnit, auto_limiter_waits_for_enough_samples) {
    std::unique_ptr<ConcurrencyLimiter> l(CreateConcurrencyLimiter(AdaptiveMaxConcurrency("auto")));
    const int before = l->MaxConcurrency();
    for (int i = 0; i < FLAGS_auto_cl_min_sample_count - 1; ++i) l->OnResponded(0, 1000);
    EXPECT_EQ(l->MaxConcurrency(), before);
}

TEST(LimiterUnit, auto_limiter_ignores_its_own_rejections) {
    std::unique_ptr<ConcurrencyLimiter> l(CreateConcurrencyLimiter(AdaptiveMaxConcurrency("auto")));
    const int before = l->MaxConcurrency();
    for (int i = 0; i < 5 * FLAGS_auto_cl_max_sample_count; ++i) l->OnResponded(ELIMIT, 10);
    EXPECT_EQ(l->MaxConcurrency(), before);
}

TEST(LimiterUnit, auto_limiter_recomputes_after_a_full_window) {
    std::unique_ptr<ConcurrencyLimiter> l(CreateConcurrencyLimiter(AdaptiveMaxConcurrency("auto")));
    const int before = l->MaxConcurrency();
    // max_sample_count samples close a window at once; the new limit is
    // min_latency * peak_qps * (1 + explore ratio) >= 1
    for (int i = 0; i < FLAGS_auto_cl_max_sample_count; ++i) l->OnResponded(0, 2000);
    EXPECT_NE(l->MaxConcurrency(), before);
    EXPECT_GE(l->MaxConcurrency(), 1);
}

TEST(LimiterUnit, timeout_limiter_caps_at_its_max) {
    FlagScope f(&FLAGS_timeout_cl_max_concurrency, 10);
    std::unique_ptr<ConcurrencyLimiter> l(CreateConcurrencyLimiter(AdaptiveMaxConcurrency("timeout")));
    ASSERT_TRUE(l != nullptr);
    EXPECT_EQ(l->MaxConcurrency(), 10);
    EXPECT_TRUE(l->OnRequested(10, nullptr));
    EXPECT_FALSE(l->OnRequested(11, nullptr));
}

TEST(LimiterUnit, timeout_limiter_rejects_what_would_miss_the_deadline) {
    FlagScope f1(&FLAGS_timeout_cl_max_concurrency, 100000);
    FlagScope f2(&FLAGS_timeout_cl_default_timeout_ms, 10);
    FlagScope f3(&FLAGS_timeout_cl_initial_avg_latency_us, 1000);
    std::unique_ptr<ConcurrencyLimiter> l(CreateConcurrencyLimiter(AdaptiveMaxConcurrency("timeout")));
    // queueing estimate cur * 1 ms / 8 against a 10 ms budget: 80 fit, 81 do not
    EXPECT_TRUE(l->OnRequested(80, nullptr));
    EXPECT_FALSE(l->OnRequested(81, nullptr));
}

TEST(LimiterUnit, timeout_limiter_learns_from_successes_only) {
    FlagScope f1(&FLAGS_timeout_cl_max_concurrency, 100000);
    FlagScope f2(&FLAGS_timeout_cl_default_timeout_ms, 10);
    FlagScope f3(&FLAGS_timeout_cl_initial_avg_latency_us, 1000);
    std::unique_ptr<ConcurrencyLimiter> l(CreateConcurrencyLimiter(AdaptiveMaxConcurrency("timeout")));
    for (int i = 0; i < 100; ++i) l->OnResponded(EINTERNAL, 1000000);  // failures: ignored
    EXPECT_TRUE(l->OnRequested(80, nullptr));
    for (int i = 0; i < 100; ++i) l->OnResponded(0, 10000);  // slow successes: avg -> ~10 ms
    EXPECT_FALSE(l->OnRequested(80, nullptr));
    EXPECT_TRUE(l->OnRequested(8, nullptr));
}

TEST(LimiterUnit, user_registered_limiters_are_created_by_name) {
    RegisterConcurrencyLimiter("every_third", new CountingLimiter);
    std::unique_ptr<ConcurrencyLimiter> l(CreateConcurrencyLimiter(AdaptiveMaxConcurrency("every_third")));
    ASSERT_TRUE(l != nullptr);
    EXPECT_EQ(l->MaxConcurrency(), -7);
    int admitted = 0;
    for (int i = 0; i < 9; ++i) admitted += l->OnRequested(1, nullptr) ? 1 : 0;
    EXPECT_EQ(admitted, 6);
    EXPECT_TRUE(CreateConcurrencyLimiter(AdaptiveMaxConcurrency("no_such_limiter")) == nullptr);
}

TEST(BreakerUnit, reset_forgets_errors) {
    CircuitBreaker b;
    for (int i = 0; i < 3000; ++i) b.OnCallEnd(0, 1000);  // past the initialization windows
    int tripped_at = -1;
    for (int i = 0; i < 500 && tripped_at < 0; ++i) {
        if (!b.OnCallEnd(EINTERNAL, 1000)) tripped_at = i;
    }
    ASSERT_TRUE(tripped_at >= 0);
    b.Reset();
    // a fresh initialization window: a few errors are tolerated again
    EXPECT_TRUE(b.OnCallEnd(EINTERNAL, 1000));
    EXPECT_TRUE(b.OnCallEnd(0, 1000));
}

TEST(BreakerUnit, isolation_marks_and_expires) {
    FlagScope f(&FLAGS_circuit_breaker_min_isolation_duration_ms, 20);
    CircuitBreaker b;
    const int64_t now = monotonic_us();
    EXPECT_FALSE(b.isolated(now));
    b.MarkIsolated(now);
    EXPECT_EQ(b.isolated_times(), 1);
    EXPECT_TRUE(b.isolated(now + 1000));
    EXPECT_FALSE(b.OnCallEnd(0, 100));  // isolated: every call counts as refused
    EXPECT_FALSE(b.isolated(now + (int64_t)b.isolation_duration_ms() * 1000 + 1));
}

TEST(BreakerUnit, isolation_duration_is_capped) {
    FlagScope f1(&FLAGS_circuit_breaker_min_isolation_duration_ms, 100);
    FlagScope f2(&FLAGS_circuit_breaker_max_isolation_duration_ms, 1000);
    CircuitBreaker b;
    int64_t now = monotonic_us();
    int last = 0;
    for (int i = 0; i < 10; ++i) {
        b.MarkIsolated(now);
        last = b.isolation_duration_ms();
        EXPECT_LE(last, 1000);
    }
    EXPECT_EQ(last, 1000);
    EXPECT_EQ(b.isolated_times(), 10);
}

TEST(BreakerUnit, isolation_restarts_small_after_a_long_healthy_spell) {
    FlagScope f1(&FLAGS_circuit_breaker_min_isolation_duration_ms, 100);
    FlagScope f2(&FLAGS_circuit_breaker_max_isolation_duration_ms, 1000);
    CircuitBreaker b;
    const int64_t now = monotonic_us();
    b.MarkIsolated(now);
    b.MarkIsolated(now);
    EXPECT_TRUE(b.isolation_duration_ms() > 100);
    // the next trip comes long (> max isolation) after the last reset
    b.MarkIsolated(now + 5 * 1000 * 1000);
    EXPECT_EQ(b.isolation_duration_ms(), 100);
}

TEST(BreakerUnit, unknown_servers_are_never_isolated) {
    EXPECT_FALSE(IsIsolatedByCircuitBreaker((SocketId)0x7fff0000deadbeefull));
    FeedCircuitBreaker((SocketId)0x7fff0000deadbef0ull, 0, 100);
    EXPECT_FALSE(IsIsolatedByCircuitBreaker((SocketId)0x7fff0000deadbef0ull));
}
