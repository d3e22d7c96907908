// CircuitBreaker behaviour (spirit of the reference's
// test/brpc_circuit_breaker_unittest.cpp): healthy traffic never trips,
// the initialization window counts errors, a failure burst after warm-up
// trips within the window's error budget, a low error rate does not, the
// error cost decays, and isolation durations double on repeated trips.
#include <cstdlib>

#include "base/flags.h"
#include "base/time.h"
#include "cluster/circuit_breaker.h"
#include "rpc/errno.h"
#include "tests/test.h"

DECLARE_int32(circuit_breaker_short_window_size);
DECLARE_int32(circuit_breaker_long_window_size);
DECLARE_int32(circuit_breaker_short_window_error_percent);
DECLARE_int32(circuit_breaker_long_window_error_percent);
DECLARE_int32(circuit_breaker_min_isolation_duration_ms);
DECLARE_int32(circuit_breaker_max_isolation_duration_ms);

using namespace mrpc;

namespace {

// Feeds n calls; returns the index of the first call that tripped, or -1.
int feed(CircuitBreaker& b, int n, int error_code, int64_t latency_us) {
    for (int i = 0; i < n; ++i) {
        if (!b.OnCallEnd(error_code, latency_us)) return i;
    }
    return -1;
}

}  // namespace

TEST(Breaker, healthy_traffic_never_trips) {
    CircuitBreaker b;
    srand(1);
    for (int i = 0; i < 20000; ++i) {
        ASSERT_TRUE(b.OnCallEnd(0, 800 + rand() % 400));
    }
}

TEST(Breaker, initialization_window_counts_errors) {
    // before the short window (1500 samples) has filled, the breaker trips
    // once errors exceed 10% of the window: the 151st error
    CircuitBreaker b;
    EXPECT_EQ(feed(b, 1000, EINTERNAL, 1000), 150);
}

TEST(Breaker, burst_after_warmup_trips_within_the_error_budget) {
    CircuitBreaker b;
    ASSERT_EQ(feed(b, 3000, 0, 1000), -1);  // both windows warm, ema latency 1000 us
    // each failure costs at most 2 x ema latency; the short window tolerates
    // 1000 * 1500 * 10% * 1.02 us of cost: ~77 back-to-back failures
    const int at = feed(b, 1000, EINTERNAL, 5000);
    EXPECT_GE(at, 70);
    EXPECT_LE(at, 80);
}

TEST(Breaker, low_error_rate_stays_healthy) {
    CircuitBreaker b;
    ASSERT_EQ(feed(b, 3000, 0, 1000), -1);
    // 1 failure in 50 (2%), below both windows' budgets (10% / 5%)
    for (int i = 0; i < 30000; ++i) {
        ASSERT_TRUE(b.OnCallEnd(i % 50 == 0 ? EINTERNAL : 0, 1000));
    }
}

TEST(Breaker, error_cost_decays_with_successes) {
    CircuitBreaker b;
    ASSERT_EQ(feed(b, 3000, 0, 1000), -1);
    ASSERT_EQ(feed(b, 60, EINTERNAL, 1000), -1);  // most of the short budget used
    // without successes in between, 30 more failures would trip; after a
    // long healthy stretch the same 30 are absorbed
    ASSERT_EQ(feed(b, 5000, 0, 1000), -1);
    EXPECT_EQ(feed(b, 30, EINTERNAL, 1000), -1);
}

TEST(Breaker, isolation_doubles_when_tripping_again_soon) {
    const int32_t min0 = FLAGS_circuit_breaker_min_isolation_duration_ms;
    CircuitBreaker b;
    const int64_t now = monotonic_us();
    b.MarkIsolated(now);
    EXPECT_EQ(b.isolation_duration_ms(), 2 * min0);  // first trip right after the start counts as "soon"
    EXPECT_TRUE(b.isolated(now + 1000));
    EXPECT_FALSE(b.isolated(now + (int64_t)b.isolation_duration_ms() * 1000 + 1));
    b.MarkIsolated(now + 1000);
    EXPECT_EQ(b.isolation_duration_ms(), 4 * min0);
    b.MarkIsolated(now + 2000);
    EXPECT_EQ(b.isolation_duration_ms(), 8 * min0);
    EXPECT_EQ(b.isolated_times(), 3);
    // capped at the maximum
    for (int i = 0; i < 20; ++i) b.MarkIsolated(now + 3000 + i);
    EXPECT_EQ(b.isolation_duration_ms(), FLAGS_circuit_breaker_max_isolation_duration_ms);
    // a trip long after the last reset starts over at the minimum
    b.MarkIsolated(now + (int64_t)(FLAGS_circuit_breaker_max_isolation_duration_ms + 1000) * 1000 + 5000);
    EXPECT_EQ(b.isolation_duration_ms(), min0);
}

TEST(Breaker, isolated_breaker_refuses_calls) {
    CircuitBreaker b;
    b.MarkIsolated(monotonic_us());
    EXPECT_FALSE(b.OnCallEnd(0, 1000));
}

TEST(Breaker, per_server_registry) {
    const SocketId a = 0x7000000000001ull, c = 0x7000000000002ull;
    EXPECT_FALSE(IsIsolatedByCircuitBreaker(a));
    for (int i = 0; i < 400 && !IsIsolatedByCircuitBreaker(a); ++i) FeedCircuitBreaker(a, EINTERNAL, 1000);
    EXPECT_TRUE(IsIsolatedByCircuitBreaker(a));
    EXPECT_FALSE(IsIsolatedByCircuitBreaker(c));  // another server is unaffected
}
