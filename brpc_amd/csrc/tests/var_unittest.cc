// Metrics tests (spirit of reference test/bvar_reducer_unittest.cpp,
// bvar_percentile_unittest.cpp, bvar_latency_recorder_unittest.cpp).
#include <thread>
#include <vector>

#include "base/time.h"
#include "var/var.h"
#include "tests/test.h"

using namespace mrpc;
using namespace mrpc::var;

TEST(Var, adder_multithread) {
    Adder<int64_t> a("test_adder_mt");
    std::vector<std::thread> ths;
    for (int t = 0; t < 8; ++t) {
        ths.emplace_back([&a] {
            for (int i = 0; i < 100000; ++i) a << 1;
        });
    }
    for (auto& t : ths) t.join();  // agents merged at thread exit
    EXPECT_EQ(a.get_value(), 800000);
    EXPECT_EQ(Variable::describe_exposed("test_adder_mt"), "800000");
    // update cost
    int64_t t0 = monotonic_ns();
    for (int i = 0; i < 1000000; ++i) a << 1;
    int64_t dt = monotonic_ns() - t0;
    printf("  Adder update: %.2f ns\n", dt / 1e6);
    EXPECT_LT(dt / 1e6, 100.0);
}

TEST(Var, maxer_miner_status) {
    Maxer<int64_t> mx;
    Miner<int64_t> mn;
    for (int i = -5; i <= 5; ++i) {
        mx << i;
        mn << i;
    }
    EXPECT_EQ(mx.get_value(), 5);
    EXPECT_EQ(mn.get_value(), -5);
    EXPECT_EQ(mx.reset(), 5);
    var::Status<std::string> s("test_status_str", "hello");
    EXPECT_EQ(Variable::describe_exposed("test_status_str"), "hello");
    PassiveStatus<int> ps("test_passive", [] { return 42; });
    EXPECT_EQ(Variable::describe_exposed("test_passive"), "42");
    std::vector<std::pair<std::string, std::string>> dumped;
    Variable::dump_exposed(&dumped, "test_pass*");
    ASSERT_EQ(dumped.size(), 1u);
    EXPECT_EQ(dumped[0].second, "42");
    std::string prom = Variable::dump_prometheus();
    EXPECT_TRUE(prom.find("test_passive 42") != std::string::npos);
}

TEST(Var, percentile_accuracy) {
    Percentile p(10);
    for (int i = 1; i <= 100000; ++i) p << i;
    uint32_t p50 = p.get_number(0.5);
    uint32_t p99 = p.get_number(0.99);
    EXPECT_NEAR(p50, 50000, 5000);
    EXPECT_NEAR(p99, 99000, 3000);
}

TEST(Var, latency_histogram_exact) {
    LatencyHistogram h;
    for (int i = 1; i <= 10000; ++i) h.add(i);
    EXPECT_EQ(h.count(), 10000);
    EXPECT_NEAR(h.percentile(0.5), 5000, 60);
    EXPECT_NEAR(h.percentile(0.99), 9900, 100);
    EXPECT_EQ(h.max(), 10000);
    LatencyHistogram h2;
    h2.add(1000000);
    h.merge(h2);
    EXPECT_EQ(h.max(), 1000000);
}

TEST(Var, latency_recorder_expose) {
    LatencyRecorder lr("test_lr");
    for (int i = 0; i < 1000; ++i) lr << (100 + i % 10);
    EXPECT_EQ(lr.count(), 1000);
    EXPECT_GE(lr.latency_percentile(0.99), 100);
    std::string v = Variable::describe_exposed("test_lr_count");
    EXPECT_EQ(v, "1000");
    EXPECT_FALSE(Variable::describe_exposed("test_lr_latency_99").empty());
}

TEST(Var, multi_dimension) {
    MultiDimension<Adder<int64_t>> md("test_md_requests", {"method", "code"});
    *md.get_stats({"Echo", "0"}) << 3;
    *md.get_stats({"Echo", "1008"}) << 1;
    EXPECT_EQ(md.count_stats(), 2u);
    std::string prom = Variable::dump_prometheus();
    EXPECT_TRUE(prom.find("test_md_requests{method=\"Echo\",code=\"0\"} 3") != std::string::npos);
}
