// Metrics tests (spirit of reference test/bvar_reducer_unittest.cpp,
// bvar_percentile_unittest.cpp, bvar_latency_recorder_unittest.cpp).
#include <unistd.h>

#include <mutex>
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
    EXPECT_LT(dt / 1e6, 100.0 * mtest::kSlowdown);
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

TEST(Var, multi_dimension_latency_family) {
    MultiDimension<LatencyRecorder> md("test_md_rpc", {"service", "method"});
    LatencyRecorder* a = md.get_stats({"Echo", "Echo"});
    LatencyRecorder* b = md.get_stats({"Kv", "Get"});
    ASSERT_TRUE(a != nullptr && b != nullptr);
    EXPECT_TRUE(md.get_stats({"Echo", "Echo"}) == a);  // same tuple, same metric
    for (int i = 1; i <= 1000; ++i) *a << i;
    *b << 5;
    EXPECT_TRUE(md.get_stats({"only-one"}) == nullptr);  // wrong arity
    std::string prom = Variable::dump_prometheus();
    EXPECT_TRUE(prom.find("# TYPE test_md_rpc_latency summary") != std::string::npos);
    EXPECT_TRUE(prom.find("test_md_rpc_latency{service=\"Echo\",method=\"Echo\",quantile=\"0.99\"}") !=
                std::string::npos);
    EXPECT_TRUE(prom.find("test_md_rpc_latency_count{service=\"Echo\",method=\"Echo\"} 1000") != std::string::npos);
    EXPECT_TRUE(prom.find("test_md_rpc_max_latency{service=\"Kv\",method=\"Get\"} ") != std::string::npos);  // windowed
    EXPECT_TRUE(prom.find("test_md_rpc_qps{service=\"Kv\",method=\"Get\"}") != std::string::npos);
}

TEST(Var, multi_dimension_list_delete_and_cap) {
    MultiDimension<Adder<int64_t>> md("test_md_cap", {"k"});
    for (int i = 0; i < 10; ++i) *md.get_stats({std::to_string(i)}) << i;
    std::vector<std::vector<std::string>> keys;
    md.list_stats(&keys);
    EXPECT_EQ(keys.size(), 10u);
    md.delete_stats({"3"});
    EXPECT_FALSE(md.has_stats({"3"}));
    EXPECT_EQ(md.count_stats(), 9u);
    const int64_t saved = FLAGS_var_max_multi_dimension_stats_count;
    FLAGS_var_max_multi_dimension_stats_count = 9;
    EXPECT_TRUE(md.get_stats({"new"}) == nullptr);  // family full
    EXPECT_TRUE(md.get_stats({"5"}) != nullptr);    // existing tuples still served
    FLAGS_var_max_multi_dimension_stats_count = saved;
    // label values are escaped in the exposition format
    *md.get_stats({"a\"b"}) << 1;
    EXPECT_TRUE(Variable::dump_prometheus().find("test_md_cap{k=\"a\\\"b\"} 1") != std::string::npos);
    md.clear_stats();
    EXPECT_EQ(md.count_stats(), 0u);
}

TEST(Var, multi_dimension_concurrent_get_stats) {
    MultiDimension<Adder<int64_t>> md("test_md_conc", {"shard"});
    std::vector<std::thread> th;
    for (int t = 0; t < 8; ++t) {
        th.emplace_back([&md, t] {
            for (int i = 0; i < 20000; ++i) *md.get_stats({std::to_string((i + t) % 16)}) << 1;
        });
    }
    for (auto& x : th) x.join();
    EXPECT_EQ(md.count_stats(), 16u);
    int64_t total = 0;
    std::vector<std::vector<std::string>> keys;
    md.list_stats(&keys);
    for (auto& k : keys) total += md.get_stats(k)->get_value();
    EXPECT_EQ(total, 8 * 20000);
}

TEST(Var, gflag_follows_flag_value) {
    GFlag g("var_max_multi_dimension_stats_count", "test_gflag_md_cap");
    ASSERT_TRUE(g.valid());
    const std::string before = Variable::describe_exposed("test_gflag_md_cap");
    EXPECT_EQ(before, std::to_string(FLAGS_var_max_multi_dimension_stats_count));
    std::string err;
    ASSERT_TRUE(SetFlag("var_max_multi_dimension_stats_count", "777", false, &err));
    EXPECT_EQ(Variable::describe_exposed("test_gflag_md_cap"), "777");
    double v = 0;
    EXPECT_TRUE(g.get_number(&v));
    EXPECT_EQ(v, 777.0);
    EXPECT_TRUE(Variable::dump_prometheus().find("test_gflag_md_cap 777") != std::string::npos);
    SetFlag("var_max_multi_dimension_stats_count", before, false, &err);
    GFlag bad("no_such_flag_anywhere", "test_gflag_bad");
    EXPECT_FALSE(bad.valid());
    EXPECT_FALSE(bad.get_number(&v));
}

TEST(Var, mutex_with_recorders_measure_contention) {
    MutexWithRecorder<std::mutex> mu;
    MutexWithLatencyRecorder<std::mutex> mu2("test_lock_timer");
    std::vector<std::thread> th;
    int64_t counter = 0;
    for (int t = 0; t < 4; ++t) {
        th.emplace_back([&] {
            for (int i = 0; i < 200; ++i) {
                std::lock_guard<MutexWithRecorder<std::mutex>> g(mu);
                ++counter;
                usleep(50);  // hold it: the others wait
            }
        });
    }
    for (auto& x : th) x.join();
    EXPECT_EQ(counter, 800);
    EXPECT_EQ(mu.recorder().get_value().num, 800);
    EXPECT_GT(mu.recorder().get_value().get_average_int(), 10);  // waited behind holders
    {
        std::unique_lock<MutexWithLatencyRecorder<std::mutex>> g(mu2);
    }
    EXPECT_TRUE(mu2.try_lock());
    mu2.unlock();
    EXPECT_EQ(mu2.recorder().count(), 2);
    EXPECT_FALSE(Variable::describe_exposed("test_lock_timer_count").empty());
    // LockTimer on a plain mutex
    std::mutex raw;
    IntRecorder waits;
    {
        LockTimer<std::mutex, IntRecorder> t(raw, waits);
        EXPECT_FALSE(raw.try_lock());
    }
    EXPECT_TRUE(raw.try_lock());
    raw.unlock();
    EXPECT_EQ(waits.get_value().num, 1);
}
