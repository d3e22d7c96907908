// Metrics depth, round 6 (spirit of the reference's bvar_reducer_unittest,
// bvar_recorder_unittest, bvar_status_unittest, bvar_multi_dimension_unittest,
// bvar_variable_unittest, bvar_percentile_unittest): reducer identities and
// resets, values merged from exited threads, recorder overflow-free sums,
// passive/status types, registry rendering, multi-dimension families and the
// percentile estimator's accuracy bands.
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <limits>
#include <random>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "tests/test.h"
#include "var/var.h"

using namespace mrpc;
using namespace mrpc::var;

namespace {
bool has(const std::string& hay, const std::string& needle) { return hay.find(needle) != std::string::npos; }
std::string describe(const Variable& v) {
    std::ostringstream os;
    v.describe(os, false);
    return os.str();
}
}  // namespace

TEST(VarMore, adder_identity_is_zero_and_reset_returns_the_sum) {
    Adder<int64_t> a;
    EXPECT_EQ(a.get_value(), 0);
    a << 5 << -2 << 10;
    EXPECT_EQ(a.get_value(), 13);
    EXPECT_EQ(a.reset(), 13);
    EXPECT_EQ(a.get_value(), 0);
    a << 1;
    EXPECT_EQ(a.get_value(), 1);
}

TEST(VarMore, adder_of_doubles_sums_fractions) {
    Adder<double> a;
    for (int i = 0; i < 10; ++i) a << 0.25;
    EXPECT_TRUE(std::fabs(a.get_value() - 2.5) < 1e-9);
}

TEST(VarMore, maxer_and_miner_ignore_the_identity) {
    Maxer<int64_t> mx;
    Miner<int64_t> mn;
    mx << -5 << -9;
    mn << 7 << 3 << 11;
    EXPECT_EQ(mx.get_value(), -5);
    EXPECT_EQ(mn.get_value(), 3);
    EXPECT_EQ(describe(mx), "-5");
    EXPECT_EQ(describe(mn), "3");
}

TEST(VarMore, values_of_exited_threads_are_kept) {
    Adder<int64_t> a;
    Maxer<int64_t> mx;
    std::vector<std::thread> ths;
    for (int t = 0; t < 8; ++t) {
        ths.emplace_back([&, t] {
            for (int i = 0; i < 1000; ++i) a << 1;
            mx << t * 10;
        });
    }
    for (auto& th : ths) th.join();
    // every thread is gone: its agent merged into the global value
    EXPECT_EQ(a.get_value(), 8000);
    EXPECT_EQ(mx.get_value(), 70);
}

TEST(VarMore, reset_while_writers_run_loses_nothing) {
    Adder<int64_t> a;
    std::atomic<bool> stop{false};
    std::atomic<int64_t> written{0};
    std::vector<std::thread> ths;
    for (int t = 0; t < 4; ++t) {
        ths.emplace_back([&] {
            int64_t n = 0;
            while (!stop.load(std::memory_order_relaxed)) {
                a << 1;
                ++n;
            }
            written.fetch_add(n);
        });
    }
    int64_t collected = 0;
    for (int i = 0; i < 50; ++i) {
        collected += a.reset();
        usleep(1000);
    }
    stop = true;
    for (auto& th : ths) th.join();
    collected += a.reset();
    EXPECT_EQ(collected, written.load());
}

TEST(VarMore, many_reducers_on_one_thread) {
    std::vector<std::unique_ptr<Adder<int64_t>>> v;
    for (int i = 0; i < 300; ++i) v.emplace_back(new Adder<int64_t>);
    for (int i = 0; i < 300; ++i) *v[i] << i;
    int64_t sum = 0;
    for (int i = 0; i < 300; ++i) sum += v[i]->get_value();
    EXPECT_EQ(sum, 299 * 300 / 2);
    // destroying some and creating new ones reuses agent slots cleanly
    v.resize(100);
    for (int i = 0; i < 100; ++i) v.emplace_back(new Adder<int64_t>);
    for (int i = 100; i < 200; ++i) EXPECT_EQ(v[i]->get_value(), 0);
}

TEST(VarMore, int_recorder_counts_and_averages) {
    IntRecorder r;
    EXPECT_EQ(r.get_value().num, 0);
    EXPECT_EQ(r.get_value().get_average_int(), 0);
    for (int i = 1; i <= 100; ++i) r << i;
    const Stat s = r.get_value();
    EXPECT_EQ(s.num, 100);
    EXPECT_EQ(s.sum, 5050);
    EXPECT_TRUE(std::fabs(s.average() - 50.5) < 1e-9);
    EXPECT_EQ(describe(r), "50");
}

TEST(VarMore, int_recorder_from_many_threads) {
    IntRecorder r;
    std::vector<std::thread> ths;
    for (int t = 0; t < 6; ++t) {
        ths.emplace_back([&] {
            for (int i = 0; i < 500; ++i) r << 4;
        });
    }
    for (auto& th : ths) th.join();
    EXPECT_EQ(r.get_value().num, 3000);
    EXPECT_EQ(r.get_value().get_average_int(), 4);
}

TEST(VarMore, passive_status_reads_its_getter_every_time) {
    int x = 1;
    PassiveStatus<int> p([&] { return x; });
    EXPECT_EQ(p.get_value(), 1);
    x = 42;
    EXPECT_EQ(p.get_value(), 42);
    EXPECT_EQ(describe(p), "42");
    double d = 0;
    EXPECT_TRUE(p.get_number(&d));
    EXPECT_EQ(d, 42.0);
}

TEST(VarMore, passive_status_of_strings_is_not_numeric) {
    PassiveStatus<std::string> p([] { return std::string("hello"); });
    double d = 0;
    EXPECT_FALSE(p.get_number(&d));
    std::ostringstream q;
    p.describe(q, true);
    EXPECT_TRUE(has(q.str(), "\"hello\""));
    EXPECT_EQ(describe(p), "hello");
}

TEST(VarMore, status_set_and_get_across_threads) {
    var::Status<int64_t> s(7);
    EXPECT_EQ(s.get_value(), 7);
    std::thread th([&] { s.set_value(99); });
    th.join();
    EXPECT_EQ(s.get_value(), 99);
    var::Status<std::string> t("x");
    t.set_value("y z");
    EXPECT_EQ(t.get_value(), "y z");
}

TEST(VarMore, exposed_variable_found_by_name) {
    Adder<int64_t> a("var_more_exposed_adder");
    a << 3;
    EXPECT_EQ(Variable::describe_exposed("var_more_exposed_adder"), "3");
    EXPECT_TRUE(a.is_exposed());
    EXPECT_TRUE(a.hide());
    EXPECT_FALSE(a.is_exposed());
    EXPECT_EQ(Variable::describe_exposed("var_more_exposed_adder"), "");
}

TEST(VarMore, expose_as_joins_prefix_and_name) {
    Adder<int64_t> a("var_more", "pre fixed");
    std::vector<std::string> names;
    Variable::list_exposed(&names);
    EXPECT_TRUE(std::find(names.begin(), names.end(), "var_more_pre_fixed") != names.end());
}

TEST(VarMore, exposing_a_taken_name_fails) {
    Adder<int64_t> a("var_more_taken");
    Adder<int64_t> b;
    EXPECT_EQ(b.expose("var_more_taken"), -1);
    EXPECT_FALSE(b.is_exposed());
    a.hide();
    EXPECT_EQ(b.expose("var_more_taken"), 0);
}

TEST(VarMore, count_exposed_tracks_lifetimes) {
    const int before = Variable::count_exposed();
    {
        Adder<int64_t> a("var_more_count_a");
        Maxer<int64_t> b("var_more_count_b");
        EXPECT_EQ(Variable::count_exposed(), before + 2);
    }
    EXPECT_EQ(Variable::count_exposed(), before);
}

TEST(VarMore, prometheus_dump_lists_numeric_variables) {
    Adder<int64_t> a("var_more_prom_adder");
    a << 12;
    var::Status<std::string> s("var_more_prom_text", "abc");
    const std::string p = Variable::dump_prometheus();
    EXPECT_TRUE(has(p, "var_more_prom_adder 12"));
    EXPECT_FALSE(has(p, "var_more_prom_text"));
}

TEST(VarMore, multi_dimension_rejects_wrong_arity) {
    MultiDimension<Adder<int64_t>> md("var_more_md_arity", {"method", "code"});
    EXPECT_TRUE(md.get_stats({"only_one"}) == nullptr);
    EXPECT_TRUE(md.get_stats({"a", "b", "c"}) == nullptr);
    EXPECT_TRUE(md.get_stats({"a", "b"}) != nullptr);
    EXPECT_EQ(md.count_stats(), 1u);
}

TEST(VarMore, multi_dimension_same_labels_same_metric) {
    MultiDimension<Adder<int64_t>> md("var_more_md_same", {"k"});
    Adder<int64_t>* a = md.get_stats({"x"});
    Adder<int64_t>* b = md.get_stats({"x"});
    EXPECT_EQ(a, b);
    *a << 2;
    *b << 3;
    EXPECT_EQ(md.get_stats({"x"})->get_value(), 5);
    EXPECT_TRUE(md.has_stats({"x"}));
    EXPECT_FALSE(md.has_stats({"y"}));
}

TEST(VarMore, multi_dimension_renders_labels_escaped) {
    MultiDimension<Adder<int64_t>> md("var_more_md_render", {"path"});
    *md.get_stats({"a\"b\\c"}) << 4;
    const std::string d = describe(md);
    EXPECT_TRUE(has(d, "path=\"a\\\"b\\\\c\""));
    EXPECT_TRUE(has(d, "4"));
}

TEST(VarMore, multi_dimension_clear_and_list) {
    MultiDimension<Maxer<int64_t>> md("var_more_md_clear", {"a", "b"});
    md.get_stats({"1", "2"});
    md.get_stats({"3", "4"});
    std::vector<std::vector<std::string>> keys;
    md.list_stats(&keys);
    EXPECT_EQ(keys.size(), 2u);
    md.clear_stats();
    EXPECT_EQ(md.count_stats(), 0u);
    md.list_stats(&keys);
    EXPECT_TRUE(keys.empty());
}

TEST(VarMore, percentile_of_uniform_values_is_within_bands) {
    LatencyRecorder r(10);
    std::mt19937 rng(7);
    std::uniform_int_distribution<int> d(1, 10000);
    for (int i = 0; i < 20000; ++i) r << d(rng);
    const int64_t p50 = r.latency_percentile(0.5);
    const int64_t p99 = r.latency_percentile(0.99);
    EXPECT_GT(p50, 4000);
    EXPECT_LT(p50, 6000);
    EXPECT_GT(p99, 9300);
    EXPECT_LE(p99, 10000 * 11 / 10);
    EXPECT_LE(p50, p99);
}

TEST(VarMore, percentile_of_a_constant_is_the_constant) {
    LatencyRecorder r(10);
    for (int i = 0; i < 1000; ++i) r << 250;
    const int64_t p = r.latency_percentile(0.9);
    EXPECT_GE(p, 225);
    EXPECT_LE(p, 275);
}

TEST(VarMore, latency_recorder_counts_every_sample) {
    LatencyRecorder r(10);
    std::vector<std::thread> ths;
    for (int t = 0; t < 4; ++t) {
        ths.emplace_back([&] {
            for (int i = 0; i < 250; ++i) r << 100;
        });
    }
    for (auto& th : ths) th.join();
    EXPECT_EQ(r.count(), 1000);
}

TEST(VarMore, latency_recorder_percentiles_json_is_ordered) {
    LatencyRecorder r(10);
    for (int i = 1; i <= 1000; ++i) r << i;
    const std::string j = r.latency_percentiles_json();
    EXPECT_EQ(j.front(), '[');
    EXPECT_EQ(j.back(), ']');
    // the rendered percentiles never decrease
    std::vector<long> v;
    for (size_t i = 1; i < j.size();) {
        char* end = nullptr;
        const long x = strtol(j.c_str() + i, &end, 10);
        if (end == j.c_str() + i) {
            ++i;
            continue;
        }
        v.push_back(x);
        i = end - j.c_str();
    }
    EXPECT_GE(v.size(), 2u);
    for (size_t i = 1; i < v.size(); ++i) EXPECT_LE(v[i - 1], v[i]);
}

TEST(VarMore, latency_recorder_expose_and_hide) {
    LatencyRecorder r("var_more_lat", 10);
    r << 10;
    std::vector<std::string> names;
    Variable::list_exposed(&names);
    int found = 0;
    for (const std::string& n : names) found += n.rfind("var_more_lat", 0) == 0;
    EXPECT_GE(found, 3);  // latency, max, qps, count, percentiles...
    r.hide();
    Variable::list_exposed(&names);
    found = 0;
    for (const std::string& n : names) found += n.rfind("var_more_lat", 0) == 0;
    EXPECT_EQ(found, 0);
}
