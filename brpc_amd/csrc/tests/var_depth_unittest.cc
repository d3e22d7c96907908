// Metrics depth (spirit of the reference's test/bvar_variable_unittest.cpp,
// bvar_reducer_unittest.cpp, bvar_recorder_unittest.cpp,
// bvar_window_unittest.cpp): exposure naming and uniqueness, dump filters,
// reducer reset semantics across threads, recorders, windows over a live
// sampler, quoting and the Prometheus text.
#include <unistd.h>

#include <sstream>
#include <thread>
#include <vector>

#include "var/var.h"
#include "tests/test.h"

using namespace mrpc;
using namespace mrpc::var;

TEST(VarDepth, expose_normalizes_and_names_are_unique) {
    const int before = Variable::count_exposed();
    Adder<int> a;
    EXPECT_EQ(a.expose("depth one.two-three"), 0);
    EXPECT_EQ(a.name(), "depth_one_two_three");
    EXPECT_EQ(Variable::count_exposed(), before + 1);
    Adder<int> b;
    EXPECT_EQ(b.expose("depth_one_two_three"), -1);  // taken
    EXPECT_FALSE(b.is_exposed());
    EXPECT_EQ(b.expose_as("depth", "prefixed"), 0);
    EXPECT_EQ(b.name(), "depth_prefixed");
    EXPECT_TRUE(a.hide());
    EXPECT_FALSE(a.is_exposed());
    EXPECT_EQ(b.expose("depth one.two-three"), 0);  // free again once hidden
    EXPECT_EQ(Variable::count_exposed(), before + 1);
    EXPECT_EQ(Variable::describe_exposed("no_such_variable_here"), "");
    std::ostringstream os;
    EXPECT_EQ(Variable::describe_exposed("no_such_variable_here", os), -1);
}

TEST(VarDepth, destroyed_variables_leave_the_registry) {
    const int before = Variable::count_exposed();
    {
        Adder<int64_t> a("depth_scoped_adder");
        Maxer<int64_t> m("depth_scoped_maxer");
        EXPECT_EQ(Variable::count_exposed(), before + 2);
    }
    EXPECT_EQ(Variable::count_exposed(), before);
    std::vector<std::string> names;
    Variable::list_exposed(&names);
    for (const std::string& n : names) EXPECT_TRUE(n.compare(0, 12, "depth_scoped") != 0);
}

TEST(VarDepth, dump_filters_wildcards_and_alternatives) {
    var::Status<int> s1("depth_fa_x1", 1);
    var::Status<int> s2("depth_fa_x22", 2);
    var::Status<int> s3("depth_fb_y", 3);
    std::vector<std::pair<std::string, std::string>> out;
    Variable::dump_exposed(&out, "depth_fa_x?");
    ASSERT_EQ(out.size(), 1u);
    EXPECT_EQ(out[0].first, "depth_fa_x1");
    out.clear();
    Variable::dump_exposed(&out, "depth_fa_*");
    EXPECT_EQ(out.size(), 2u);
    out.clear();
    Variable::dump_exposed(&out, "depth_fa_x1;depth_fb_*");
    ASSERT_EQ(out.size(), 2u);
    EXPECT_EQ(out[1].second, "3");
    out.clear();
    Variable::dump_exposed(&out, "depth_nothing_*");
    EXPECT_TRUE(out.empty());
}

TEST(VarDepth, reducer_reset_collects_every_thread) {
    Adder<int64_t> a;
    Maxer<int64_t> mx;
    Miner<int64_t> mn;
    std::vector<std::thread> ths;
    for (int t = 0; t < 6; ++t) {
        ths.emplace_back([&, t] {
            for (int i = 0; i < 10000; ++i) {
                a << 2;
                mx << (int64_t)t * 1000 + i;
                mn << -(int64_t)t * 1000 - i;
            }
        });
    }
    for (auto& th : ths) th.join();
    EXPECT_EQ(a.get_value(), 120000);
    EXPECT_EQ(mx.get_value(), 5 * 1000 + 9999);
    EXPECT_EQ(mn.get_value(), -(5 * 1000 + 9999));
    EXPECT_EQ(a.reset(), 120000);
    EXPECT_EQ(a.get_value(), 0);
    // live threads' agents are reset too
    std::atomic<int> phase{0};
    std::thread live([&] {
        a << 5;
        phase = 1;
        while (phase.load() != 2) usleep(100);
        a << 7;
        phase = 3;
    });
    while (phase.load() != 1) usleep(100);
    EXPECT_EQ(a.reset(), 5);
    phase = 2;
    while (phase.load() != 3) usleep(100);
    live.join();
    EXPECT_EQ(a.get_value(), 7);
}

TEST(VarDepth, int_recorder_average_and_negative_values) {
    IntRecorder r("depth_recorder");
    for (int i = -50; i <= 150; ++i) r << i;
    const Stat s = r.get_value();
    EXPECT_EQ(s.num, 201);
    EXPECT_EQ(s.sum, 201 * 50);
    EXPECT_EQ(s.get_average_int(), 50);
    EXPECT_EQ(Variable::describe_exposed("depth_recorder"), "50");
    IntRecorder empty;
    EXPECT_EQ(empty.get_value().average(), 0.0);
}

TEST(VarDepth, status_quoting_and_prometheus_text) {
    var::Status<std::string> s("depth_status_text", "ready");
    std::ostringstream q, plain;
    Variable::describe_exposed("depth_status_text", q, /*quote_string=*/true);
    Variable::describe_exposed("depth_status_text", plain, false);
    EXPECT_EQ(q.str(), "\"ready\"");
    EXPECT_EQ(plain.str(), "ready");
    s.set_value("busy");
    EXPECT_EQ(s.get_value(), "busy");
    Adder<int64_t> n("depth_prom_counter");
    n << 41 << 1;
    PassiveStatus<double> d("depth_prom_ratio", [] { return 0.25; });
    const std::string prom = Variable::dump_prometheus();
    EXPECT_TRUE(prom.find("depth_prom_counter 42") != std::string::npos);
    EXPECT_TRUE(prom.find("depth_prom_ratio 0.25") != std::string::npos);
    EXPECT_TRUE(prom.find("depth_status_text") == std::string::npos);  // not numeric
}

TEST(VarDepth, window_and_per_second_follow_the_sampler) {
    Adder<int64_t> a;
    Window<Adder<int64_t>> w("depth_window", &a, 2);
    PerSecond<Adder<int64_t>> ps("depth_per_second", &a, 2);
    Maxer<int64_t> mx;
    Window<Maxer<int64_t>> wm(&mx, 2);
    EXPECT_EQ(wm.get_value(), 0);  // identity shows as 0
    // ~1000/s for about 2.5 s
    for (int i = 0; i < 25; ++i) {
        a << 100;
        mx << i;
        usleep(100000);
    }
    const int64_t wv = w.get_value();
    EXPECT_GE(wv, 1000);  // 2 s of samples, loose bounds for a loaded host
    EXPECT_LE(wv, 2600);
    const double rate = ps.get_value();
    EXPECT_GE(rate, 400.0);
    EXPECT_LE(rate, 1600.0);
    EXPECT_GE(wm.get_value(), 10);
    EXPECT_LE(wm.get_value(), 24);
    EXPECT_TRUE(Variable::series_exposed("depth_window").size() > 2);
}

TEST(VarDepth, latency_recorder_renders_as_prometheus_summary) {
    LatencyRecorder lr;
    lr.expose("depth_summary_rec");
    for (int i = 1; i <= 1000; ++i) lr << i;
    const std::string prom = Variable::dump_prometheus();
    EXPECT_TRUE(prom.find("# TYPE depth_summary_rec summary\n") != std::string::npos);
    EXPECT_TRUE(prom.find("depth_summary_rec{quantile=\"0.8\"} ") != std::string::npos);
    EXPECT_TRUE(prom.find("depth_summary_rec{quantile=\"0.9999\"} ") != std::string::npos);
    EXPECT_TRUE(prom.find("depth_summary_rec{quantile=\"1\"} ") != std::string::npos);
    EXPECT_TRUE(prom.find("depth_summary_rec_count 1000\n") != std::string::npos);
    EXPECT_TRUE(prom.find("depth_summary_rec_sum ") != std::string::npos);
    // members of the summary are not repeated as gauges; qps stays one
    EXPECT_TRUE(prom.find("# TYPE depth_summary_rec_latency_80 gauge") == std::string::npos);
    EXPECT_TRUE(prom.find("# TYPE depth_summary_rec_count gauge") == std::string::npos);
    EXPECT_TRUE(prom.find("# TYPE depth_summary_rec_qps gauge") != std::string::npos);
    // exactly one summary header
    const size_t a = prom.find("# TYPE depth_summary_rec summary");
    EXPECT_EQ(prom.find("# TYPE depth_summary_rec summary", a + 1), std::string::npos);
    // a plain variable ending in _count is still a gauge
    Adder<int64_t> c("depth_lonely_count");
    c << 3;
    EXPECT_TRUE(Variable::dump_prometheus().find("depth_lonely_count 3\n") != std::string::npos);
}
