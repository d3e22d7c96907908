// Minimal gtest-like harness for the native unit tests (gtest is not
// available in this environment). Tests are registered with TEST(suite,
// name); main() runs those matching --filter=<substring>[,<substring>...].
// pytest drives the binary per suite (tests/test_native_unittests.py).
#pragma once

#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <sstream>
#include <string>
#include <vector>

namespace mtest {

// Wall-clock bounds of timing tests are multiplied by this under the
// sanitizers (TSan runs code 5-15x slower and serialises on its shadow)
#if defined(__SANITIZE_THREAD__) || defined(__SANITIZE_ADDRESS__)
constexpr int kSlowdown = 20;
#else
constexpr int kSlowdown = 1;
#endif

struct TestCase {
    const char* suite;
    const char* name;
    void (*fn)();
};

std::vector<TestCase>& registry();
extern int g_failures_in_current;

struct Registrar {
    Registrar(const char* s, const char* n, void (*f)()) { registry().push_back(TestCase{s, n, f}); }
};

template <typename A, typename B>
std::string fmt2(const A& a, const B& b) {
    std::ostringstream os;
    os << a << " vs " << b;
    return os.str();
}

void report_failure(const char* file, int line, const std::string& msg);

}  // namespace mtest

#define TEST(suite, name)                                                              \
    static void mtest_##suite##_##name();                                              \
    static mtest::Registrar mtest_reg_##suite##_##name(#suite, #name, mtest_##suite##_##name); \
    static void mtest_##suite##_##name()

#define MTEST_CHECK_(cond, msg, on_fail)                                  \
    do {                                                                  \
        if (!(cond)) {                                                    \
            mtest::report_failure(__FILE__, __LINE__, msg);               \
            on_fail;                                                      \
        }                                                                 \
    } while (0)

#define EXPECT_TRUE(c) MTEST_CHECK_((c), "EXPECT_TRUE(" #c ")", (void)0)
#define EXPECT_FALSE(c) MTEST_CHECK_(!(c), "EXPECT_FALSE(" #c ")", (void)0)
#define ASSERT_TRUE(c) MTEST_CHECK_((c), "ASSERT_TRUE(" #c ")", return)
// with a context message (a std::string expression)
#define EXPECT_TRUE_M(c, m) MTEST_CHECK_((c), std::string("EXPECT_TRUE(" #c ") ") + (m), (void)0)
#define EXPECT_FALSE_M(c, m) MTEST_CHECK_(!(c), std::string("EXPECT_FALSE(" #c ") ") + (m), (void)0)
#define ASSERT_TRUE_M(c, m) MTEST_CHECK_((c), std::string("ASSERT_TRUE(" #c ") ") + (m), return)
#define ASSERT_FALSE(c) MTEST_CHECK_(!(c), "ASSERT_FALSE(" #c ")", return)
#define MTEST_CMP_(a, b, op, on_fail) \
    MTEST_CHECK_(((a)op(b)), std::string(#a " " #op " " #b " : ") + mtest::fmt2((a), (b)), on_fail)
#define EXPECT_EQ(a, b) MTEST_CMP_(a, b, ==, (void)0)
#define EXPECT_NE(a, b) MTEST_CMP_(a, b, !=, (void)0)
#define EXPECT_LT(a, b) MTEST_CMP_(a, b, <, (void)0)
#define EXPECT_LE(a, b) MTEST_CMP_(a, b, <=, (void)0)
#define EXPECT_GT(a, b) MTEST_CMP_(a, b, >, (void)0)
#define EXPECT_GE(a, b) MTEST_CMP_(a, b, >=, (void)0)
#define ASSERT_EQ(a, b) MTEST_CMP_(a, b, ==, return)
#define ASSERT_NE(a, b) MTEST_CMP_(a, b, !=, return)
#define ASSERT_LT(a, b) MTEST_CMP_(a, b, <, return)
#define ASSERT_LE(a, b) MTEST_CMP_(a, b, <=, return)
#define ASSERT_GT(a, b) MTEST_CMP_(a, b, >, return)
#define ASSERT_GE(a, b) MTEST_CMP_(a, b, >=, return)
#define EXPECT_NEAR(a, b, eps) \
    MTEST_CHECK_(std::fabs((double)(a) - (double)(b)) <= (eps), "EXPECT_NEAR(" #a ", " #b ") " + mtest::fmt2((a), (b)), (void)0)
