// CallId (the correlation id of every RPC attempt, fiber/call_id.h): version
// ranges, join before/after destruction, queued errors, about_to_destroy and
// range resets, from fibers and from plain pthreads. Behaviour parity with
// the reference's test/bthread_id_unittest.cpp (join_after_destroy,
// join_before_destroy, error_is_destroy[_ranged], doubly_destroy,
// many_error, reset_range, about_to_destroy_{before,during}_locking,
// about_to_destroy_cancelled, error_with_descriptions).
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "base/time.h"
#include "fiber/call_id.h"
#include "fiber/fiber.h"
#include "tests/test.h"

using namespace mrpc;
using namespace mrpc::fiber;

namespace {

struct ErrLog {
    std::mutex mu;
    std::vector<int> codes;
    std::vector<std::string> texts;
    bool destroy_on_stop = true;
};

// Records the error; ESTOP destroys the id, anything else just unlocks.
int log_error(CallId id, void* data, int code, const std::string& text) {
    ErrLog* l = static_cast<ErrLog*>(data);
    {
        std::lock_guard<std::mutex> g(l->mu);
        l->codes.push_back(code);
        l->texts.push_back(text);
    }
    if (code == ESTOP && l->destroy_on_stop) return call_id_unlock_and_destroy(id);
    return call_id_unlock(id);
}

}  // namespace

TEST(CallIdRange, join_after_destroy) {
    CallId id;
    ASSERT_EQ(call_id_create(&id, nullptr, nullptr), 0);
    EXPECT_TRUE(call_id_exists(id));
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    ASSERT_EQ(call_id_unlock_and_destroy(id), 0);
    EXPECT_FALSE(call_id_exists(id));
    EXPECT_EQ(call_id_join(id), 0);  // returns at once
    EXPECT_EQ(call_id_lock(id, nullptr), EINVAL);
    EXPECT_EQ(call_id_error(id, EINVAL), EINVAL);
}

TEST(CallIdRange, join_before_destroy_from_fibers_and_pthreads) {
    CallId id;
    ASSERT_EQ(call_id_create(&id, nullptr, nullptr), 0);
    std::atomic<int> joined{0};
    std::vector<fiber_t> fibers(4);
    for (auto& f : fibers) start([&] { call_id_join(id); joined.fetch_add(1); }, false, nullptr, &f);
    std::vector<std::thread> threads;
    for (int i = 0; i < 2; ++i) threads.emplace_back([&] { call_id_join(id); joined.fetch_add(1); });
    ::usleep(20000);
    EXPECT_EQ(joined.load(), 0);
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    ::usleep(5000);
    EXPECT_EQ(joined.load(), 0);  // locked is not destroyed
    ASSERT_EQ(call_id_unlock_and_destroy(id), 0);
    for (auto f : fibers) join(f);
    for (auto& t : threads) t.join();
    EXPECT_EQ(joined.load(), 6);
}

TEST(CallIdRange, default_error_destroys_every_version_of_the_range) {
    CallId id;
    ASSERT_EQ(call_id_create_ranged(&id, nullptr, nullptr, 4), 0);
    for (int v = 0; v < 4; ++v) EXPECT_TRUE(call_id_exists(call_id_with_version(id, v)));
    EXPECT_FALSE(call_id_exists(call_id_with_version(id, 4)));  // past the range
    ASSERT_EQ(call_id_error(call_id_with_version(id, 2), ECANCELED), 0);
    for (int v = 0; v < 4; ++v) EXPECT_FALSE(call_id_exists(call_id_with_version(id, v)));
    EXPECT_EQ(call_id_join(id), 0);
}

TEST(CallIdRange, doubly_destroy_and_unlock_of_unlocked) {
    CallId id;
    ASSERT_EQ(call_id_create(&id, nullptr, nullptr), 0);
    EXPECT_EQ(call_id_unlock(id), EPERM);              // not locked
    EXPECT_EQ(call_id_unlock_and_destroy(id), EPERM);  // not locked either
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    ASSERT_EQ(call_id_unlock_and_destroy(id), 0);
    EXPECT_EQ(call_id_unlock_and_destroy(id), EINVAL);
    EXPECT_EQ(call_id_cancel(id), EINVAL);
}

TEST(CallIdRange, stale_id_of_a_reused_slot_is_rejected) {
    CallId a;
    ASSERT_EQ(call_id_create(&a, nullptr, nullptr), 0);
    ASSERT_EQ(call_id_cancel(a), 0);  // never locked: destroyed directly
    // the slot comes back with versions past every one handed out before
    CallId b;
    ASSERT_EQ(call_id_create_ranged(&b, nullptr, nullptr, 3), 0);
    EXPECT_NE(a.value, b.value);
    EXPECT_EQ(call_id_lock(a, nullptr), EINVAL);
    EXPECT_EQ(call_id_error(a, 1), EINVAL);
    ASSERT_EQ(call_id_lock(b, nullptr), 0);
    ASSERT_EQ(call_id_unlock_and_destroy(b), 0);
}

TEST(CallIdRange, errors_queued_while_locked_run_in_order_at_unlock) {
    ErrLog log;
    CallId id;
    ASSERT_EQ(call_id_create_ranged(&id, &log, log_error, 2), 0);
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    // errors from pthreads and fibers while the owner holds the lock
    const int kPerThread = 25;
    std::vector<std::thread> threads;
    for (int t = 0; t < 4; ++t) {
        threads.emplace_back([&, t] {
            for (int i = 0; i < kPerThread; ++i) call_id_error(call_id_with_version(id, i % 2), 1000 + t);
        });
    }
    for (auto& t : threads) t.join();
    {
        std::lock_guard<std::mutex> g(log.mu);
        EXPECT_TRUE(log.codes.empty());  // nothing runs while locked
    }
    // unlock hands the lock to the first queued handler, whose unlock runs
    // the next one, ... until the queue is empty
    ASSERT_EQ(call_id_unlock(id), 0);
    {
        std::lock_guard<std::mutex> g(log.mu);
        EXPECT_EQ((int)log.codes.size(), 4 * kPerThread);
    }
    EXPECT_TRUE(call_id_exists(id));
    // the id is usable again, and an ESTOP destroys it
    ASSERT_EQ(call_id_error(id, ESTOP, "stop"), 0);
    EXPECT_FALSE(call_id_exists(id));
    std::lock_guard<std::mutex> g(log.mu);
    EXPECT_EQ(log.codes.back(), ESTOP);
    EXPECT_EQ(log.texts.back(), "stop");
}

TEST(CallIdRange, destroy_drops_queued_errors) {
    ErrLog log;
    CallId id;
    ASSERT_EQ(call_id_create(&id, &log, log_error), 0);
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    ASSERT_EQ(call_id_error(id, 7), 0);
    ASSERT_EQ(call_id_error(id, 8), 0);
    ASSERT_EQ(call_id_unlock_and_destroy(id), 0);
    std::lock_guard<std::mutex> g(log.mu);
    EXPECT_TRUE(log.codes.empty());
}

TEST(CallIdRange, lock_and_reset_range_extends_the_versions) {
    CallId id;
    ASSERT_EQ(call_id_create(&id, nullptr, nullptr), 0);
    EXPECT_FALSE(call_id_exists(call_id_with_version(id, 5)));
    void* d = nullptr;
    ASSERT_EQ(call_id_lock_and_reset_range(id, &d, 1000), 0);
    EXPECT_TRUE(call_id_exists(call_id_with_version(id, 5)));
    EXPECT_TRUE(call_id_exists(call_id_with_version(id, 999)));
    EXPECT_FALSE(call_id_exists(call_id_with_version(id, 1000)));
    ASSERT_EQ(call_id_unlock(call_id_with_version(id, 999)), 0);  // any version of the range unlocks
    // a smaller range later never shrinks what was handed out
    ASSERT_EQ(call_id_lock_and_reset_range(id, &d, 300), 0);
    EXPECT_TRUE(call_id_exists(call_id_with_version(id, 999)));
    EXPECT_EQ(call_id_lock_and_reset_range(id, &d, 0), EINVAL);
    EXPECT_EQ(call_id_lock_and_reset_range(id, &d, 5000), EINVAL);
    ASSERT_EQ(call_id_unlock_and_destroy(call_id_with_version(id, 3)), 0);
    EXPECT_FALSE(call_id_exists(call_id_with_version(id, 999)));
}

TEST(CallIdRange, about_to_destroy_before_locking) {
    CallId id;
    ASSERT_EQ(call_id_create(&id, nullptr, nullptr), 0);
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    ASSERT_EQ(call_id_about_to_destroy(id), 0);
    std::atomic<int> eperm{0};
    std::thread th([&] { eperm.fetch_add(call_id_lock(id, nullptr) == EPERM); });
    fiber_t f;
    start([&] { eperm.fetch_add(call_id_lock(id, nullptr) == EPERM); }, false, nullptr, &f);
    th.join();
    join(f);
    EXPECT_EQ(eperm.load(), 2);
    EXPECT_EQ(call_id_error(id, 1), EPERM);  // errors are refused too
    ASSERT_EQ(call_id_unlock_and_destroy(id), 0);
}

TEST(CallIdRange, about_to_destroy_cancelled_by_unlock) {
    CallId id;
    ASSERT_EQ(call_id_create(&id, nullptr, nullptr), 0);
    EXPECT_EQ(call_id_about_to_destroy(id), EPERM);  // must hold the lock
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    ASSERT_EQ(call_id_about_to_destroy(id), 0);
    ASSERT_EQ(call_id_unlock(id), 0);  // changed our mind
    std::atomic<int> ok{0};
    std::thread th([&] {
        if (call_id_lock(id, nullptr) == 0) ok.fetch_add(call_id_unlock(id) == 0);
    });
    fiber_t f;
    start([&] {
        if (call_id_lock(id, nullptr) == 0) ok.fetch_add(call_id_unlock(id) == 0);
    }, false, nullptr, &f);
    th.join();
    join(f);
    EXPECT_EQ(ok.load(), 2);
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    ASSERT_EQ(call_id_unlock_and_destroy(id), 0);
}

TEST(CallIdRange, about_to_destroy_wakes_blocked_lockers) {
    CallId id;
    ASSERT_EQ(call_id_create(&id, nullptr, nullptr), 0);
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    std::atomic<int> done{0}, eperm{0};
    std::thread th([&] {
        eperm.fetch_add(call_id_lock(id, nullptr) == EPERM);
        done.fetch_add(1);
    });
    fiber_t f;
    start([&] {
        eperm.fetch_add(call_id_lock(id, nullptr) == EPERM);
        done.fetch_add(1);
    }, false, nullptr, &f);
    ::usleep(50000);
    EXPECT_EQ(done.load(), 0);  // both wait for the lock
    ASSERT_EQ(call_id_about_to_destroy(id), 0);
    th.join();
    join(f);
    EXPECT_EQ(eperm.load(), 2);
    ASSERT_EQ(call_id_unlock_and_destroy(id), 0);
}

TEST(CallIdRange, trylock_and_error_text) {
    ErrLog log;
    log.destroy_on_stop = false;
    CallId id;
    ASSERT_EQ(call_id_create(&id, &log, log_error), 0);
    void* d = nullptr;
    ASSERT_EQ(call_id_trylock(id, &d), 0);
    EXPECT_EQ(d, (void*)&log);
    EXPECT_EQ(call_id_trylock(id, &d), EBUSY);
    ASSERT_EQ(call_id_unlock(id), 0);
    // handled in place (unlocked id): the text reaches the handler as given
    ASSERT_EQ(call_id_error(id, ECONNREFUSED, "connection refused by 10.0.0.1:80"), 0);
    ASSERT_EQ(call_id_error(id, EINTR), 0);
    {
        std::lock_guard<std::mutex> g(log.mu);
        ASSERT_EQ(log.codes.size(), 2u);
        EXPECT_EQ(log.codes[0], ECONNREFUSED);
        EXPECT_EQ(log.texts[0], "connection refused by 10.0.0.1:80");
        EXPECT_EQ(log.texts[1], "");
    }
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    ASSERT_EQ(call_id_unlock_and_destroy(id), 0);
}

TEST(CallIdRange, contended_lock_from_pthreads_and_fibers) {
    CallId id;
    int64_t counter = 0;
    ASSERT_EQ(call_id_create(&id, &counter, nullptr), 0);
    auto work = [id] {
        for (int i = 0; i < 500; ++i) {
            void* d;
            if (call_id_lock(id, &d) == 0) {
                ++*static_cast<int64_t*>(d);
                call_id_unlock(id);
            }
        }
    };
    std::vector<std::thread> threads;
    for (int i = 0; i < 4; ++i) threads.emplace_back(work);
    std::vector<fiber_t> fibers(8);
    for (auto& f : fibers) start(work, false, nullptr, &f);
    for (auto& t : threads) t.join();
    for (auto f : fibers) join(f);
    EXPECT_EQ(counter, 12 * 500);
    ASSERT_EQ(call_id_lock(id, nullptr), 0);
    ASSERT_EQ(call_id_unlock_and_destroy(id), 0);
}
