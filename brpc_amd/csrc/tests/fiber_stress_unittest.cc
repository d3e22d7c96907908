// Fiber runtime under load (spirit of the reference's
// test/bthread_ping_pong_unittest.cpp, bthread_cond_bug_unittest.cpp,
// bthread_setconcurrency_unittest.cpp, bthread_mutex_unittest.cpp's
// contention cases and bthread_countdown_event_unittest.cpp): strict
// alternation over two butexes, broadcast storms with predicates, a counter
// under heavy mutex contention, many signalers of one countdown, thousands
// of joins, and concurrency that only grows.
#include <unistd.h>

#include <atomic>
#include <memory>
#include <thread>
#include <vector>

#include "base/time.h"
#include "fiber/butex.h"
#include "fiber/fiber.h"
#include "fiber/sync.h"
#include "tests/test.h"

using namespace mrpc;
using namespace mrpc::fiber;

TEST(FiberStress, ping_pong_alternates_strictly) {
    // two fibers hand a token back and forth through two butexes; each
    // side checks it only ever sees its own turn
    struct PP {
        std::atomic<int>* ping = butex_create();
        std::atomic<int>* pong = butex_create();
        std::atomic<int> turn{0};  // even: A, odd: B
        std::atomic<int> bad{0};
        int rounds = 20000;
    };
    auto* pp = new PP;
    pp->ping->store(0);
    pp->pong->store(0);
    auto side = [pp](bool a) {
        std::atomic<int>* mine = a ? pp->ping : pp->pong;
        std::atomic<int>* other = a ? pp->pong : pp->ping;
        for (int i = 0; i < pp->rounds; ++i) {
            for (;;) {
                const int seen = mine->load(std::memory_order_acquire);
                if ((pp->turn.load() & 1) == (a ? 0 : 1)) break;
                butex_wait(mine, seen);  // returns at once if `mine` moved meanwhile
            }
            if ((pp->turn.load() & 1) != (a ? 0 : 1)) pp->bad.fetch_add(1);
            pp->turn.fetch_add(1);
            other->fetch_add(1, std::memory_order_release);
            butex_wake(other);
        }
    };
    fiber_t ta, tb;
    ASSERT_EQ(start([&] { side(true); }, false, nullptr, &ta), 0);
    ASSERT_EQ(start([&] { side(false); }, false, nullptr, &tb), 0);
    join(ta);
    join(tb);
    EXPECT_EQ(pp->turn.load(), 2 * pp->rounds);
    EXPECT_EQ(pp->bad.load(), 0);
    butex_destroy(pp->ping);
    butex_destroy(pp->pong);
    delete pp;
}

TEST(FiberStress, broadcast_storm_loses_no_wakeup) {
    // 64 waiters each wait for the generation to pass their target; the
    // producer bumps it 200 times with notify_all; everyone finishes
    Mutex mu;
    ConditionVariable cv;
    int generation = 0;
    std::atomic<int> done{0};
    std::vector<fiber_t> ids(64);
    for (int w = 0; w < 64; ++w) {
        const int target = 50 + (w * 37) % 150;
        ASSERT_EQ(start([&, target] {
                      mu.lock();
                      while (generation < target) cv.wait(mu);
                      mu.unlock();
                      done.fetch_add(1);
                  },
                        false, nullptr, &ids[w]),
                  0);
    }
    for (int g = 0; g < 200; ++g) {
        mu.lock();
        ++generation;
        cv.notify_all();
        mu.unlock();
        if (g % 20 == 0) fiber::usleep(200);
    }
    for (fiber_t t : ids) join(t);
    EXPECT_EQ(done.load(), 64);
}

TEST(FiberStress, mutex_counter_under_contention) {
    Mutex mu;
    int64_t counter = 0;
    std::vector<fiber_t> ids(500);
    for (auto& t : ids) {
        ASSERT_EQ(start([&] {
                      for (int i = 0; i < 200; ++i) {
                          mu.lock();
                          ++counter;
                          if (i % 50 == 0) fiber::usleep(10);  // hold across a park now and then
                          mu.unlock();
                      }
                  },
                        false, nullptr, &t),
                  0);
    }
    // pthreads contend on the same mutex
    std::vector<std::thread> ths;
    for (int p = 0; p < 3; ++p) {
        ths.emplace_back([&] {
            for (int i = 0; i < 5000; ++i) {
                mu.lock();
                ++counter;
                mu.unlock();
            }
        });
    }
    for (fiber_t t : ids) join(t);
    for (auto& th : ths) th.join();
    EXPECT_EQ(counter, 500 * 200 + 3 * 5000);
}

TEST(FiberStress, countdown_with_many_signalers) {
    CountdownEvent ev(300);
    std::atomic<int> signaled{0};
    for (int i = 0; i < 300; ++i) {
        ASSERT_EQ(start([&, i] {
                      if (i % 7 == 0) fiber::usleep(100 + i);
                      signaled.fetch_add(1);
                      ev.signal();
                  }),
                  0);
    }
    EXPECT_EQ(ev.wait(), 0);
    EXPECT_EQ(signaled.load(), 300);
    EXPECT_EQ(ev.count(), 0);
    // reset and reuse, with a deadline that passes first
    ev.reset(2);
    ev.signal();
    const timespec soon = realtime_after_us(20000);
    EXPECT_NE(ev.timed_wait(&soon), 0);
    ev.signal();
    EXPECT_EQ(ev.wait(), 0);
}

TEST(FiberStress, thousands_of_fibers_join) {
    std::atomic<int> ran{0};
    std::vector<fiber_t> ids(3000);
    for (size_t i = 0; i < ids.size(); ++i) {
        ASSERT_EQ(start([&ran, i] {
                      if (i % 100 == 0) fiber::usleep(1000);
                      ran.fetch_add(1);
                  },
                        (i % 3) == 0, nullptr, &ids[i]),
                  0);
    }
    for (fiber_t t : ids) EXPECT_EQ(join(t), 0);
    EXPECT_EQ(ran.load(), 3000);
    for (size_t i = 0; i < ids.size(); i += 500) EXPECT_FALSE(exists(ids[i]));
}

TEST(FiberStress, concurrency_only_grows) {
    const int n = get_concurrency();
    EXPECT_GT(n, 0);
    EXPECT_EQ(set_concurrency(n + 2), 0);
    EXPECT_GE(get_concurrency(), n + 2);
    EXPECT_NE(set_concurrency(1), 0);  // cannot shrink
    EXPECT_GE(get_concurrency(), n + 2);
    // the new workers take work: 64 fibers that all sleep at once finish
    // in about one sleep, not 64
    std::vector<fiber_t> ids(64);
    const int64_t t0 = monotonic_us();
    for (auto& t : ids) ASSERT_EQ(start([] { fiber::usleep(20000); }, false, nullptr, &t), 0);
    for (fiber_t t : ids) join(t);
    EXPECT_LT(monotonic_us() - t0, 1000000);
}
