// Fiber runtime depth, round 6 (spirit of the reference's
// bthread_timer_thread_unittest, bthread_key_unittest, bthread_cond_unittest,
// bthread_mutex_unittest, bthread_rwlock_unittest, bthread_countdown_event,
// bthread_fd_unittest and bthread_unittest): timer ordering and
// cancellation, fiber keys with destructors, condition variables with
// deadlines, mutex fairness under contention, rwlock exclusion, barriers,
// countdown events, fd waits, stop/yield/usleep semantics.
#include <fcntl.h>
#include <pthread.h>
#include <sys/epoll.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <mutex>
#include <thread>
#include <vector>

#include "base/time.h"
#include "fiber/fiber.h"
#include "fiber/sync.h"
#include "fiber/timer.h"
#include "tests/test.h"

using namespace mrpc;

namespace {
timespec after_us(int64_t us) {
    const int64_t t = realtime_us() + us;
    timespec ts;
    ts.tv_sec = t / 1000000;
    ts.tv_nsec = (t % 1000000) * 1000;
    return ts;
}

void wait_until(const std::function<bool()>& cond, int max_ms = 3000) {
    for (int i = 0; i < max_ms && !cond(); ++i) ::usleep(1000);
}
}  // namespace

TEST(FiberMore, timers_fire_in_deadline_order) {
    static std::mutex mu;
    static std::vector<int> order;
    order.clear();
    fiber::TimerId ids[5];
    const int delays[5] = {50000, 10000, 40000, 20000, 30000};
    static int tags[5] = {0, 1, 2, 3, 4};
    for (int i = 0; i < 5; ++i) {
        ASSERT_EQ(fiber::timer_add_us(&ids[i], delays[i],
                                      [](void* a) {
                                          std::lock_guard<std::mutex> g(mu);
                                          order.push_back(*static_cast<int*>(a));
                                      },
                                      &tags[i]),
                  0);
    }
    wait_until([] {
        std::lock_guard<std::mutex> g(mu);
        return order.size() == 5;
    });
    std::lock_guard<std::mutex> g(mu);
    ASSERT_EQ(order.size(), 5u);
    EXPECT_EQ(order[0], 1);
    EXPECT_EQ(order[1], 3);
    EXPECT_EQ(order[2], 4);
    EXPECT_EQ(order[3], 2);
    EXPECT_EQ(order[4], 0);
}

TEST(FiberMore, deleted_timer_never_fires) {
    static std::atomic<int> fired{0};
    fired = 0;
    fiber::TimerId id;
    ASSERT_EQ(fiber::timer_add_us(&id, 30000, [](void*) { fired.fetch_add(1); }, nullptr), 0);
    EXPECT_EQ(fiber::timer_del(id), 0);
    ::usleep(80000);
    EXPECT_EQ(fired.load(), 0);
    // a second delete of the same id reports that nothing was pending
    EXPECT_NE(fiber::timer_del(id), 0);
}

TEST(FiberMore, timer_in_the_past_fires_promptly) {
    static std::atomic<int64_t> fired_at{0};
    fired_at = 0;
    fiber::TimerId id;
    const int64_t t0 = monotonic_us();
    ASSERT_EQ(fiber::timer_add(&id, after_us(-100000), [](void*) { fired_at = monotonic_us(); }, nullptr), 0);
    wait_until([] { return fired_at.load() != 0; });
    EXPECT_GT(fired_at.load(), 0);
    EXPECT_LT(fired_at.load() - t0, 100000);
}

TEST(FiberMore, many_timers_all_fire_once) {
    static std::atomic<int> fired{0};
    fired = 0;
    for (int i = 0; i < 2000; ++i) {
        fiber::TimerId id;
        ASSERT_EQ(fiber::timer_add_us(&id, 1000 + (i % 50) * 100, [](void*) { fired.fetch_add(1); }, nullptr), 0);
    }
    wait_until([] { return fired.load() == 2000; });
    ::usleep(20000);
    EXPECT_EQ(fired.load(), 2000);
}

TEST(FiberMore, key_values_are_per_fiber) {
    fiber::FiberKey key;
    ASSERT_EQ(fiber::key_create(&key, nullptr), 0);
    std::atomic<int> ok{0};
    std::vector<fiber::fiber_t> ts(16);
    for (int i = 0; i < 16; ++i) {
        fiber::start(
            [&, i] {
                intptr_t mine = 1000 + i;
                fiber::setspecific(key, reinterpret_cast<void*>(mine));
                fiber::usleep(1000);  // other fibers run and set theirs meanwhile
                if (reinterpret_cast<intptr_t>(fiber::getspecific(key)) == mine) ok.fetch_add(1);
            },
            false, nullptr, &ts[i]);
    }
    for (auto t : ts) fiber::join(t, nullptr);
    EXPECT_EQ(ok.load(), 16);
    fiber::key_delete(key);
}

TEST(FiberMore, key_destructor_runs_at_fiber_exit) {
    static std::atomic<int> destroyed{0};
    destroyed = 0;
    fiber::FiberKey key;
    ASSERT_EQ(fiber::key_create(&key, [](void* p) {
                  delete static_cast<int*>(p);
                  destroyed.fetch_add(1);
              }),
              0);
    std::vector<fiber::fiber_t> ts(8);
    for (int i = 0; i < 8; ++i) {
        fiber::start([&] { fiber::setspecific(key, new int(5)); }, false, nullptr, &ts[i]);
    }
    for (auto t : ts) fiber::join(t, nullptr);
    wait_until([] { return destroyed.load() == 8; });
    EXPECT_EQ(destroyed.load(), 8);
    fiber::key_delete(key);
}

TEST(FiberMore, unset_key_reads_null) {
    fiber::FiberKey key;
    ASSERT_EQ(fiber::key_create(&key, nullptr), 0);
    std::atomic<int> null_seen{0};
    fiber::fiber_t t;
    fiber::start([&] { null_seen = fiber::getspecific(key) == nullptr; }, false, nullptr, &t);
    fiber::join(t, nullptr);
    EXPECT_EQ(null_seen.load(), 1);
    fiber::key_delete(key);
}

TEST(FiberMore, deleted_key_is_rejected) {
    fiber::FiberKey key;
    ASSERT_EQ(fiber::key_create(&key, nullptr), 0);
    ASSERT_EQ(fiber::key_delete(key), 0);
    std::atomic<int> rc{0};
    fiber::fiber_t t;
    fiber::start([&] { rc = fiber::setspecific(key, (void*)1); }, false, nullptr, &t);
    fiber::join(t, nullptr);
    EXPECT_NE(rc.load(), 0);
}

TEST(FiberMore, condition_wait_for_times_out) {
    fiber::Mutex m;
    fiber::ConditionVariable cv;
    std::atomic<int> rc{-7};
    std::atomic<int64_t> took{0};
    fiber::fiber_t t;
    fiber::start(
        [&] {
            m.lock();
            const int64_t t0 = monotonic_us();
            rc = cv.wait_for_us(m, 30000);
            took = monotonic_us() - t0;
            m.unlock();
        },
        false, nullptr, &t);
    fiber::join(t, nullptr);
    EXPECT_EQ(rc.load(), ETIMEDOUT);
    EXPECT_GE(took.load(), 25000);
}

TEST(FiberMore, condition_notify_one_wakes_one_waiter) {
    fiber::Mutex m;
    fiber::ConditionVariable cv;
    int ready = 0;
    std::atomic<int> woken{0};
    std::vector<fiber::fiber_t> ts(4);
    for (int i = 0; i < 4; ++i) {
        fiber::start(
            [&] {
                m.lock();
                while (ready == 0) cv.wait(m);
                --ready;
                woken.fetch_add(1);
                m.unlock();
            },
            false, nullptr, &ts[i]);
    }
    ::usleep(20000);
    for (int k = 1; k <= 4; ++k) {
        m.lock();
        ++ready;
        cv.notify_one();
        m.unlock();
        wait_until([&] { return woken.load() == k; }, 2000);
        EXPECT_EQ(woken.load(), k);
    }
    for (auto t : ts) fiber::join(t, nullptr);
}

TEST(FiberMore, condition_notify_all_wakes_everyone) {
    fiber::Mutex m;
    fiber::ConditionVariable cv;
    bool go = false;
    std::atomic<int> woken{0};
    std::vector<fiber::fiber_t> ts(10);
    for (int i = 0; i < 10; ++i) {
        fiber::start(
            [&] {
                m.lock();
                while (!go) cv.wait(m);
                m.unlock();
                woken.fetch_add(1);
            },
            false, nullptr, &ts[i]);
    }
    ::usleep(20000);
    m.lock();
    go = true;
    cv.notify_all();
    m.unlock();
    for (auto t : ts) fiber::join(t, nullptr);
    EXPECT_EQ(woken.load(), 10);
}

TEST(FiberMore, mutex_protects_a_counter_under_contention) {
    fiber::Mutex m;
    int64_t counter = 0;
    std::vector<fiber::fiber_t> ts(16);
    for (int i = 0; i < 16; ++i) {
        fiber::start(
            [&] {
                for (int k = 0; k < 2000; ++k) {
                    m.lock();
                    ++counter;
                    if (k % 200 == 0) fiber::yield();
                    m.unlock();
                }
            },
            false, nullptr, &ts[i]);
    }
    for (auto t : ts) fiber::join(t, nullptr);
    EXPECT_EQ(counter, 32000);
}

TEST(FiberMore, mutex_shared_by_pthreads_and_fibers) {
    fiber::Mutex m;
    int64_t counter = 0;
    std::vector<std::thread> ths;
    for (int i = 0; i < 3; ++i) {
        ths.emplace_back([&] {
            for (int k = 0; k < 3000; ++k) {
                fiber::LockGuard<fiber::Mutex> g(m);
                ++counter;
            }
        });
    }
    std::vector<fiber::fiber_t> ts(3);
    for (int i = 0; i < 3; ++i) {
        fiber::start(
            [&] {
                for (int k = 0; k < 3000; ++k) {
                    fiber::LockGuard<fiber::Mutex> g(m);
                    ++counter;
                }
            },
            false, nullptr, &ts[i]);
    }
    for (auto& th : ths) th.join();
    for (auto t : ts) fiber::join(t, nullptr);
    EXPECT_EQ(counter, 18000);
}

TEST(FiberMore, mutex_timed_lock_expires) {
    fiber::Mutex m;
    m.lock();
    std::atomic<int> got{-1};
    fiber::fiber_t t;
    fiber::start(
        [&] {
            const timespec ts = after_us(20000);
            got = m.timed_lock(&ts) ? 1 : 0;
        },
        false, nullptr, &t);
    fiber::join(t, nullptr);
    EXPECT_EQ(got.load(), 0);
    m.unlock();
    const timespec ts2 = after_us(20000);
    EXPECT_TRUE(m.timed_lock(&ts2));
    m.unlock();
}

TEST(FiberMore, rwlock_readers_share_writers_exclude) {
    fiber::RWLock rw;
    std::atomic<int> readers{0}, max_readers{0}, writer_overlap{0};
    std::atomic<bool> writing{false};
    std::vector<fiber::fiber_t> ts;
    for (int i = 0; i < 12; ++i) {
        fiber::fiber_t t;
        const bool writer = i % 4 == 0;
        fiber::start(
            [&, writer] {
                for (int k = 0; k < 200; ++k) {
                    if (writer) {
                        rw.wrlock();
                        if (readers.load() != 0 || writing.exchange(true)) writer_overlap.fetch_add(1);
                        fiber::yield();
                        writing = false;
                        rw.unlock();
                    } else {
                        rw.rdlock();
                        if (writing.load()) writer_overlap.fetch_add(1);
                        const int r = readers.fetch_add(1) + 1;
                        int m = max_readers.load();
                        while (r > m && !max_readers.compare_exchange_weak(m, r)) {
                        }
                        fiber::yield();
                        readers.fetch_sub(1);
                        rw.unlock_shared();
                    }
                }
            },
            false, nullptr, &t);
        ts.push_back(t);
    }
    for (auto t : ts) fiber::join(t, nullptr);
    EXPECT_EQ(writer_overlap.load(), 0);
    EXPECT_GE(max_readers.load(), 1);
}

TEST(FiberMore, rwlock_try_variants) {
    fiber::RWLock rw;
    EXPECT_TRUE(rw.try_rdlock());
    EXPECT_TRUE(rw.try_rdlock());
    EXPECT_FALSE(rw.try_wrlock());
    rw.unlock_shared();
    rw.unlock_shared();
    EXPECT_TRUE(rw.try_wrlock());
    EXPECT_FALSE(rw.try_rdlock());
    rw.unlock();
}

TEST(FiberMore, countdown_event_releases_at_zero) {
    fiber::CountdownEvent ev(3);
    std::atomic<int> passed{0};
    fiber::fiber_t t;
    fiber::start(
        [&] {
            ev.wait();
            passed = 1;
        },
        false, nullptr, &t);
    ev.signal();
    ev.signal();
    ::usleep(10000);
    EXPECT_EQ(passed.load(), 0);
    ev.signal();
    fiber::join(t, nullptr);
    EXPECT_EQ(passed.load(), 1);
    EXPECT_EQ(ev.count(), 0);
}

TEST(FiberMore, countdown_event_timed_wait_and_add_count) {
    fiber::CountdownEvent ev(1);
    ev.add_count(2);
    EXPECT_EQ(ev.count(), 3);
    const timespec ts = after_us(20000);
    EXPECT_EQ(ev.timed_wait(&ts), ETIMEDOUT);
    ev.signal(3);
    const timespec ts2 = after_us(20000);
    EXPECT_EQ(ev.timed_wait(&ts2), 0);
    ev.reset(2);
    EXPECT_EQ(ev.count(), 2);
}

TEST(FiberMore, fd_timedwait_times_out_and_sees_data) {
    int p[2];
    ASSERT_EQ(pipe(p), 0);
    fcntl(p[0], F_SETFL, fcntl(p[0], F_GETFL) | O_NONBLOCK);
    std::atomic<int> rc1{-7}, rc2{-7};
    fiber::fiber_t t;
    fiber::start(
        [&] {
            const timespec ts = after_us(20000);
            rc1 = fiber::fd_timedwait(p[0], EPOLLIN, &ts);
            const timespec ts2 = after_us(2000000);
            rc2 = fiber::fd_timedwait(p[0], EPOLLIN, &ts2);
        },
        false, nullptr, &t);
    ::usleep(60000);
    ASSERT_EQ(write(p[1], "z", 1), 1);
    fiber::join(t, nullptr);
    EXPECT_EQ(rc1.load(), -1);
    EXPECT_EQ(rc2.load(), 0);
    close(p[0]);
    close(p[1]);
}

TEST(FiberMore, usleep_sleeps_at_least_the_time) {
    std::atomic<int64_t> took{0};
    fiber::fiber_t t;
    fiber::start(
        [&] {
            const int64_t t0 = monotonic_us();
            fiber::usleep(15000);
            took = monotonic_us() - t0;
        },
        false, nullptr, &t);
    fiber::join(t, nullptr);
    EXPECT_GE(took.load(), 14000);
    EXPECT_LT(took.load(), 500000);
}

TEST(FiberMore, stop_wakes_a_sleeping_fiber_early) {
    std::atomic<int> rc{0};
    std::atomic<int64_t> took{0};
    fiber::fiber_t t;
    fiber::start(
        [&] {
            const int64_t t0 = monotonic_us();
            rc = fiber::usleep(5000000);
            took = monotonic_us() - t0;
        },
        false, nullptr, &t);
    ::usleep(20000);
    fiber::stop(t);
    fiber::join(t, nullptr);
    EXPECT_NE(rc.load(), 0);
    EXPECT_LT(took.load(), 2000000);
}

TEST(FiberMore, yield_lets_others_run) {
    std::atomic<int> turns{0};
    std::atomic<bool> stop{false};
    fiber::fiber_t a, b;
    fiber::start(
        [&] {
            while (!stop.load()) {
                turns.fetch_add(1);
                fiber::yield();
            }
        },
        false, nullptr, &a);
    fiber::start(
        [&] {
            for (int i = 0; i < 100; ++i) fiber::yield();
            stop = true;
        },
        false, nullptr, &b);
    fiber::join(b, nullptr);
    fiber::join(a, nullptr);
    EXPECT_GT(turns.load(), 0);
}

TEST(FiberMore, self_and_in_fiber_report_the_context) {
    EXPECT_FALSE(fiber::in_fiber());  // the test runs on a plain pthread
    std::atomic<int> inside{0};
    std::atomic<uint64_t> me{0};
    fiber::fiber_t t;
    fiber::start(
        [&] {
            inside = fiber::in_fiber() ? 1 : 0;
            me = fiber::self();
        },
        false, nullptr, &t);
    fiber::join(t, nullptr);
    EXPECT_EQ(inside.load(), 1);
    EXPECT_EQ(me.load(), (uint64_t)t);
}

TEST(FiberMore, thousands_of_short_fibers) {
    std::atomic<int> ran{0};
    std::vector<fiber::fiber_t> ts(5000);
    for (auto& t : ts) fiber::start([&] { ran.fetch_add(1); }, false, nullptr, &t);
    for (auto t : ts) fiber::join(t, nullptr);
    EXPECT_EQ(ran.load(), 5000);
}

TEST(FiberMore, urgent_start_runs_before_the_caller_continues) {
    std::atomic<int> seq{0}, child_at{-1}, parent_at{-1};
    fiber::fiber_t outer;
    fiber::start(
        [&] {
            fiber::fiber_t child;
            fiber::start([&] { child_at = seq.fetch_add(1); }, /*urgent=*/true, nullptr, &child);
            parent_at = seq.fetch_add(1);
            fiber::join(child, nullptr);
        },
        false, nullptr, &outer);
    fiber::join(outer, nullptr);
    EXPECT_EQ(child_at.load(), 0);
    EXPECT_EQ(parent_at.load(), 1);
}
