// Fiber synchronization primitives, one behaviour per case (spirit of the
// reference's test/bthread_mutex_unittest.cpp, bthread_cond_unittest.cpp,
// bthread_rwlock_unittest.cpp, bthread_countdown_event_unittest.cpp,
// bthread_butex_unittest.cpp, bthread_key_unittest.cpp,
// bthread_execution_queue_unittest.cpp, bthread_timer_thread_unittest.cpp).
#include <unistd.h>

#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "base/time.h"
#include "fiber/butex.h"
#include "fiber/execution_queue.h"
#include "fiber/fiber.h"
#include "fiber/sync.h"
#include "tests/test.h"

using namespace mrpc;
using namespace mrpc::fiber;

namespace {
// Runs fn in N fibers and joins them.
void RunFibers(int n, const std::function<void(int)>& fn) {
    std::vector<fiber_t> ids(n);
    struct Arg {
        const std::function<void(int)>* fn;
        int i;
    };
    std::vector<Arg> args(n);
    for (int i = 0; i < n; ++i) {
        args[i] = Arg{&fn, i};
        start_background(&ids[i], nullptr,
                         [](void* p) -> void* {
                             Arg* a = static_cast<Arg*>(p);
                             (*a->fn)(a->i);
                             return nullptr;
                         },
                         &args[i]);
    }
    for (fiber_t t : ids) join(t);
}
timespec after_ms(int ms) {
    const int64_t us = realtime_us() + ms * 1000LL;
    return timespec{(time_t)(us / 1000000), (long)(us % 1000000) * 1000};
}
}  // namespace

TEST(FiberSync, mutex_try_lock_and_timed_lock) {
    Mutex m;
    EXPECT_TRUE(m.try_lock());
    EXPECT_FALSE(m.try_lock());
    std::atomic<int> rc{-1};
    RunFibers(1, [&](int) {
        timespec ts = after_ms(30);
        const int64_t t0 = monotonic_us();
        rc = m.timed_lock(&ts) ? 1 : 0;
        EXPECT_GE(monotonic_us() - t0, 20000);
    });
    EXPECT_EQ(rc.load(), 0);  // timed out: still held by us
    m.unlock();
    EXPECT_TRUE(m.try_lock());
    m.unlock();
}

TEST(FiberSync, mutex_excludes_pthreads_and_fibers_together) {
    Mutex m;
    int64_t counter = 0;
    std::thread t([&] {
        for (int i = 0; i < 20000; ++i) {
            LockGuard<Mutex> g(m);
            ++counter;
        }
    });
    RunFibers(8, [&](int) {
        for (int i = 0; i < 5000; ++i) {
            LockGuard<Mutex> g(m);
            ++counter;
        }
    });
    t.join();
    EXPECT_EQ(counter, 20000 + 8 * 5000);
}

TEST(FiberSync, condition_variable_wait_for_times_out) {
    Mutex m;
    ConditionVariable cv;
    std::atomic<int> rc{0};
    RunFibers(1, [&](int) {
        LockGuard<Mutex> g(m);
        const int64_t t0 = monotonic_us();
        rc = cv.wait_for_us(m, 20000);
        EXPECT_GE(monotonic_us() - t0, 15000);
    });
    EXPECT_EQ(rc.load(), ETIMEDOUT);
}

TEST(FiberSync, condition_variable_notify_all_wakes_every_waiter) {
    Mutex m;
    ConditionVariable cv;
    bool go = false;
    std::atomic<int> woke{0};
    std::thread notifier([&] {
        ::usleep(20000);
        {
            LockGuard<Mutex> g(m);
            go = true;
        }
        cv.notify_all();
    });
    RunFibers(16, [&](int) {
        LockGuard<Mutex> g(m);
        while (!go) cv.wait(m);
        ++woke;
    });
    notifier.join();
    EXPECT_EQ(woke.load(), 16);
}

TEST(FiberSync, rwlock_readers_share_writer_excludes) {
    RWLock rw;
    std::atomic<int> readers_in{0}, max_readers{0};
    std::atomic<bool> writer_in{false}, overlap{false};
    RunFibers(12, [&](int i) {
        for (int k = 0; k < 200; ++k) {
            if (i % 4 == 0) {
                rw.wrlock();
                writer_in = true;
                if (readers_in.load() != 0) overlap = true;
                fiber::usleep(10);
                writer_in = false;
                rw.unlock();
            } else {
                rw.rdlock();
                const int n = ++readers_in;
                int m = max_readers.load();
                while (n > m && !max_readers.compare_exchange_weak(m, n)) {
                }
                if (writer_in.load()) overlap = true;
                fiber::usleep(10);
                --readers_in;
                rw.unlock_shared();
            }
        }
    });
    EXPECT_FALSE(overlap.load());
    EXPECT_GT(max_readers.load(), 1);
    EXPECT_TRUE(rw.try_wrlock());
    EXPECT_FALSE(rw.try_rdlock());
    rw.unlock();
    EXPECT_TRUE(rw.try_rdlock());
    EXPECT_FALSE(rw.try_wrlock());
    rw.unlock_shared();
}

TEST(FiberSync, barrier_releases_generations_with_one_serial) {
    Barrier b(4);
    std::atomic<int> serial{0}, passed{0};
    RunFibers(4, [&](int) {
        for (int gen = 0; gen < 5; ++gen) {
            if (b.wait()) ++serial;
            ++passed;
        }
    });
    EXPECT_EQ(serial.load(), 5);
    EXPECT_EQ(passed.load(), 20);
}

TEST(FiberSync, countdown_event_add_and_timed_wait) {
    CountdownEvent ev(2);
    ev.add_count(1);
    EXPECT_EQ(ev.count(), 3);
    timespec ts = after_ms(20);
    EXPECT_NE(ev.timed_wait(&ts), 0);  // nobody signalled
    ev.signal(2);
    std::thread t([&] {
        ::usleep(10000);
        ev.signal();
    });
    EXPECT_EQ(ev.wait(), 0);
    t.join();
    ev.reset(1);
    EXPECT_EQ(ev.count(), 1);
}

TEST(FiberSync, butex_value_mismatch_returns_immediately) {
    std::atomic<int>* b = butex_create();
    b->store(5);
    errno = 0;
    EXPECT_EQ(butex_wait(b, 4), -1);  // expected != current
    EXPECT_EQ(errno, EWOULDBLOCK);
    timespec ts = after_ms(10);
    EXPECT_EQ(butex_wait(b, 5, &ts), -1);
    EXPECT_EQ(errno, ETIMEDOUT);
    EXPECT_EQ(butex_wake(b), 0);  // nobody waiting
    butex_destroy(b);
}

TEST(FiberSync, butex_wake_all_and_requeue) {
    std::atomic<int>* b1 = butex_create();
    std::atomic<int>* b2 = butex_create();
    b1->store(0);
    b2->store(0);
    std::atomic<int> woke{0};
    std::vector<fiber_t> ids(6);
    for (auto& id : ids) {
        start_background(&id, nullptr,
                         [](void* p) -> void* {
                             auto* bs = static_cast<std::pair<std::atomic<int>*, std::atomic<int>*>*>(p);
                             butex_wait(bs->first, 0);
                             delete bs;
                             return nullptr;
                         },
                         new std::pair<std::atomic<int>*, std::atomic<int>*>(b1, b2));
    }
    ::usleep(20000);  // all parked on b1
    b1->store(1);
    EXPECT_EQ(butex_requeue(b1, b2), 1);  // one woken, the rest moved to b2
    ::usleep(10000);
    int alive = 0;
    for (fiber_t t : ids) alive += exists(t) ? 1 : 0;
    EXPECT_EQ(alive, 5);
    EXPECT_EQ(butex_wake_all(b2), 5);
    for (fiber_t t : ids) join(t);
    (void)woke;
    butex_destroy(b1);
    butex_destroy(b2);
}

TEST(FiberSync, keys_are_per_fiber_with_destructors) {
    static std::atomic<int> destroyed{0};
    FiberKey key;
    ASSERT_EQ(key_create(&key, [](void* p) {
                  delete static_cast<int*>(p);
                  ++destroyed;
              }),
              0);
    std::atomic<int> mismatches{0};
    RunFibers(10, [&](int i) {
        EXPECT_TRUE(getspecific(key) == nullptr);
        setspecific(key, new int(i));
        fiber::usleep(1000);  // others run and set theirs meanwhile
        if (*static_cast<int*>(getspecific(key)) != i) ++mismatches;
    });
    EXPECT_EQ(mismatches.load(), 0);
    EXPECT_EQ(destroyed.load(), 10);  // destructors ran as each fiber ended
    EXPECT_EQ(key_delete(key), 0);
}

TEST(FiberSync, stop_and_interrupt_sleeping_fiber) {
    fiber_t t;
    std::atomic<int> rc{0}, err{0};
    struct A {
        std::atomic<int>* rc;
        std::atomic<int>* err;
    } a{&rc, &err};
    start_background(&t, nullptr,
                     [](void* p) -> void* {
                         A* a = static_cast<A*>(p);
                         *a->rc = fiber::usleep(5000000);
                         *a->err = errno;
                         return nullptr;
                     },
                     &a);
    ::usleep(10000);
    EXPECT_FALSE(stopped(t));
    const int64_t t0 = monotonic_us();
    EXPECT_EQ(stop(t), 0);
    join(t);
    EXPECT_LT(monotonic_us() - t0, 1000000);
    EXPECT_EQ(rc.load(), -1);
    EXPECT_EQ(err.load(), ESTOP);
    EXPECT_FALSE(exists(t));
    EXPECT_NE(join(t), 0 + 12345);  // joining an ended fiber returns at once
}

TEST(FiberSync, start_urgent_runs_before_caller_continues) {
    std::atomic<int> order{0}, child_pos{-1}, parent_pos{-1};
    RunFibers(1, [&](int) {
        fiber_t c;
        start_urgent(&c, nullptr,
                     [](void* p) -> void* {
                         auto* o = static_cast<std::pair<std::atomic<int>*, std::atomic<int>*>*>(p);
                         o->second->store(o->first->fetch_add(1));
                         delete o;
                         return nullptr;
                     },
                     new std::pair<std::atomic<int>*, std::atomic<int>*>(&order, &child_pos));
        parent_pos = order.fetch_add(1);
        join(c);
    });
    // The worker switches to the child at once and queues the caller; an
    // idle worker may steal the caller and run it while the child's thread is
    // descheduled (the reference's bthread_start_urgent has the same window),
    // so only "both ran, each exactly once" is guaranteed under load.
    EXPECT_EQ(child_pos.load() + parent_pos.load(), 1);
    EXPECT_TRUE(child_pos.load() == 0 || child_pos.load() == 1);
}

TEST(FiberSync, execution_queue_high_priority_and_stop) {
    struct Meta {
        std::vector<int> seen;
        bool saw_stop = false;
    } meta;
    Mutex gate;
    gate.lock();  // hold the consumer on its first task
    struct Ctx {
        Meta* m;
        Mutex* gate;
    } ctx{&meta, &gate};
    auto q = ExecutionQueue<int>::Create(
        [](void* p, ExecutionQueue<int>::Iterator& it) -> int {
            Ctx* c = static_cast<Ctx*>(p);
            if (it.is_queue_stopped()) {
                c->m->saw_stop = true;
                return 0;
            }
            for (; it; ++it) {
                if (*it == 0) {
                    c->gate->lock();  // block until the producer released it
                    c->gate->unlock();
                }
                c->m->seen.push_back(*it);
            }
            return 0;
        },
        &ctx);
    q->execute(0);
    ::usleep(10000);  // consumer is now blocked inside task 0
    for (int i = 1; i <= 3; ++i) q->execute(i);
    q->execute(100, /*high_priority=*/true);
    gate.unlock();
    q->stop();
    q->join();
    ASSERT_EQ(meta.seen.size(), 5u);
    EXPECT_EQ(meta.seen[0], 0);
    EXPECT_EQ(meta.seen[1], 100);  // high priority jumps the queued normal tasks
    EXPECT_EQ(meta.seen[4], 3);
    EXPECT_TRUE(meta.saw_stop);
    EXPECT_NE(q->execute(7), 0);  // stopped queues refuse work
}

TEST(FiberSync, execution_queue_cancel_before_the_consumer_takes_it) {
    struct Meta {
        std::vector<int> seen;
    } meta;
    Mutex gate;
    gate.lock();
    struct Ctx {
        Meta* m;
        Mutex* gate;
    } ctx{&meta, &gate};
    auto q = ExecutionQueue<int>::Create(
        [](void* p, ExecutionQueue<int>::Iterator& it) -> int {
            Ctx* c = static_cast<Ctx*>(p);
            if (it.is_queue_stopped()) return 0;
            for (; it; ++it) {
                if (*it == 0) {
                    c->gate->lock();
                    c->gate->unlock();
                }
                c->m->seen.push_back(*it);
            }
            return 0;
        },
        &ctx);
    ExecutionQueue<int>::TaskHandle h0, h1, h2, h3, hp;
    ASSERT_EQ(q->execute(0, false, &h0), 0);
    ::usleep(10000);  // the consumer holds task 0
    q->execute(1, false, &h1);
    q->execute(2, false, &h2);
    q->execute(3, false, &h3);
    q->execute(50, true, &hp);
    EXPECT_EQ(q->cancel(h2), 0);    // queued: removed
    EXPECT_EQ(q->cancel(h2), 1);    // not there any more
    EXPECT_EQ(q->cancel(hp), 0);    // high-priority tasks cancel too
    EXPECT_EQ(q->cancel(h0), 1);    // already running
    EXPECT_EQ(q->cancel(ExecutionQueue<int>::TaskHandle()), -1);
    auto other = ExecutionQueue<int>::Create([](void*, ExecutionQueue<int>::Iterator&) -> int { return 0; }, nullptr);
    EXPECT_EQ(other->cancel(h1), -1);  // a handle of another queue
    gate.unlock();
    q->stop();
    q->join();
    ASSERT_EQ(meta.seen.size(), 3u);
    EXPECT_EQ(meta.seen[0], 0);
    EXPECT_EQ(meta.seen[1], 1);
    EXPECT_EQ(meta.seen[2], 3);
    EXPECT_EQ(q->cancel(h3), 1);  // ran
    other->stop();
    other->join();
}

TEST(FiberSync, timer_add_and_delete) {
    std::atomic<int> fired{0};
    TimerId a, b;
    ASSERT_EQ(timer_add_us(&a, 10000, [](void* p) { static_cast<std::atomic<int>*>(p)->fetch_add(1); }, &fired), 0);
    ASSERT_EQ(timer_add_us(&b, 30000, [](void* p) { static_cast<std::atomic<int>*>(p)->fetch_add(10); }, &fired), 0);
    EXPECT_EQ(timer_del(b), 0);  // removed before it ran
    ::usleep(60000);
    EXPECT_EQ(fired.load(), 1);
    EXPECT_EQ(timer_del(a), 1);  // already ran
}

TEST(FiberSync, worker_index_and_self_inside_fibers) {
    std::atomic<int> bad{0};
    RunFibers(20, [&](int) {
        if (!in_fiber() || self() == 0 || worker_index() < 0 || worker_index() >= get_concurrency()) ++bad;
    });
    EXPECT_EQ(bad.load(), 0);
    EXPECT_FALSE(in_fiber());
    EXPECT_EQ(worker_index(), -1);
}

// The contention profiler samples pthread mutexes (std::mutex included)
// through the pthread_mutex_lock interposer (reference:
// src/bthread/mutex.cpp:367-423); with the profiler off nothing is counted.
TEST(FiberSync, contention_profiler_sees_pthread_mutexes) {
    std::mutex mu;  // a pthread mutex underneath
    auto contend = [&mu](int rounds) {
        std::vector<std::thread> ts;
        for (int t = 0; t < 4; ++t) {
            ts.emplace_back([&mu, rounds] {
                for (int i = 0; i < rounds; ++i) {
                    {
                        std::lock_guard<std::mutex> g(mu);
                        ::usleep(500);
                    }
                    ::usleep(300);  // let the waiters in (glibc mutexes are unfair)
                }
            });
        }
        for (auto& t : ts) t.join();
    };
    const int64_t c0 = fiber::PthreadContentionCount();
    contend(10);
    EXPECT_EQ(fiber::PthreadContentionCount(), c0);  // profiler off
    ASSERT_TRUE(fiber::ContentionProfilerStart(nullptr));
    contend(20);
    fiber::ContentionProfilerStop();
    const int64_t n = fiber::PthreadContentionCount() - c0;
    EXPECT_GE(n, 10);  // 4 threads x 20 rounds holding the lock 0.5 ms: many acquisitions wait
    const std::string dump = fiber::ContentionProfilerDump();
    EXPECT_NE(dump.find("0x"), std::string::npos);  // sampled callers (waits >= 1 ms always kept)
}
