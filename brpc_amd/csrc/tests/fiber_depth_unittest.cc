// Fiber runtime depth (spirit of the reference's bthread_unittest.cpp,
// bthread_butex_unittest.cpp, bthread_fd_unittest.cpp): join semantics and
// versioned ids, fibers started and joined from plain pthreads, stack
// kinds, deferred signalling, stop on a butex waiter, ordered wake-ups of
// many sleepers, fd waits with deadlines, key destructors, fiber counts.
#include <fcntl.h>
#include <pthread.h>
#include <sys/epoll.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <mutex>
#include <vector>

#include "base/time.h"
#include "fiber/butex.h"
#include "fiber/fiber.h"
#include "fiber/interrupt_pthread.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

void* set_flag(void* arg) {
    static_cast<std::atomic<int>*>(arg)->store(1);
    return nullptr;
}

void* return_arg(void* arg) { return arg; }

// abstime deadlines are CLOCK_REALTIME (as bthread's)
timespec microseconds_from_now(int64_t us) {
    const int64_t t = realtime_us() + us;
    timespec ts;
    ts.tv_sec = t / 1000000;
    ts.tv_nsec = (t % 1000000) * 1000;
    return ts;
}

int recurse(int depth) {
    volatile char pad[256];
    pad[0] = (char)depth;
    return depth == 0 ? pad[0] : recurse(depth - 1) + 1;
}

}  // namespace

TEST(FiberDepth, join_semantics_and_versioned_ids) {
    fiber::fiber_t t1 = 0;
    ASSERT_EQ(fiber::start_background(&t1, nullptr, return_arg, (void*)0x1234), 0);
    void* ret = nullptr;
    ASSERT_EQ(fiber::join(t1, &ret), 0);
    EXPECT_EQ(ret, nullptr);  // return values are not kept (bthread's behaviour)
    EXPECT_FALSE(fiber::exists(t1));
    EXPECT_EQ(fiber::join(t1, nullptr), 0);  // joining a finished fiber returns at once
    EXPECT_EQ(fiber::join(fiber::INVALID_FIBER, nullptr), EINVAL);
    // slots are reused with a new version: old ids never alias new fibers
    std::vector<fiber::fiber_t> ids;
    for (int i = 0; i < 200; ++i) {
        fiber::fiber_t t = 0;
        ASSERT_EQ(fiber::start_background(&t, nullptr, return_arg, nullptr), 0);
        ids.push_back(t);
        fiber::join(t, nullptr);
    }
    std::sort(ids.begin(), ids.end());
    EXPECT_TRUE(std::adjacent_find(ids.begin(), ids.end()) == ids.end());
    // a fiber cannot join itself
    std::atomic<int> self_join{-1};
    fiber::start([&] { self_join = fiber::join(fiber::self(), nullptr); });
    for (int i = 0; i < 1000 && self_join.load() < 0; ++i) ::usleep(1000);
    EXPECT_EQ(self_join.load(), EINVAL);
}

TEST(FiberDepth, started_and_joined_from_plain_pthreads) {
    struct Arg {
        std::atomic<int> done{0};
        int rc = -1;
    } a;
    pthread_t th;
    ASSERT_EQ(pthread_create(
                  &th, nullptr,
                  [](void* p) -> void* {
                      Arg* a = static_cast<Arg*>(p);
                      fiber::fiber_t t = 0;
                      if (fiber::start_background(&t, nullptr, set_flag, &a->done) != 0) return nullptr;
                      a->rc = fiber::join(t, nullptr);  // a pthread blocks on the fiber's butex
                      return nullptr;
                  },
                  &a),
              0);
    pthread_join(th, nullptr);
    EXPECT_EQ(a.rc, 0);
    EXPECT_EQ(a.done.load(), 1);
    EXPECT_FALSE(fiber::in_fiber());
    EXPECT_EQ(fiber::self(), fiber::INVALID_FIBER);
}

TEST(FiberDepth, stack_kinds_run_their_code) {
    std::atomic<int> depth_small{0}, depth_normal{0}, on_pthread{0};
    fiber::fiber_t a = 0, b = 0, c = 0;
    fiber::start([&] { depth_small = recurse(40); }, false, &fiber::ATTR_SMALL, &a);  // ~10 KiB of stack
    fiber::start([&] { depth_normal = recurse(2000); }, false, &fiber::ATTR_NORMAL, &b);  // ~500 KiB
    fiber::start([&] { on_pthread = 1; }, false, &fiber::ATTR_PTHREAD, &c);
    fiber::join(a, nullptr);
    fiber::join(b, nullptr);
    fiber::join(c, nullptr);
    EXPECT_EQ(depth_small.load(), 40);
    EXPECT_EQ(depth_normal.load(), 2000);
    EXPECT_EQ(on_pthread.load(), 1);
}

TEST(FiberDepth, nosignal_tasks_run_after_flush) {
    std::atomic<int> ran{0};
    std::vector<fiber::fiber_t> ts;
    std::atomic<int> done{0};
    fiber::start([&] {
        fiber::Attr attr(fiber::STACK_NORMAL, fiber::ATTR_NOSIGNAL);
        for (int i = 0; i < 32; ++i) {
            fiber::fiber_t t = 0;
            fiber::start([&] { ran.fetch_add(1); }, false, &attr, &t);
        }
        fiber::flush();
        done = 1;
    });
    for (int i = 0; i < 2000 && (done.load() == 0 || ran.load() < 32); ++i) ::usleep(1000);
    EXPECT_EQ(ran.load(), 32);
}

TEST(FiberDepth, stop_wakes_a_butex_waiter) {
    std::atomic<int>* bx = fiber::butex_create();
    bx->store(0);
    std::atomic<int> rc{1}, err{0};
    fiber::fiber_t t = 0;
    fiber::start(
        [&] {
            rc = fiber::butex_wait(bx, 0, nullptr);
            err = errno;
        },
        false, nullptr, &t);
    ::usleep(20000);
    EXPECT_TRUE(fiber::exists(t));
    EXPECT_EQ(fiber::stop(t), 0);
    fiber::join(t, nullptr);
    EXPECT_EQ(rc.load(), -1);
    EXPECT_TRUE(err.load() == EINTR || err.load() == -fiber::ESTOP || err.load() == fiber::ESTOP);
    EXPECT_TRUE(fiber::stopped(t));
    EXPECT_EQ(fiber::stop(t), EINVAL);  // already gone
    fiber::butex_destroy(bx);
}

TEST(FiberDepth, many_sleepers_never_wake_early) {
    // 400 fibers sleeping 20..60 ms, started in a scrambled order: none wakes
    // before its deadline and the typical lateness stays small (the timer
    // thread keeps one heap and runs without timer slack)
    const int n = 400;
    std::vector<int64_t> late(n, -1);
    std::vector<fiber::fiber_t> ts(n);
    for (int i = 0; i < n; ++i) {
        const int k = (i * 7919) % n;
        fiber::start(
            [&late, k] {
                const uint64_t d = 20000 + (uint64_t)k * 100;
                const int64_t s = monotonic_us();
                fiber::usleep(d);
                late[k] = monotonic_us() - s - (int64_t)d;
            },
            false, nullptr, &ts[i]);
    }
    for (auto t : ts) fiber::join(t, nullptr);
    std::vector<int64_t> sorted = late;
    std::sort(sorted.begin(), sorted.end());
    EXPECT_GE(sorted.front(), 0);             // never early
    // median lateness well under the 100 us .. ms range (not under the
    // sanitizers: a TSan timer thread sharing the host with other TSan
    // suites runs 100+ ms late whatever the scheduler does)
    if (mtest::kSlowdown == 1) EXPECT_LT(sorted[n / 2], 5000);
    EXPECT_LT(sorted.back(), 500000 * mtest::kSlowdown);
}

TEST(FiberDepth, fd_timedwait_times_out_then_sees_data) {
    int p[2];
    ASSERT_EQ(pipe(p), 0);
    fcntl(p[0], F_SETFL, O_NONBLOCK);
    std::atomic<int> first{1}, second{1};
    std::atomic<int64_t> waited{0};
    fiber::fiber_t t = 0;
    fiber::start(
        [&] {
            const int64_t s = monotonic_us();
            timespec dl = microseconds_from_now(30000);
            first = fiber::fd_timedwait(p[0], EPOLLIN, &dl);
            waited = monotonic_us() - s;
            dl = microseconds_from_now(2000000);
            second = fiber::fd_timedwait(p[0], EPOLLIN, &dl);
        },
        false, nullptr, &t);
    ::usleep(100000);
    ASSERT_EQ(write(p[1], "x", 1), 1);
    fiber::join(t, nullptr);
    EXPECT_EQ(first.load(), -1);  // ETIMEDOUT after ~30 ms
    EXPECT_GE(waited.load(), 29000);
    EXPECT_EQ(second.load(), 0);
    close(p[0]);
    close(p[1]);
}

TEST(FiberDepth, key_destructors_run_per_fiber_with_their_values) {
    static std::atomic<int> sum{0};
    fiber::FiberKey key;
    ASSERT_EQ(fiber::key_create(&key, [](void* v) { sum.fetch_add((int)(intptr_t)v); }), 0);
    std::vector<fiber::fiber_t> ts(10);
    for (int i = 0; i < 10; ++i) {
        fiber::start(
            [key, i] {
                fiber::setspecific(key, (void*)(intptr_t)(i + 1));
                fiber::yield();
                if (fiber::getspecific(key) != (void*)(intptr_t)(i + 1)) sum.fetch_add(1000);
            },
            false, nullptr, &ts[i]);
    }
    for (auto t : ts) fiber::join(t, nullptr);
    EXPECT_EQ(sum.load(), 55);  // 1 + ... + 10, each destructor once, no cross-talk
    EXPECT_EQ(fiber::key_delete(key), 0);
}

TEST(FiberDepth, fiber_count_tracks_live_fibers) {
    // Measured against the count while the 50 are alive, not against a
    // sample taken before them: fibers of earlier cases may still be
    // exiting when this starts, and exits only ever lower the count, so
    // both checks hold whatever else is winding down.
    std::atomic<int> release{0};
    std::atomic<int> started{0};
    std::vector<fiber::fiber_t> ts(50);
    for (auto& t : ts) {
        fiber::start(
            [&] {
                started.fetch_add(1);
                while (!release.load()) fiber::usleep(1000);
            },
            false, nullptr, &t);
    }
    for (int i = 0; i < 2000 && started.load() < 50; ++i) ::usleep(1000);
    ASSERT_EQ(started.load(), 50);
    const int64_t during = fiber::fiber_count();
    EXPECT_GE(during, 50);
    release = 1;
    for (auto t : ts) fiber::join(t, nullptr);
    for (int i = 0; i < 100 && fiber::fiber_count() > during - 50; ++i) ::usleep(1000);
    EXPECT_LE(fiber::fiber_count(), during - 50);
}

TEST(FiberDepth, interrupt_racing_a_sleep_never_loses_the_wake) {
    // interrupt() issued while the target is still getting to, or just
    // entering, its sleep: the sleep must end at once with EINTR (the
    // publish of the sleep's timer and the interrupt used to race, and the
    // fiber then slept its full time)
    const int n = 200;
    std::vector<fiber::fiber_t> ts(n);
    std::vector<int> rcs(n, 0), errs(n, 0);
    const int64_t t0 = monotonic_us();
    for (int i = 0; i < n; ++i) {
        fiber::start(
            [&rcs, &errs, i] {
                rcs[i] = fiber::usleep(3000000);
                errs[i] = errno;
            },
            false, nullptr, &ts[i]);
        if (i % 3 == 1) fiber::yield();
        fiber::interrupt(ts[i]);
    }
    for (auto t : ts) fiber::join(t, nullptr);
    EXPECT_LT(monotonic_us() - t0, 2000000);
    int eintr = 0;
    for (int i = 0; i < n; ++i) eintr += rcs[i] == -1 && errs[i] == EINTR;
    EXPECT_EQ(eintr, n);
}

TEST(FiberDepth, parked_workers_never_miss_a_signal) {
    // A signal skips FUTEX_WAKE when no worker sits in its parking lot
    // (-fiber_signal_parked_only). Four plain pthreads start fibers and
    // wake butex waiters at irregular gaps, so workers park, nap and spin
    // while signals arrive: every fiber must run, none may wait for an
    // unrelated event to be noticed.
    std::atomic<int> failures{0};
    std::vector<pthread_t> th(4);
    for (auto& t : th) {
        pthread_create(
            &t, nullptr,
            [](void* arg) -> void* {
                auto* fails = static_cast<std::atomic<int>*>(arg);
                for (int i = 0; i < 150; ++i) {
                    usleep(i % 25 == 0 ? 15000 : 50 + (i * 37) % 400);
                    std::atomic<int> done{0};
                    fiber::fiber_t f;
                    if (fiber::start_background(&f, nullptr, set_flag, &done) != 0) {
                        fails->fetch_add(1);
                        continue;
                    }
                    const int64_t t0 = monotonic_us();
                    while (done.load() == 0 && monotonic_us() - t0 < 2000000) usleep(20);
                    if (done.load() == 0) fails->fetch_add(1);
                    fiber::join(f, nullptr);
                    // a fiber parked on a butex, woken from this pthread
                    std::atomic<int>* b = fiber::butex_create();
                    b->store(0);
                    std::atomic<int> woke{0};
                    fiber::fiber_t w;
                    fiber::start(
                        [b, &woke] {
                            while (b->load() == 0) fiber::butex_wait(b, 0, nullptr);
                            woke.store(1);
                        },
                        false, nullptr, &w);
                    usleep(30 + i % 90);
                    b->store(1);
                    fiber::butex_wake_all(b);
                    const int64_t t1 = monotonic_us();
                    while (woke.load() == 0 && monotonic_us() - t1 < 2000000) usleep(20);
                    if (woke.load() == 0) fails->fetch_add(1);
                    fiber::join(w, nullptr);
                    fiber::butex_destroy(b);
                }
                return nullptr;
            },
            &failures);
    }
    for (auto& t : th) pthread_join(t, nullptr);
    EXPECT_EQ(failures.load(), 0);
}

// interrupt_pthread (reference src/bthread/interrupt_pthread.cpp): a fiber
// blocked in a system call on its worker — invisible to the runtime, no
// butex or timer to cancel — gets EINTR from fiber::interrupt().
namespace {
struct BlockedRead {
    int fd = -1;
    std::atomic<int> started{0};
    std::atomic<int> result{0};
    std::atomic<int> err{0};
};
void* blocking_read(void* arg) {
    BlockedRead* b = static_cast<BlockedRead*>(arg);
    b->started.store(1);
    char c;
    const ssize_t n = ::read(b->fd, &c, 1);  // blocks the worker pthread
    b->err.store(n < 0 ? errno : 0);
    b->result.store(n < 0 ? -1 : 2);
    return nullptr;
}
}  // namespace

TEST(FiberDepth, interrupt_wakes_a_fiber_blocked_in_a_syscall) {
    int p[2];
    ASSERT_EQ(pipe(p), 0);
    BlockedRead b;
    b.fd = p[0];
    fiber::fiber_t t = 0;
    ASSERT_EQ(fiber::start_background(&t, nullptr, blocking_read, &b), 0);
    for (int i = 0; i < 2000 && !b.started.load(); ++i) ::usleep(1000);
    ASSERT_EQ(b.started.load(), 1);
    ::usleep(20000);  // let it enter read()
    EXPECT_EQ(b.result.load(), 0);
    const long before = fiber::interrupt_pthread_signals();
    ASSERT_EQ(fiber::interrupt(t), 0);
    for (int i = 0; i < 2000 && b.result.load() == 0; ++i) ::usleep(1000);
    EXPECT_EQ(b.result.load(), -1);
    EXPECT_EQ(b.err.load(), EINTR);
    EXPECT_GT(fiber::interrupt_pthread_signals(), before);
    fiber::join(t, nullptr);
    close(p[0]);
    close(p[1]);
}

TEST(FiberDepth, interrupt_pthread_breaks_a_plain_blocking_call) {
    int p[2];
    ASSERT_EQ(pipe(p), 0);
    std::atomic<int> err{0};
    std::atomic<int> in{0};
    pthread_t th;
    struct Args {
        int fd;
        std::atomic<int>* err;
        std::atomic<int>* in;
    } a{p[0], &err, &in};
    ASSERT_EQ(pthread_create(&th, nullptr,
                             [](void* x) -> void* {
                                 Args* a = static_cast<Args*>(x);
                                 a->in->store(1);
                                 char c;
                                 const ssize_t n = ::read(a->fd, &c, 1);
                                 a->err->store(n < 0 ? errno : -1);
                                 return nullptr;
                             },
                             &a),
              0);
    for (int i = 0; i < 2000 && !in.load(); ++i) ::usleep(1000);
    ::usleep(20000);
    ASSERT_EQ(fiber::interrupt_pthread(th), 0);
    pthread_join(th, nullptr);
    EXPECT_EQ(err.load(), EINTR);
    close(p[0]);
    close(p[1]);
}
