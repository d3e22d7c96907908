// Wake paths of the fiber runtime (fiber/runtime.cc signal_task,
// spin_for_task; fiber/internal.h ParkingLot), after the reference's
// test/bthread_unittest.cpp and bthread_butex_unittest.cpp: ready fibers
// must never be stranded by a skipped wake. Covers the parked-only signal
// (no FUTEX_WAKE without a parked worker), the spinner skip (no wake while
// an idle worker spins, -fiber_idle_spin_us > 0) and its race with a
// spinner that gives up and parks, ATTR_NOSIGNAL + flush, remote starts from
// plain pthreads, butex wake variants for fiber and pthread waiters, fd waits
// and timers.
#include <fcntl.h>
#include <sys/epoll.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "base/flags.h"
#include "base/time.h"
#include "fiber/butex.h"
#include "fiber/fiber.h"
#include "fiber/sync.h"
#include "tests/test.h"

using namespace mrpc;
using namespace mrpc::fiber;

namespace {

// Sets a runtime flag for the scope of a test and restores it after.
struct ScopedFlag {
    std::string name, old;
    ScopedFlag(const char* n, const char* v) : name(n) {
        GetFlag(name, &old);
        SetFlag(name, v);
    }
    ~ScopedFlag() { SetFlag(name, old); }
};

std::atomic<int64_t> g_ran{0};
void* bump(void*) {
    g_ran.fetch_add(1, std::memory_order_relaxed);
    return nullptr;
}

// Waits (from a pthread) until g_ran reaches want or the deadline passes.
bool wait_ran(int64_t want, int timeout_ms) {
    const int64_t end = monotonic_us() + (int64_t)timeout_ms * 1000;
    while (g_ran.load() < want) {
        if (monotonic_us() > end) return false;
        ::usleep(200);
    }
    return true;
}

// Let every worker go idle and park (or finish its spin).
void let_workers_park() { ::usleep(20000); }

}  // namespace

TEST(FiberWake, remote_starts_from_pthreads_all_run_with_spinning_on) {
    ScopedFlag spin("fiber_idle_spin_us", "30");
    g_ran = 0;
    std::vector<std::thread> ts;
    for (int t = 0; t < 4; ++t) {
        ts.emplace_back([] {
            for (int i = 0; i < 5000; ++i) {
                fiber_t tid;
                ASSERT_EQ(start_background(&tid, nullptr, bump, nullptr), 0);
            }
        });
    }
    for (auto& t : ts) t.join();
    EXPECT_TRUE(wait_ran(20000, 10000));
}

TEST(FiberWake, fibers_starting_fibers_all_run_with_spinning_on) {
    ScopedFlag spin("fiber_idle_spin_us", "30");
    g_ran = 0;
    CountdownEvent done(8);
    for (int f = 0; f < 8; ++f) {
        start([&done] {
            std::vector<fiber_t> tids(64);
            for (int round = 0; round < 40; ++round) {
                for (auto& t : tids) start_background(&t, nullptr, bump, nullptr);
                for (auto t : tids) join(t);
            }
            done.signal();
        });
    }
    done.wait();
    EXPECT_EQ(g_ran.load(), 8 * 40 * 64);
}

// The skipped-wake race: a spinner about to give up is counted when the
// starter skips the wake; it must not park through the new task. Every start
// lands on an idle runtime, from a pthread (the remote queue: no worker of
// the starter's own picks it up).
TEST(FiberWake, idle_runtime_answers_every_lone_remote_start) {
    ScopedFlag spin("fiber_idle_spin_us", "5");
    g_ran = 0;
    for (int i = 0; i < 200; ++i) {
        if (i % 20 == 0) let_workers_park();
        else ::usleep((useconds_t)(i % 7) * 3);  // around the 5 us spin budget
        fiber_t tid;
        ASSERT_EQ(start_background(&tid, nullptr, bump, nullptr), 0);
        ASSERT_TRUE(wait_ran(i + 1, 2000));
    }
}

TEST(FiberWake, idle_runtime_answers_lone_starts_with_spinning_off) {
    ScopedFlag spin("fiber_idle_spin_us", "0");
    g_ran = 0;
    for (int i = 0; i < 50; ++i) {
        if (i % 10 == 0) let_workers_park();
        fiber_t tid;
        ASSERT_EQ(start_background(&tid, nullptr, bump, nullptr), 0);
        ASSERT_TRUE(wait_ran(i + 1, 2000));
    }
}

TEST(FiberWake, skip_when_spinning_off_still_runs_everything) {
    ScopedFlag spin("fiber_idle_spin_us", "30");
    ScopedFlag skip("fiber_signal_skip_when_spinning", "false");
    g_ran = 0;
    for (int i = 0; i < 3000; ++i) {
        fiber_t tid;
        start_background(&tid, nullptr, bump, nullptr);
    }
    EXPECT_TRUE(wait_ran(3000, 10000));
}

TEST(FiberWake, unconditional_signals_still_run_everything) {
    ScopedFlag parked("fiber_signal_parked_only", "false");
    g_ran = 0;
    for (int i = 0; i < 3000; ++i) {
        fiber_t tid;
        start_background(&tid, nullptr, bump, nullptr);
    }
    EXPECT_TRUE(wait_ran(3000, 10000));
}

TEST(FiberWake, nosignal_batch_runs_after_flush) {
    g_ran = 0;
    CountdownEvent done(1);
    start([&done] {
        Attr attr = ATTR_NORMAL;
        attr.flags |= ATTR_NOSIGNAL;
        std::vector<fiber_t> tids(500);
        for (auto& t : tids) start_background(&t, &attr, bump, nullptr);
        flush();
        for (auto t : tids) join(t);
        done.signal();
    });
    done.wait();
    EXPECT_EQ(g_ran.load(), 500);
}

TEST(FiberWake, nosignal_from_a_pthread_runs_after_flush) {
    g_ran = 0;
    Attr attr = ATTR_NORMAL;
    attr.flags |= ATTR_NOSIGNAL;
    let_workers_park();
    for (int i = 0; i < 100; ++i) {
        fiber_t tid;
        start_background(&tid, &attr, bump, nullptr);
    }
    flush();
    EXPECT_TRUE(wait_ran(100, 5000));
}

TEST(FiberWake, butex_ping_pong_with_spinning_on) {
    ScopedFlag spin("fiber_idle_spin_us", "20");
    std::atomic<int>* b = butex_create();
    b->store(0);
    const int kRounds = 5000;
    CountdownEvent done(2);
    for (int side = 0; side < 2; ++side) {
        start([b, side, &done] {
            for (int i = side; i < 2 * kRounds; i += 2) {
                for (int v; (v = b->load()) != i;) butex_wait(b, v);
                b->store(i + 1);
                butex_wake(b);
            }
            done.signal();
        });
    }
    done.wait();
    EXPECT_EQ(b->load(), 2 * kRounds);
    butex_destroy(b);
}

TEST(FiberWake, butex_wakes_a_pthread_waiter_from_a_fiber) {
    std::atomic<int>* b = butex_create();
    b->store(0);
    std::atomic<bool> woke{false};
    std::thread waiter([&] {
        while (b->load() == 0) butex_wait(b, 0);
        woke = true;
    });
    ::usleep(10000);
    CountdownEvent done(1);
    start([&] {
        b->store(1);
        butex_wake_all(b);
        done.signal();
    });
    done.wait();
    waiter.join();
    EXPECT_TRUE(woke.load());
    butex_destroy(b);
}

TEST(FiberWake, butex_wake_except_spares_one_waiter) {
    std::atomic<int>* b = butex_create();
    b->store(0);
    std::atomic<int> woken{0};
    std::vector<fiber_t> tids(4);
    for (auto& t : tids) {
        start(
            [b, &woken] {
                const timespec dl = realtime_after_us(300000);
                if (butex_wait(b, 0, &dl) == 0) woken.fetch_add(1);
            },
            false, nullptr, &t);
    }
    ::usleep(30000);  // all four parked on b
    EXPECT_EQ(butex_wake_except(b, tids[2]), 3);
    for (auto t : tids) join(t);
    EXPECT_EQ(woken.load(), 3);  // the spared one timed out
    butex_destroy(b);
}

TEST(FiberWake, many_fibers_wait_on_their_own_pipes) {
    const int kN = 32;
    std::vector<int> rd(kN), wr(kN);
    for (int i = 0; i < kN; ++i) {
        int p[2];
        ASSERT_EQ(pipe(p), 0);
        rd[i] = p[0];
        wr[i] = p[1];
    }
    std::atomic<int> ok{0};
    std::vector<fiber_t> tids(kN);
    for (int i = 0; i < kN; ++i) {
        start(
            [&, i] {
                if (fd_wait(rd[i], EPOLLIN) == 0) {
                    char c;
                    if (read(rd[i], &c, 1) == 1 && c == (char)('a' + i % 26)) ok.fetch_add(1);
                }
            },
            false, nullptr, &tids[i]);
    }
    ::usleep(20000);
    for (int i = kN - 1; i >= 0; --i) {  // in reverse: readiness, not order
        const char c = (char)('a' + i % 26);
        ASSERT_EQ(write(wr[i], &c, 1), 1);
    }
    for (auto t : tids) join(t);
    EXPECT_EQ(ok.load(), kN);
    for (int i = 0; i < kN; ++i) {
        close(rd[i]);
        close(wr[i]);
    }
}

TEST(FiberWake, timers_fire_in_deadline_order_and_delete_semantics) {
    static std::atomic<int> seq{0}, done{0};
    static int order[3];
    seq = 0;
    done = 0;
    auto rec = [](void* a) {
        order[seq.fetch_add(1)] = (int)(intptr_t)a;
        done.fetch_add(1, std::memory_order_release);  // the slot is written before it counts
    };
    TimerId t30, t10, t20, never;
    (void)t30;
    (void)t20;
    ASSERT_EQ(timer_add_us(&t30, 30000, rec, (void*)30), 0);
    ASSERT_EQ(timer_add_us(&t10, 10000, rec, (void*)10), 0);
    ASSERT_EQ(timer_add_us(&t20, 20000, rec, (void*)20), 0);
    ASSERT_EQ(timer_add_us(&never, 5000000, rec, (void*)99), 0);
    EXPECT_EQ(timer_del(never), 0);  // removed before it ran
    const int64_t end = monotonic_us() + 2000000;
    while (done.load(std::memory_order_acquire) < 3 && monotonic_us() < end) ::usleep(1000);
    ASSERT_EQ(done.load(std::memory_order_acquire), 3);
    EXPECT_EQ(order[0], 10);
    EXPECT_EQ(order[1], 20);
    EXPECT_EQ(order[2], 30);
    EXPECT_NE(timer_del(t10), 0);  // already ran: not "removed before it ran"
}

TEST(FiberWake, usleep_in_fibers_overlaps) {
    const int64_t t0 = monotonic_us();
    std::vector<fiber_t> tids(64);
    for (auto& t : tids) start([] { fiber::usleep(30000); }, false, nullptr, &t);
    for (auto t : tids) join(t);
    const int64_t took = monotonic_us() - t0;
    EXPECT_GE(took, 28000);
    EXPECT_LT(took, 1000000);  // 64 sleepers in parallel, not 64 x 30 ms
}
