// Fiber runtime tests (spirit of reference test/bthread_unittest.cpp,
// bthread_butex_unittest.cpp, bthread_id_unittest.cpp,
// bthread_execution_queue_unittest.cpp, bthread_timer_thread_unittest.cpp).
#include <fcntl.h>
#include <sys/epoll.h>
#include <unistd.h>

#include <atomic>
#include <thread>
#include <vector>

#include "base/time.h"
#include "fiber/butex.h"
#include "fiber/call_id.h"
#include "fiber/execution_queue.h"
#include "fiber/fiber.h"
#include "fiber/sync.h"
#include "tests/test.h"

using namespace mrpc;
using namespace mrpc::fiber;

TEST(Fiber, start_and_join) {
    std::atomic<int> counter{0};
    std::vector<fiber_t> tids(200);
    for (auto& t : tids) {
        ASSERT_EQ(start([&counter] { counter.fetch_add(1); }, false, nullptr, &t), 0);
    }
    for (auto t : tids) EXPECT_EQ(join(t), 0);
    EXPECT_EQ(counter.load(), 200);
}

TEST(Fiber, urgent_nested_and_yield) {
    std::atomic<int> order{0};
    fiber_t outer;
    start([&order] {
        fiber_t inner;
        start([&order] { order.fetch_add(1); yield(); order.fetch_add(1); }, true, nullptr, &inner);
        join(inner);
        order.fetch_add(10);
    }, false, nullptr, &outer);
    join(outer);
    EXPECT_EQ(order.load(), 12);
}

TEST(Fiber, usleep_accuracy) {
    fiber_t t;
    int64_t elapsed = 0;
    start([&elapsed] {
        int64_t t0 = monotonic_us();
        fiber::usleep(20000);
        elapsed = monotonic_us() - t0;
    }, false, nullptr, &t);
    join(t);
    EXPECT_GE(elapsed, 19000);
    EXPECT_LT(elapsed, 200000);
}

TEST(Fiber, many_fibers_mutex) {
    Mutex mu;
    int64_t sum = 0;
    std::vector<fiber_t> tids(64);
    for (auto& t : tids) {
        start([&mu, &sum] {
            for (int i = 0; i < 1000; ++i) {
                mu.lock();
                ++sum;
                if (i % 100 == 0) yield();
                mu.unlock();
            }
        }, false, nullptr, &t);
    }
    for (auto t : tids) join(t);
    EXPECT_EQ(sum, 64000);
}

TEST(Fiber, cond_and_countdown) {
    Mutex mu;
    ConditionVariable cv;
    bool ready = false;
    CountdownEvent done(10);
    for (int i = 0; i < 10; ++i) {
        start([&] {
            mu.lock();
            while (!ready) cv.wait(mu);
            mu.unlock();
            done.signal();
        });
    }
    fiber::usleep(5000);
    mu.lock();
    ready = true;
    cv.notify_all();
    mu.unlock();
    EXPECT_EQ(done.wait(), 0);
}

TEST(Fiber, butex_timeout_and_wake) {
    std::atomic<int>* b = butex_create();
    b->store(0);
    fiber_t t;
    int rc = 0, err = 0;
    start([&] {
        timespec ts = realtime_after_us(10000);
        rc = butex_wait(b, 0, &ts);
        err = errno;
    }, false, nullptr, &t);
    join(t);
    EXPECT_EQ(rc, -1);
    EXPECT_EQ(err, ETIMEDOUT);
    // wake path
    std::atomic<int> woke{0};
    start([&] {
        if (butex_wait(b, 0, nullptr) == 0) woke = 1;
    }, false, nullptr, &t);
    fiber::usleep(5000);
    b->store(1);
    butex_wake(b);
    join(t);
    EXPECT_EQ(woke.load(), 1);
    // pthread waiter
    b->store(0);
    std::thread th([&] {
        timespec ts = realtime_after_us(2000000);
        butex_wait(b, 0, &ts);
    });
    ::usleep(5000);
    b->store(2);
    butex_wake_all(b);
    th.join();
    butex_destroy(b);
}

TEST(Fiber, interrupt_sleep) {
    fiber_t t;
    int rc = 0, err = 0;
    start([&] {
        rc = fiber::usleep(5000000);
        err = errno;
    }, false, nullptr, &t);
    fiber::usleep(10000);
    interrupt(t);
    int64_t t0 = monotonic_us();
    join(t);
    EXPECT_LT(monotonic_us() - t0, 1000000);
    EXPECT_EQ(rc, -1);
    EXPECT_EQ(err, EINTR);
}

TEST(Fiber, fiber_local_storage) {
    FiberKey k;
    static std::atomic<int> dtor_calls{0};
    ASSERT_EQ(key_create(&k, [](void* p) { dtor_calls++; delete (int*)p; }), 0);
    std::vector<fiber_t> tids(8);
    std::atomic<int> ok{0};
    for (int i = 0; i < 8; ++i) {
        start([k, i, &ok] {
            EXPECT_TRUE(getspecific(k) == nullptr);
            setspecific(k, new int(i));
            yield();
            if (*(int*)getspecific(k) == i) ok++;
        }, false, nullptr, &tids[i]);
    }
    for (auto t : tids) join(t);
    EXPECT_EQ(ok.load(), 8);
    EXPECT_EQ(dtor_calls.load(), 8);
    key_delete(k);
}

TEST(Fiber, timer) {
    std::atomic<int> fired{0};
    TimerId id1, id2;
    timer_add_us(&id1, 5000, [](void* a) { ((std::atomic<int>*)a)->fetch_add(1); }, &fired);
    timer_add_us(&id2, 500000, [](void* a) { ((std::atomic<int>*)a)->fetch_add(100); }, &fired);
    EXPECT_EQ(timer_del(id2), 0);
    ::usleep(50000);
    EXPECT_EQ(fired.load(), 1);
    EXPECT_EQ(timer_del(id1), 1);
}

TEST(Fiber, fd_wait_pipe) {
    int fds[2];
    ASSERT_EQ(pipe2(fds, O_NONBLOCK), 0);
    fiber_t t;
    int got = 0;
    start([&] {
        if (fd_wait(fds[0], EPOLLIN) == 0) {
            char c;
            if (read(fds[0], &c, 1) == 1) got = c;
        }
    }, false, nullptr, &t);
    fiber::usleep(5000);
    ASSERT_EQ(write(fds[1], "Z", 1), 1);
    join(t);
    EXPECT_EQ(got, 'Z');
    close(fds[0]);
    close(fds[1]);
}

static int on_err(CallId id, void* data, int code, const std::string&) {
    *(int*)data = code;
    return call_id_unlock_and_destroy(id);
}

TEST(CallId, lock_error_join) {
    int code = 0;
    CallId id;
    ASSERT_EQ(call_id_create_ranged(&id, &code, on_err, 3), 0);
    void* data;
    ASSERT_EQ(call_id_lock(id, &data), 0);
    EXPECT_EQ(data, (void*)&code);
    // error while locked is queued
    EXPECT_EQ(call_id_error(call_id_with_version(id, 1), 1008), 0);
    EXPECT_EQ(code, 0);
    fiber_t joiner;
    std::atomic<bool> joined{false};
    start([&] { call_id_join(id); joined = true; }, false, nullptr, &joiner);
    fiber::usleep(2000);
    EXPECT_FALSE(joined.load());
    // unlock runs the pending error handler which destroys the id
    EXPECT_EQ(call_id_unlock(id), 0);
    EXPECT_EQ(code, 1008);
    join(joiner);
    EXPECT_TRUE(joined.load());
    EXPECT_EQ(call_id_lock(id, &data), EINVAL);
    EXPECT_FALSE(call_id_exists(call_id_with_version(id, 2)));
}

TEST(CallId, contended_lock) {
    CallId id;
    int64_t counter = 0;
    ASSERT_EQ(call_id_create(&id, &counter, nullptr), 0);
    std::vector<fiber_t> tids(16);
    for (auto& t : tids) {
        start([id] {
            for (int i = 0; i < 200; ++i) {
                void* d;
                if (call_id_lock(id, &d) == 0) {
                    ++*(int64_t*)d;
                    call_id_unlock(id);
                }
            }
        }, false, nullptr, &t);
    }
    for (auto t : tids) join(t);
    EXPECT_EQ(counter, 16 * 200);
    void* d;
    call_id_lock(id, &d);
    call_id_unlock_and_destroy(id);
}

struct EqState {
    std::atomic<int64_t> sum{0};
    std::atomic<int> stopped{0};
    std::atomic<int> max_batch{0};
};

static int eq_execute(void* meta, ExecutionQueue<int>::Iterator& it) {
    EqState* s = (EqState*)meta;
    if (it.is_queue_stopped()) {
        s->stopped = 1;
        return 0;
    }
    int n = 0;
    for (; it; ++it) {
        s->sum += *it;
        ++n;
    }
    if (n > s->max_batch) s->max_batch = n;
    return 0;
}

TEST(ExecutionQueue, ordered_batches) {
    EqState st;
    auto q = ExecutionQueue<int>::Create(eq_execute, &st);
    std::vector<std::thread> ths;
    for (int t = 0; t < 4; ++t) {
        ths.emplace_back([&q] {
            for (int i = 1; i <= 1000; ++i) q->execute(i);
        });
    }
    for (auto& t : ths) t.join();
    q->stop();
    q->join();
    EXPECT_EQ(st.sum.load(), 4 * 500500);
    EXPECT_EQ(st.stopped.load(), 1);
    EXPECT_EQ(q->execute(1), EINVAL);
}

TEST(Fiber, scheduling_latency_and_throughput) {
    // create->run latency and creation throughput (reference
    // docs/cn/bthread_or_not.md:55, memory_management.md:32).
    const int N = 20000;
    std::atomic<int> done{0};
    int64_t t0 = monotonic_ns();
    std::vector<fiber_t> tids(N);
    for (int i = 0; i < N; ++i) start_background(&tids[i], nullptr, [](void* a) -> void* {
        ((std::atomic<int>*)a)->fetch_add(1);
        return nullptr;
    }, &done);
    for (int i = 0; i < N; ++i) join(tids[i]);
    int64_t dt = monotonic_ns() - t0;
    EXPECT_EQ(done.load(), N);
    printf("  fiber create+run+join: %.1f ns/fiber\n", (double)dt / N);
}

extern "C" const char* mrpc_fiber_dump();

namespace {
void* sleepy_fiber(void*) {
    mrpc::fiber::usleep(300000);
    return nullptr;
}
}  // namespace

TEST(Fiber, describe_lists_suspended_fibers_for_debuggers) {
    mrpc::fiber::fiber_t t[3];
    for (auto& x : t) mrpc::fiber::start_background(&x, nullptr, sleepy_fiber, nullptr);
    mrpc::fiber::usleep(50000);
    const std::string d = mrpc::fiber::DescribeFibers(1000);
    char fn[32];
    snprintf(fn, sizeof(fn), "fn=%p", (void*)sleepy_fiber);
    size_t n = 0;
    for (size_t p = d.find(fn); p != std::string::npos; p = d.find(fn, p + 1)) ++n;
    EXPECT_EQ(n, 3u);
    EXPECT_TRUE(d.find("sp=0x") != std::string::npos);
    EXPECT_TRUE(std::string(mrpc_fiber_dump()).find(fn) != std::string::npos);
    for (auto& x : t) mrpc::fiber::join(x);
    EXPECT_TRUE(mrpc::fiber::DescribeFibers(1000).find(fn) == std::string::npos);
}
