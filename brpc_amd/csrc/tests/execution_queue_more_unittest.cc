// More ExecutionQueue cases (fiber/execution_queue.h), after the reference's
// test/bthread_execution_queue_unittest.cpp: refusal after stop, repeated
// stop/join, the stop callback of an idle queue, priority order, cancel
// handles that name nothing / another queue / a finished task, pending
// counts, move-only tasks, one consumer at a time under fiber and pthread
// producers, consumers that restart after idling, and queues whose owner
// lets go while work is still queued.
#include <unistd.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "fiber/execution_queue.h"
#include "fiber/sync.h"
#include "tests/test.h"

using namespace mrpc;
using namespace mrpc::fiber;

namespace {

typedef ExecutionQueue<int> IQ;

struct Seen {
    std::mutex mu;
    std::vector<int> v;
    std::vector<size_t> batch_sizes;
    std::atomic<int> stops{0};
    std::atomic<int> calls{0};
    Mutex* gate = nullptr;  // held by the test to park the first consumer call
    bool gated_once = false;
};

int collect(void* meta, IQ::Iterator& it) {
    Seen* s = static_cast<Seen*>(meta);
    s->calls.fetch_add(1);
    if (s->gate && !s->gated_once) {
        s->gated_once = true;
        s->gate->lock();
        s->gate->unlock();
    }
    if (it.is_queue_stopped()) {
        s->stops.fetch_add(1);
        return 0;
    }
    std::lock_guard<std::mutex> g(s->mu);
    s->batch_sizes.push_back(it.size());
    for (; it; ++it) s->v.push_back(*it);
    return 0;
}

}  // namespace

TEST(ExecutionQueueMore, execute_after_stop_is_refused) {
    Seen s;
    auto q = IQ::Create(collect, &s);
    EXPECT_EQ(q->execute(1), 0);
    q->stop();
    EXPECT_TRUE(q->stopped());
    EXPECT_EQ(q->execute(2), EINVAL);
    q->join();
    EXPECT_EQ(s.v.size(), 1u);
    EXPECT_EQ(s.stops.load(), 1);
}

TEST(ExecutionQueueMore, stop_and_join_twice_are_harmless) {
    Seen s;
    auto q = IQ::Create(collect, &s);
    q->execute(5);
    q->stop();
    q->stop();
    EXPECT_EQ(q->join(), 0);
    EXPECT_EQ(q->join(), 0);
    EXPECT_EQ(s.stops.load(), 1);
}

TEST(ExecutionQueueMore, idle_queue_still_gets_one_stop_call) {
    Seen s;
    auto q = IQ::Create(collect, &s);
    q->stop();
    q->join();
    EXPECT_EQ(s.calls.load(), 1);
    EXPECT_EQ(s.stops.load(), 1);
    EXPECT_TRUE(s.v.empty());
}

TEST(ExecutionQueueMore, high_priority_overtakes_queued_normal_tasks) {
    Seen s;
    Mutex gate;
    gate.lock();
    s.gate = &gate;
    auto q = IQ::Create(collect, &s);
    q->execute(0);  // taken by the first (parked) call
    while (s.calls.load() == 0) ::usleep(100);
    for (int i = 1; i <= 5; ++i) q->execute(i);
    q->execute(100, true);
    q->execute(101, true);
    gate.unlock();
    q->stop();
    q->join();
    std::vector<int> want = {0, 100, 101, 1, 2, 3, 4, 5};
    EXPECT_TRUE(s.v == want);
}

TEST(ExecutionQueueMore, cancel_with_a_foreign_or_empty_handle) {
    Seen s1, s2;
    auto a = IQ::Create(collect, &s1);
    auto b = IQ::Create(collect, &s2);
    IQ::TaskHandle none;
    EXPECT_EQ(a->cancel(none), -1);
    Mutex gate;
    gate.lock();
    s2.gate = &gate;
    IQ::TaskHandle hb;
    b->execute(1, false, &hb);
    EXPECT_EQ(a->cancel(hb), -1);  // names a task of b
    gate.unlock();
    a->stop();
    b->stop();
    a->join();
    b->join();
    EXPECT_EQ(s2.v.size(), 1u);
}

TEST(ExecutionQueueMore, cancel_after_the_task_ran_says_one) {
    Seen s;
    auto q = IQ::Create(collect, &s);
    IQ::TaskHandle h;
    q->execute(9, false, &h);
    while (true) {
        {
            std::lock_guard<std::mutex> g(s.mu);
            if (!s.v.empty()) break;
        }
        ::usleep(100);
    }
    EXPECT_EQ(q->cancel(h), 1);
    q->stop();
    q->join();
}

TEST(ExecutionQueueMore, cancelled_tasks_leave_the_rest_in_order) {
    Seen s;
    Mutex gate;
    gate.lock();
    s.gate = &gate;
    auto q = IQ::Create(collect, &s);
    q->execute(0);
    while (s.calls.load() == 0) ::usleep(100);
    std::vector<IQ::TaskHandle> hs(10);
    for (int i = 1; i <= 10; ++i) q->execute(i, false, &hs[i - 1]);
    EXPECT_EQ(q->pending(), 10u);
    EXPECT_EQ(q->cancel(hs[1]), 0);  // 2
    EXPECT_EQ(q->cancel(hs[4]), 0);  // 5
    EXPECT_EQ(q->cancel(hs[9]), 0);  // 10
    EXPECT_EQ(q->cancel(hs[4]), 1);  // already gone
    EXPECT_EQ(q->pending(), 7u);
    gate.unlock();
    q->stop();
    q->join();
    std::vector<int> want = {0, 1, 3, 4, 6, 7, 8, 9};
    EXPECT_TRUE(s.v == want);
}

TEST(ExecutionQueueMore, move_only_tasks) {
    typedef ExecutionQueue<std::unique_ptr<int>> UQ;
    struct Sum {
        std::atomic<int> total{0};
    } sum;
    auto q = UQ::Create(
        [](void* m, UQ::Iterator& it) -> int {
            for (; it; ++it) static_cast<Sum*>(m)->total.fetch_add(**it);
            return 0;
        },
        &sum);
    for (int i = 1; i <= 100; ++i) EXPECT_EQ(q->execute(std::unique_ptr<int>(new int(i))), 0);
    q->stop();
    q->join();
    EXPECT_EQ(sum.total.load(), 5050);
}

TEST(ExecutionQueueMore, one_consumer_at_a_time_under_mixed_producers) {
    struct Guard {
        std::atomic<int> inside{0};
        std::atomic<int> overlap{0};
        std::atomic<long> count{0};
    } g;
    auto q = IQ::Create(
        [](void* m, IQ::Iterator& it) -> int {
            Guard* g = static_cast<Guard*>(m);
            if (g->inside.fetch_add(1) != 0) g->overlap.fetch_add(1);
            for (; it; ++it) g->count.fetch_add(1);
            g->inside.fetch_sub(1);
            return 0;
        },
        &g);
    std::vector<std::thread> ts;
    for (int t = 0; t < 4; ++t) {
        ts.emplace_back([&q] {
            for (int i = 0; i < 3000; ++i) q->execute(i);
        });
    }
    CountdownEvent fibers_done(4);
    for (int f = 0; f < 4; ++f) {
        start([&q, &fibers_done] {
            for (int i = 0; i < 3000; ++i) {
                q->execute(i);
                if (i % 256 == 0) yield();
            }
            fibers_done.signal();
        });
    }
    for (auto& t : ts) t.join();
    fibers_done.wait();
    q->stop();
    q->join();
    EXPECT_EQ(g.count.load(), 24000);
    EXPECT_EQ(g.overlap.load(), 0);
}

TEST(ExecutionQueueMore, consumer_restarts_after_idling) {
    Seen s;
    auto q = IQ::Create(collect, &s);
    for (int round = 0; round < 5; ++round) {
        q->execute(round);
        for (;;) {
            {
                std::lock_guard<std::mutex> g(s.mu);
                if ((int)s.v.size() == round + 1) break;
            }
            ::usleep(200);
        }
        ::usleep(2000);  // let the consumer fiber exit
    }
    q->stop();
    q->join();
    std::vector<int> want = {0, 1, 2, 3, 4};
    EXPECT_TRUE(s.v == want);
    EXPECT_TRUE(s.calls.load() >= 6);  // at least one call per round + stop
}

TEST(ExecutionQueueMore, queue_outlives_its_owner_until_the_work_is_done) {
    Seen s;
    Mutex gate;
    gate.lock();
    s.gate = &gate;
    std::weak_ptr<IQ> weak;
    {
        auto q = IQ::Create(collect, &s);
        weak = q;
        for (int i = 0; i < 50; ++i) q->execute(i);
        while (s.calls.load() == 0) ::usleep(100);
    }
    EXPECT_FALSE(weak.expired());  // the running consumer holds it
    gate.unlock();
    for (int i = 0; i < 2000 && !weak.expired(); ++i) ::usleep(1000);
    EXPECT_TRUE(weak.expired());
    std::lock_guard<std::mutex> g(s.mu);  // expired() is a relaxed load: no ordering with the consumer's writes
    EXPECT_EQ(s.v.size(), 50u);
}

TEST(ExecutionQueueMore, batch_of_one) {
    Seen s;
    IQ::Options o;
    o.max_batch = 1;
    auto q = IQ::Create(collect, &s, o);
    for (int i = 0; i < 200; ++i) q->execute(i);
    q->stop();
    q->join();
    EXPECT_EQ(s.v.size(), 200u);
    for (size_t b : s.batch_sizes) EXPECT_EQ(b, 1u);
    for (int i = 0; i < 200; ++i) EXPECT_EQ(s.v[(size_t)i], i);
}
