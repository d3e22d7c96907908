// ExecutionQueue depth (fiber/execution_queue.h), in the spirit of the
// reference's test/bthread_execution_queue_unittest.cpp: order per producer
// under many producers, batch bounds, stop semantics with pending work,
// consumers that do not iterate, re-entrant execute, and cancel from every
// side (self, random under load, high priority).
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <random>
#include <set>
#include <thread>
#include <vector>

#include "fiber/execution_queue.h"
#include "fiber/sync.h"
#include "tests/test.h"

using namespace mrpc;
using namespace mrpc::fiber;

namespace {

typedef ExecutionQueue<int64_t> Q;

struct Log {
    std::mutex mu;
    std::vector<int64_t> seen;
    std::vector<size_t> batches;
    std::atomic<int> stops{0};
};

int record(void* meta, Q::Iterator& it) {
    Log* l = static_cast<Log*>(meta);
    if (it.is_queue_stopped()) {
        l->stops.fetch_add(1);
        return 0;
    }
    std::lock_guard<std::mutex> g(l->mu);
    l->batches.push_back(it.size());
    for (; it; ++it) l->seen.push_back(*it);
    return 0;
}

}  // namespace

TEST(ExecutionQueueDepth, single_producer_order_is_exact) {
    Log log;
    auto q = Q::Create(record, &log);
    for (int64_t i = 0; i < 10000; ++i) ASSERT_EQ(q->execute(i), 0);
    q->stop();
    q->join();
    ASSERT_EQ(log.seen.size(), 10000u);
    for (int64_t i = 0; i < 10000; ++i) ASSERT_EQ(log.seen[(size_t)i], i);
    EXPECT_EQ(log.stops.load(), 1);
}

TEST(ExecutionQueueDepth, every_producer_keeps_its_order) {
    Log log;
    auto q = Q::Create(record, &log);
    const int P = 6, N = 5000;
    std::vector<std::thread> ts;
    for (int p = 0; p < P; ++p) {
        ts.emplace_back([&q, p] {
            for (int i = 0; i < N; ++i) q->execute(((int64_t)p << 32) | i);
        });
    }
    for (auto& t : ts) t.join();
    q->stop();
    q->join();
    ASSERT_EQ(log.seen.size(), (size_t)P * N);
    std::vector<int64_t> last(P, -1);
    for (int64_t v : log.seen) {
        const int p = (int)(v >> 32);
        const int64_t i = v & 0xffffffff;
        ASSERT_EQ(i, last[p] + 1);
        last[p] = i;
    }
}

TEST(ExecutionQueueDepth, batches_respect_max_batch) {
    Log log;
    Q::Options o;
    o.max_batch = 7;
    Mutex gate;
    gate.lock();
    struct Ctx {
        Log* l;
        Mutex* g;
        bool first = true;
    } ctx{&log, &gate};
    auto q = Q::Create(
        [](void* m, Q::Iterator& it) -> int {
            Ctx* c = static_cast<Ctx*>(m);
            if (c->first) {  // hold the consumer until everything is queued
                c->first = false;
                c->g->lock();
                c->g->unlock();
            }
            return record(c->l, it);
        },
        &ctx, o);
    for (int64_t i = 0; i < 100; ++i) q->execute(i);
    gate.unlock();
    q->stop();
    q->join();
    ASSERT_EQ(log.seen.size(), 100u);
    for (size_t b : log.batches) EXPECT_LE(b, 7u);
    EXPECT_GE(log.batches.size(), 100u / 7);
}

TEST(ExecutionQueueDepth, stop_runs_pending_work_first) {
    Log log;
    Mutex gate;
    gate.lock();
    struct Ctx {
        Log* l;
        Mutex* g;
        bool first = true;
    } ctx{&log, &gate};
    auto q = Q::Create(
        [](void* m, Q::Iterator& it) -> int {
            Ctx* c = static_cast<Ctx*>(m);
            if (c->first && !it.is_queue_stopped()) {
                c->first = false;
                c->g->lock();
                c->g->unlock();
            }
            return record(c->l, it);
        },
        &ctx);
    for (int64_t i = 0; i < 50; ++i) q->execute(i);
    q->stop();  // while 49 tasks wait behind the held one
    q->stop();  // idempotent
    EXPECT_EQ(q->execute(99), EINVAL);
    EXPECT_TRUE(q->stopped());
    gate.unlock();
    q->join();
    EXPECT_EQ(log.seen.size(), 50u);
    EXPECT_EQ(log.stops.load(), 1);
}

TEST(ExecutionQueueDepth, consumer_that_does_not_iterate) {
    // a consumer may return without touching its batch: those tasks are
    // consumed, and the queue keeps serving later ones
    std::atomic<int> calls{0};
    std::atomic<int64_t> got{0};
    struct Ctx {
        std::atomic<int>* calls;
        std::atomic<int64_t>* got;
    } ctx{&calls, &got};
    auto q = Q::Create(
        [](void* m, Q::Iterator& it) -> int {
            Ctx* c = static_cast<Ctx*>(m);
            if (it.is_queue_stopped()) return 0;
            if (c->calls->fetch_add(1) == 0) return 0;  // skip the first batch entirely
            for (; it; ++it) c->got->fetch_add(*it);
            return 0;
        },
        &ctx);
    q->execute(1000);
    for (int i = 0; i < 200 && calls.load() == 0; ++i) ::usleep(1000);
    ASSERT_GT(calls.load(), 0);
    q->execute(5);
    q->execute(6);
    q->stop();
    q->join();
    EXPECT_EQ(got.load(), 11);
}

TEST(ExecutionQueueDepth, execute_from_inside_the_consumer) {
    struct Ctx {
        std::shared_ptr<Q> q;
        std::atomic<int64_t> sum{0};
        std::atomic<int> n{0};
    } ctx;
    ctx.q = Q::Create(
        [](void* m, Q::Iterator& it) -> int {
            Ctx* c = static_cast<Ctx*>(m);
            if (it.is_queue_stopped()) return 0;
            for (; it; ++it) {
                c->sum.fetch_add(*it);
                if (*it > 0) c->q->execute(*it - 1);  // re-entrant, never blocks
                c->n.fetch_add(1);
            }
            return 0;
        },
        &ctx);
    ctx.q->execute(100);
    for (int i = 0; i < 2000 && ctx.n.load() < 101; ++i) ::usleep(1000);
    EXPECT_EQ(ctx.n.load(), 101);
    EXPECT_EQ(ctx.sum.load(), 5050);
    ctx.q->stop();
    ctx.q->join();
    ctx.q.reset();
}

TEST(ExecutionQueueDepth, cancel_self_reports_running) {
    struct Ctx {
        std::shared_ptr<Q> q;
        Q::TaskHandle h;
        std::atomic<int> rc{-5};
        Mutex ready;
    } ctx;
    ctx.ready.lock();
    ctx.q = Q::Create(
        [](void* m, Q::Iterator& it) -> int {
            Ctx* c = static_cast<Ctx*>(m);
            if (it.is_queue_stopped()) return 0;
            c->ready.lock();  // the handle is published by now
            c->ready.unlock();
            c->rc.store(c->q->cancel(c->h));
            return 0;
        },
        &ctx);
    ASSERT_EQ(ctx.q->execute(1, false, &ctx.h), 0);
    ctx.ready.unlock();
    ctx.q->stop();
    ctx.q->join();
    EXPECT_EQ(ctx.rc.load(), 1);  // it is the running task
    ctx.q.reset();
}

TEST(ExecutionQueueDepth, random_cancel_under_load) {
    Log log;
    auto q = Q::Create(record, &log);
    const int N = 20000;
    std::vector<Q::TaskHandle> hs(N);
    std::mt19937 rng(7);
    std::set<int64_t> cancelled;
    for (int i = 0; i < N; ++i) {
        ASSERT_EQ(q->execute(i, (rng() % 5) == 0, &hs[i]), 0);
        if (i >= 10 && rng() % 3 == 0) {
            const int k = (int)(rng() % (uint32_t)i);
            if (q->cancel(hs[k]) == 0) cancelled.insert(k);
        }
    }
    q->stop();
    q->join();
    std::set<int64_t> ran(log.seen.begin(), log.seen.end());
    EXPECT_EQ(ran.size(), log.seen.size());  // nothing ran twice
    EXPECT_EQ(ran.size() + cancelled.size(), (size_t)N);
    for (int64_t c : cancelled) EXPECT_EQ(ran.count(c), 0u);
    EXPECT_FALSE(cancelled.empty());
}

TEST(ExecutionQueueDepth, cancel_queued_high_priority_tasks) {
    Log log;
    Mutex gate;
    gate.lock();
    struct Ctx {
        Log* l;
        Mutex* g;
        bool first = true;
    } ctx{&log, &gate};
    auto q = Q::Create(
        [](void* m, Q::Iterator& it) -> int {
            Ctx* c = static_cast<Ctx*>(m);
            if (c->first && !it.is_queue_stopped()) {
                c->first = false;
                c->g->lock();
                c->g->unlock();
            }
            return record(c->l, it);
        },
        &ctx);
    q->execute(0);
    ::usleep(10000);
    std::vector<Q::TaskHandle> hi(10);
    for (int i = 0; i < 10; ++i) q->execute(100 + i, true, &hi[i]);
    q->execute(1);
    EXPECT_EQ(q->pending(), 11u);
    for (int i = 0; i < 10; i += 2) EXPECT_EQ(q->cancel(hi[i]), 0);
    EXPECT_EQ(q->pending(), 6u);
    gate.unlock();
    q->stop();
    q->join();
    const std::vector<int64_t> want = {0, 101, 103, 105, 107, 109, 1};
    EXPECT_EQ(log.seen.size(), want.size());
    for (size_t i = 0; i < want.size() && i < log.seen.size(); ++i) EXPECT_EQ(log.seen[i], want[i]);
}

TEST(ExecutionQueueDepth, many_short_lived_queues) {
    std::atomic<int64_t> total{0};
    for (int round = 0; round < 200; ++round) {
        auto q = Q::Create(
            [](void* m, Q::Iterator& it) -> int {
                if (it.is_queue_stopped()) return 0;
                for (; it; ++it) static_cast<std::atomic<int64_t>*>(m)->fetch_add(*it);
                return 0;
            },
            &total);
        for (int i = 1; i <= 10; ++i) q->execute(i);
        q->stop();
        q->join();
    }
    EXPECT_EQ(total.load(), 200 * 55);
}
