// WorkStealingQueue (fiber/internal.h, the run queue of every worker):
// capacity bounds, LIFO pop / FIFO steal order, and a stress run where one
// owner pushes and pops while several thieves steal — every item must be
// taken exactly once. Parity: reference test/bthread_work_stealing_queue_unittest.cpp.
#include <atomic>
#include <memory>
#include <thread>
#include <vector>

#include "fiber/internal.h"
#include "tests/test.h"

using namespace mrpc::fiber;

TEST(WorkStealingQueue, capacity_and_order) {
    WorkStealingQueue<int> q;
    q.init(8);
    for (int i = 0; i < 8; ++i) ASSERT_TRUE(q.push(i));
    EXPECT_FALSE(q.push(8));  // full
    EXPECT_EQ(q.volatile_size(), 8u);
    int v = -1;
    ASSERT_TRUE(q.pop(&v));
    EXPECT_EQ(v, 7);  // owner: newest first
    ASSERT_TRUE(q.steal(&v));
    EXPECT_EQ(v, 0);  // thief: oldest first
    ASSERT_TRUE(q.push(100));
    ASSERT_TRUE(q.push(101));  // room again after taking two
    EXPECT_FALSE(q.push(102));
    int n = 0;
    while (q.pop(&v)) ++n;
    EXPECT_EQ(n, 8);
    EXPECT_FALSE(q.steal(&v));
    EXPECT_EQ(q.volatile_size(), 0u);
}

TEST(WorkStealingQueue, wraps_around_many_times) {
    WorkStealingQueue<int> q;
    q.init(4);
    int v;
    for (int round = 0; round < 1000; ++round) {
        ASSERT_TRUE(q.push(round));
        ASSERT_TRUE(q.push(round + 1000000));
        ASSERT_TRUE(q.steal(&v));
        EXPECT_EQ(v, round);
        ASSERT_TRUE(q.pop(&v));
        EXPECT_EQ(v, round + 1000000);
    }
}

// The last item: owner pop and thief steal race for it; exactly one wins.
TEST(WorkStealingQueue, last_item_race_has_one_winner) {
    WorkStealingQueue<int> q;
    q.init(2);
    std::atomic<int> round{-1}, stolen{0};
    std::atomic<bool> stop{false};
    std::atomic<int> thief_done{0};
    std::thread thief([&] {
        int seen = -1;
        while (!stop.load(std::memory_order_acquire)) {
            const int r = round.load(std::memory_order_acquire);
            if (r == seen) continue;
            int v;
            if (q.steal(&v)) stolen.fetch_add(1, std::memory_order_relaxed);
            seen = r;
            thief_done.store(r, std::memory_order_release);
        }
    });
    const int kRounds = 20000;
    int popped = 0;
    for (int r = 0; r < kRounds; ++r) {
        ASSERT_TRUE(q.push(r));
        round.store(r, std::memory_order_release);
        int v;
        if (q.pop(&v)) ++popped;
        while (thief_done.load(std::memory_order_acquire) != r) {
        }
        int tmp;
        EXPECT_FALSE(q.pop(&tmp));  // drained either way
    }
    stop.store(true, std::memory_order_release);
    thief.join();
    EXPECT_EQ(popped + stolen.load(), kRounds);
}

TEST(WorkStealingQueue, stress_every_item_taken_exactly_once) {
    const int kItems = 400000;
    const int kThieves = 4;
    WorkStealingQueue<int> q;
    q.init(1024);
    std::unique_ptr<std::atomic<uint8_t>[]> taken(new std::atomic<uint8_t>[kItems]);
    for (int i = 0; i < kItems; ++i) taken[i].store(0, std::memory_order_relaxed);
    std::atomic<bool> producing{true};
    std::atomic<int64_t> by_thieves{0};
    std::vector<std::thread> thieves;
    for (int t = 0; t < kThieves; ++t) {
        thieves.emplace_back([&] {
            int v;
            for (;;) {
                if (q.steal(&v)) {
                    taken[v].fetch_add(1, std::memory_order_relaxed);
                    by_thieves.fetch_add(1, std::memory_order_relaxed);
                } else if (!producing.load(std::memory_order_acquire)) {
                    if (!q.steal(&v)) break;
                    taken[v].fetch_add(1, std::memory_order_relaxed);
                    by_thieves.fetch_add(1, std::memory_order_relaxed);
                }
            }
        });
    }
    int64_t by_owner = 0;
    int next = 0;
    while (next < kItems) {
        // bursts of pushes, then the owner takes some back itself
        const int burst = 1 + (next * 7919) % 64;
        for (int i = 0; i < burst && next < kItems; ++i) {
            if (q.push(next)) {
                ++next;
            } else {
                break;  // full: pop below
            }
        }
        const int pops = (next * 104729) % 5;
        int v;
        for (int i = 0; i < pops && q.pop(&v); ++i) {
            taken[v].fetch_add(1, std::memory_order_relaxed);
            ++by_owner;
        }
    }
    int v;
    while (q.pop(&v)) {
        taken[v].fetch_add(1, std::memory_order_relaxed);
        ++by_owner;
    }
    producing.store(false, std::memory_order_release);
    for (auto& t : thieves) t.join();
    int missing = 0, dup = 0;
    for (int i = 0; i < kItems; ++i) {
        const int c = taken[i].load(std::memory_order_relaxed);
        if (c == 0) ++missing;
        if (c > 1) ++dup;
    }
    EXPECT_EQ(missing, 0);
    EXPECT_EQ(dup, 0);
    EXPECT_EQ(by_owner + by_thieves.load(), (int64_t)kItems);
    EXPECT_GT(by_thieves.load(), 0);
}
