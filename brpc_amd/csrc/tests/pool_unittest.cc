// Slab pools (base/pool.h), in the spirit of the reference's
// test/resource_pool_unittest.cpp and object_pool_unittest.cpp: stable
// ids and addresses, recycling through the thread-local free list and the
// global overflow, blocks that are never freed, for_each over everything
// constructed, and the pools under concurrent get/put from many threads.
#include <algorithm>
#include <atomic>
#include <set>
#include <thread>
#include <unordered_set>
#include <vector>

#include "base/pool.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

// Each test uses its own type so the singletons start empty.
struct RpA { int v = 0; char pad[60]; };
struct RpB { long v = 0; };
struct RpC { int v = 0; };
struct RpD { int v = 0; };
struct RpE { std::atomic<int> owner{0}; };
struct RpF { int v = 0; };
struct RpG { int v = 0; };
struct OpA { int v = 7; };
struct OpB { std::vector<int> v; };
struct OpC { int v = 0; };
struct OpD { std::atomic<int> owner{0}; };
struct OpE { int v = 0; };

}  // namespace

TEST(PoolResource, ids_map_to_stable_addresses) {
    std::vector<uint32_t> ids;
    std::vector<RpA*> ptrs;
    for (int i = 0; i < 1000; ++i) {
        uint32_t id = 0;
        RpA* p = get_resource<RpA>(&id);
        ASSERT_TRUE(p != nullptr);
        p->v = i;
        ids.push_back(id);
        ptrs.push_back(p);
    }
    std::set<uint32_t> uniq(ids.begin(), ids.end());
    EXPECT_EQ(uniq.size(), ids.size());
    for (size_t i = 0; i < ids.size(); ++i) {
        EXPECT_TRUE(address_resource<RpA>(ids[i]) == ptrs[i]);
        EXPECT_EQ(address_resource<RpA>(ids[i])->v, (int)i);
    }
    for (uint32_t id : ids) return_resource<RpA>(id);
}

TEST(PoolResource, first_ids_are_dense_in_one_block) {
    uint32_t first = 0;
    get_resource<RpB>(&first);
    for (uint32_t i = 1; i < ResourcePool<RpB>::kBlockItems; ++i) {
        uint32_t id = 0;
        get_resource<RpB>(&id);
        EXPECT_EQ(id, first + i);
    }
    EXPECT_TRUE(ResourcePool<RpB>::singleton()->capacity() >= ResourcePool<RpB>::kBlockItems);
}

TEST(PoolResource, returned_ids_are_reused_lifo_on_the_same_thread) {
    uint32_t a = 0, b = 0, c = 0;
    get_resource<RpC>(&a);
    get_resource<RpC>(&b);
    return_resource<RpC>(a);
    return_resource<RpC>(b);
    get_resource<RpC>(&c);
    EXPECT_EQ(c, b);
    get_resource<RpC>(&c);
    EXPECT_EQ(c, a);
}

TEST(PoolResource, objects_keep_their_state_across_recycling) {
    // objects are never destroyed: a recycled slot still holds what the
    // previous owner left (callers reset it, as sockets and fibers do)
    uint32_t id = 0;
    RpD* p = get_resource<RpD>(&id);
    p->v = 1234;
    return_resource<RpD>(id);
    uint32_t id2 = 0;
    RpD* q = get_resource<RpD>(&id2);
    EXPECT_EQ(id2, id);
    EXPECT_TRUE(q == p);
    EXPECT_EQ(q->v, 1234);
}

TEST(PoolResource, out_of_range_ids_have_no_address) {
    EXPECT_TRUE(address_resource<RpF>(ResourcePool<RpF>::kInvalid) == nullptr);
    // a block that was never allocated
    EXPECT_TRUE(address_resource<RpF>((ResourcePool<RpF>::kMaxBlocks - 1) << ResourcePool<RpF>::kBlockShift) ==
                nullptr);
}

TEST(PoolResource, overflow_to_the_global_list_feeds_other_threads) {
    const size_t n = ResourcePool<RpG>::kLocalMax * 3;
    std::vector<uint32_t> ids(n);
    for (size_t i = 0; i < n; ++i) get_resource<RpG>(&ids[i]);
    size_t cap_before = ResourcePool<RpG>::singleton()->capacity();
    for (uint32_t id : ids) return_resource<RpG>(id);
    // another thread takes ids: at least some come from the global list
    // (no new block needed for them)
    std::vector<uint32_t> taken;
    std::thread t([&] {
        for (size_t i = 0; i < ResourcePool<RpG>::kLocalMax / 2; ++i) {
            uint32_t id = 0;
            get_resource<RpG>(&id);
            taken.push_back(id);
        }
    });
    t.join();
    std::set<uint32_t> returned(ids.begin(), ids.end());
    size_t reused = 0;
    for (uint32_t id : taken) reused += returned.count(id);
    EXPECT_EQ(reused, taken.size());
    EXPECT_EQ(ResourcePool<RpG>::singleton()->capacity(), cap_before);
}

TEST(PoolResource, for_each_visits_every_constructed_slot) {
    struct RpH { int v = 0; };
    uint32_t id = 0;
    RpH* p = get_resource<RpH>(&id);
    p->v = 99;
    size_t visited = 0;
    bool seen = false;
    ResourcePool<RpH>::singleton()->for_each([&](uint32_t i, const RpH* x) {
        ++visited;
        if (i == id && x->v == 99) seen = true;
    });
    EXPECT_EQ(visited, ResourcePool<RpH>::singleton()->capacity());
    EXPECT_TRUE(seen);
}

TEST(PoolResource, concurrent_get_put_never_hands_one_slot_to_two_owners) {
    std::atomic<int> conflicts{0};
    std::vector<std::thread> ts;
    for (int t = 1; t <= 8; ++t) {
        ts.emplace_back([t, &conflicts] {
            std::vector<uint32_t> mine;
            for (int round = 0; round < 2000; ++round) {
                uint32_t id = 0;
                RpE* p = get_resource<RpE>(&id);
                int prev = 0;
                if (!p->owner.compare_exchange_strong(prev, t)) conflicts.fetch_add(1);
                mine.push_back(id);
                if (mine.size() > 50 || (round % 7) == 0) {
                    uint32_t back = mine.front();
                    mine.erase(mine.begin());
                    address_resource<RpE>(back)->owner.store(0);
                    return_resource<RpE>(back);
                }
            }
            for (uint32_t id : mine) {
                address_resource<RpE>(id)->owner.store(0);
                return_resource<RpE>(id);
            }
        });
    }
    for (auto& t : ts) t.join();
    EXPECT_EQ(conflicts.load(), 0);
}

TEST(PoolObject, get_constructs_then_recycles) {
    OpA* a = get_object<OpA>();
    EXPECT_EQ(a->v, 7);
    a->v = 8;
    return_object<OpA>(a);
    OpA* b = get_object<OpA>();
    EXPECT_TRUE(a == b);
    EXPECT_EQ(b->v, 8);  // put() keeps the object as it was
    return_object<OpA>(b);
}

TEST(PoolObject, lifo_reuse_of_a_batch) {
    std::vector<OpB*> v;
    for (int i = 0; i < 10; ++i) v.push_back(get_object<OpB>());
    std::set<OpB*> uniq(v.begin(), v.end());
    EXPECT_EQ(uniq.size(), 10u);
    for (OpB* p : v) return_object<OpB>(p);
    for (int i = 9; i >= 0; --i) {
        OpB* p = get_object<OpB>();
        EXPECT_TRUE(p == v[i]);
    }
    for (OpB* p : v) return_object<OpB>(p);
}

TEST(PoolObject, thread_exit_hands_its_cache_to_the_global_list) {
    std::vector<OpC*> made;
    std::thread t([&] {
        for (int i = 0; i < 20; ++i) made.push_back(get_object<OpC>());
        for (OpC* p : made) return_object<OpC>(p);
    });
    t.join();
    // this thread's cache is empty: its gets come from what the exited
    // thread left behind
    std::set<OpC*> left(made.begin(), made.end());
    for (int i = 0; i < 20; ++i) {
        OpC* p = get_object<OpC>();
        EXPECT_EQ(left.count(p), 1u);
    }
}

TEST(PoolObject, overflow_past_the_local_limit_goes_global) {
    const size_t n = ObjectPool<OpE>::kLocalMax + 30;
    std::vector<OpE*> v;
    for (size_t i = 0; i < n; ++i) v.push_back(get_object<OpE>());
    for (OpE* p : v) return_object<OpE>(p);
    std::set<OpE*> all(v.begin(), v.end());
    std::vector<OpE*> other;
    std::thread t([&] {
        for (int i = 0; i < 30; ++i) other.push_back(get_object<OpE>());
    });
    t.join();
    for (OpE* p : other) EXPECT_EQ(all.count(p), 1u);
}

TEST(PoolObject, concurrent_threads_never_share_an_object) {
    std::atomic<int> conflicts{0};
    std::vector<std::thread> ts;
    for (int t = 1; t <= 8; ++t) {
        ts.emplace_back([t, &conflicts] {
            std::vector<OpD*> held;
            for (int i = 0; i < 3000; ++i) {
                OpD* p = get_object<OpD>();
                int prev = 0;
                if (!p->owner.compare_exchange_strong(prev, t)) conflicts.fetch_add(1);
                held.push_back(p);
                if (held.size() > 80 || i % 3 == 0) {
                    OpD* q = held.back();
                    held.pop_back();
                    q->owner.store(0);
                    return_object<OpD>(q);
                }
            }
            for (OpD* q : held) {
                q->owner.store(0);
                return_object<OpD>(q);
            }
        });
    }
    for (auto& t : ts) t.join();
    EXPECT_EQ(conflicts.load(), 0);
}

// A thread that only gets and a thread that only puts (a socket reader and
// the worker that ran its message): objects cross in batches through the
// global list, none is handed out twice, and recycling keeps the number
// ever constructed bounded by what is in flight plus the two caches.
namespace {
struct OpF {
    static std::atomic<int> constructed;
    std::atomic<int> live{0};
    OpF() { constructed.fetch_add(1); }
};
std::atomic<int> OpF::constructed{0};
}  // namespace

TEST(PoolObject, getter_and_putter_threads_recycle_in_batches) {
    const int kN = 20000, kInFlight = 100;
    std::vector<std::atomic<OpF*>> slots(kInFlight);
    for (auto& s : slots) s.store(nullptr);
    std::atomic<int> dup{0}, got{0};
    std::atomic<bool> done{false};
    std::thread getter([&] {
        for (int i = 0; i < kN; ++i) {
            OpF* p = get_object<OpF>();
            if (p->live.exchange(1) != 0) dup.fetch_add(1);
            std::atomic<OpF*>& s = slots[i % kInFlight];
            while (s.load(std::memory_order_acquire) != nullptr) std::this_thread::yield();
            s.store(p, std::memory_order_release);
            got.fetch_add(1);
        }
        done = true;
    });
    std::thread putter([&] {
        int put = 0;
        while (put < kN) {
            for (auto& s : slots) {
                OpF* p = s.load(std::memory_order_acquire);
                if (!p) continue;
                s.store(nullptr, std::memory_order_release);
                p->live.store(0);
                return_object<OpF>(p);
                ++put;
            }
        }
    });
    getter.join();
    putter.join();
    EXPECT_EQ(got.load(), kN);
    EXPECT_EQ(dup.load(), 0);
    // in flight + the putter's cache + a batch on its way: far below kN
    EXPECT_TRUE(OpF::constructed.load() <= kInFlight + 2 * (int)ObjectPool<OpF>::kLocalMax + 1);
}
