// Container depth (base/containers.h), in the spirit of the reference's
// test/flat_map_unittest.cpp, bounded_queue_unittest.cpp,
// mru_cache_unittest.cpp and doubly_buffered_data_unittest.cpp: values
// initialized on first access, copies and swaps, case-ignored keys,
// removal under probe chains against std::map as an oracle, iteration,
// MRU eviction order, ring wrap-around and concurrent read/modify.
#include <atomic>
#include <map>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "base/containers.h"
#include "tests/test.h"

using namespace mrpc;

TEST(ContainersDepth, values_are_initialized_on_first_access) {
    FlatMap<int, int> m;
    EXPECT_EQ(m[7], 0);
    m[7] += 3;
    EXPECT_EQ(m[7], 3);
    FlatMap<int, std::string> s;
    EXPECT_TRUE(s[1].empty());
    struct P {
        int a = 11;
        std::vector<int> v;
    };
    FlatMap<int, P> p;
    EXPECT_EQ(p[5].a, 11);
    EXPECT_TRUE(p[5].v.empty());
    EXPECT_EQ(p.size(), 1u);
}

TEST(ContainersDepth, copy_and_swap_are_independent) {
    FlatMap<std::string, int> a;
    for (int i = 0; i < 100; ++i) a["k" + std::to_string(i)] = i;
    FlatMap<std::string, int> b = a;  // deep copy
    b["k5"] = -5;
    b.erase("k6");
    EXPECT_EQ(*a.seek("k5"), 5);
    EXPECT_TRUE(a.contains("k6"));
    EXPECT_EQ(b.size(), 99u);
    FlatMap<std::string, int> c;
    c["only"] = 1;
    c.swap(a);
    EXPECT_EQ(c.size(), 100u);
    EXPECT_EQ(a.size(), 1u);
    EXPECT_EQ(*a.seek("only"), 1);
    EXPECT_EQ(*c.seek("k99"), 99);
}

TEST(ContainersDepth, case_ignored_keys) {
    CaseIgnoredFlatMap<int> m;
    m["Content-Type"] = 1;
    m["content-length"] = 2;
    EXPECT_EQ(*m.seek("CONTENT-TYPE"), 1);
    EXPECT_EQ(*m.seek("Content-Length"), 2);
    m["CONTENT-type"] = 3;  // the same key
    EXPECT_EQ(m.size(), 2u);
    EXPECT_EQ(*m.seek("content-type"), 3);
    EXPECT_EQ(m.erase("CoNtEnT-LeNgTh"), 1u);
    EXPECT_FALSE(m.contains("content-length"));
}

TEST(ContainersDepth, random_insert_erase_matches_std_map) {
    FlatMap<uint64_t, uint64_t> m(4);
    std::map<uint64_t, uint64_t> ref;
    std::mt19937_64 rng(42);
    for (int i = 0; i < 200000; ++i) {
        const uint64_t k = rng() % 5000;  // dense keys: long probe chains and shifts
        switch (rng() % 3) {
            case 0:
                m[k] = (uint64_t)i;
                ref[k] = (uint64_t)i;
                break;
            case 1:
                ASSERT_EQ(m.erase(k), ref.erase(k));
                break;
            default: {
                const uint64_t* v = m.seek(k);
                auto it = ref.find(k);
                ASSERT_EQ(v != nullptr, it != ref.end());
                if (v) ASSERT_EQ(*v, it->second);
            }
        }
    }
    ASSERT_EQ(m.size(), ref.size());
    size_t n = 0;
    m.for_each([&](const uint64_t& k, const uint64_t& v) {
        ++n;
        auto it = ref.find(k);
        EXPECT_TRUE(it != ref.end() && it->second == v);
    });
    EXPECT_EQ(n, ref.size());
}

TEST(ContainersDepth, colliding_hashes_survive_erase_shifts) {
    struct Bad {
        size_t operator()(int) const { return 7; }  // every key on one chain
    };
    FlatMap<int, int, Bad> m;
    for (int i = 0; i < 40; ++i) m[i] = i * 10;
    for (int i = 0; i < 40; i += 3) EXPECT_EQ(m.erase(i), 1u);
    for (int i = 0; i < 40; ++i) {
        const int* v = m.seek(i);
        if (i % 3 == 0) {
            EXPECT_TRUE(v == nullptr);
        } else {
            ASSERT_TRUE(v != nullptr);
            EXPECT_EQ(*v, i * 10);
        }
    }
}

TEST(ContainersDepth, iteration_visits_each_entry_and_allows_updates) {
    FlatMap<int, int> m;
    for (int i = 0; i < 1000; ++i) m[i * 7] = i;
    std::set<int> seen;
    for (auto it = m.begin(); it != m.end(); ++it) {
        EXPECT_TRUE(seen.insert(it->first).second);
        it->second += 1;  // values are writable in place
    }
    EXPECT_EQ(seen.size(), 1000u);
    EXPECT_EQ(*m.seek(7 * 500), 501);
    // erasing a collected key set after the walk (the safe pattern)
    std::vector<int> odd;
    for (auto& kv : m) {
        if (kv.second % 2) odd.push_back(kv.first);
    }
    for (int k : odd) m.erase(k);
    EXPECT_EQ(m.size(), 500u);
}

TEST(ContainersDepth, growth_keeps_every_entry_and_clear_resets) {
    FlatMap<std::string, int> m(2);
    const size_t b0 = m.bucket_count();
    for (int i = 0; i < 10000; ++i) m["key" + std::to_string(i)] = i;
    EXPECT_GT(m.bucket_count(), b0);
    EXPECT_LE(m.size() * 100, m.bucket_count() * 70);  // the load factor holds
    for (int i = 0; i < 10000; ++i) ASSERT_EQ(*m.seek("key" + std::to_string(i)), i);
    m.clear();
    EXPECT_TRUE(m.empty());
    EXPECT_FALSE(m.contains("key1"));
    m["again"] = 1;
    EXPECT_EQ(m.size(), 1u);
}

TEST(ContainersDepth, bounded_queue_wraps_around) {
    BoundedQueue<int> q(4);
    int out = -1;
    EXPECT_FALSE(q.pop(&out));
    for (int round = 0; round < 10; ++round) {
        for (int i = 0; i < 3; ++i) EXPECT_TRUE(q.push(round * 10 + i));
        for (int i = 0; i < 3; ++i) {
            ASSERT_TRUE(q.pop(&out));
            EXPECT_EQ(out, round * 10 + i);
        }
    }
    for (int i = 0; i < 4; ++i) EXPECT_TRUE(q.push(i));
    EXPECT_TRUE(q.full());
    EXPECT_FALSE(q.push(99));
    EXPECT_EQ(q.size(), 4u);
    EXPECT_EQ(q.capacity(), 4u);
}

TEST(ContainersDepth, mru_cache_evicts_the_least_recent) {
    MRUCache<int, std::string> c(3);
    int evicted = -1;
    EXPECT_FALSE(c.Put(1, "a", &evicted));
    c.Put(2, "b");
    c.Put(3, "c");
    ASSERT_TRUE(c.Get(1) != nullptr);  // 1 becomes the most recent
    EXPECT_TRUE(c.Put(4, "d", &evicted));
    EXPECT_EQ(evicted, 2);  // 2 was the least recent
    EXPECT_TRUE(c.Peek(2) == nullptr);
    EXPECT_TRUE(c.Peek(3) != nullptr);  // Peek does not refresh
    c.Put(5, "e", &evicted);
    EXPECT_EQ(evicted, 3);
    EXPECT_TRUE(c.Erase(1));
    EXPECT_FALSE(c.Erase(1));
    EXPECT_EQ(c.size(), 2u);
    c.Put(4, "dd");  // an update, not an insert
    EXPECT_EQ(*c.Get(4), "dd");
    EXPECT_EQ(c.size(), 2u);
}

TEST(ContainersDepth, doubly_buffered_data_readers_see_whole_versions) {
    DoublyBufferedData<std::vector<int>> d;
    d.Modify([](std::vector<int>& v) {
        v.assign(64, 0);
        return 1;
    });
    std::atomic<bool> stop{false};
    std::atomic<int> torn{0}, reads{0};
    std::vector<std::thread> readers;
    for (int t = 0; t < 4; ++t) {
        readers.emplace_back([&] {
            while (!stop.load(std::memory_order_relaxed)) {
                DoublyBufferedData<std::vector<int>>::ScopedPtr p;
                if (d.Read(&p) != 0) continue;
                const std::vector<int>& v = *p;
                for (int x : v) {
                    if (x != v[0]) {
                        torn.fetch_add(1);
                        break;
                    }
                }
                reads.fetch_add(1);
            }
        });
    }
    while (reads.load() < 8) std::this_thread::yield();  // readers are running
    for (int gen = 1; gen <= 300; ++gen) {
        if (gen % 30 == 0) std::this_thread::yield();
        d.Modify([gen](std::vector<int>& v) {
            for (int& x : v) x = gen;
            return 1;
        });
    }
    stop = true;
    for (auto& t : readers) t.join();
    EXPECT_EQ(torn.load(), 0);
    EXPECT_GT(reads.load(), 0);
    DoublyBufferedData<std::vector<int>>::ScopedPtr p;
    ASSERT_EQ(d.Read(&p), 0);
    EXPECT_EQ((*p)[63], 300);
}
