// More container cases (base/containers.h), after the reference's
// test/flat_map_unittest.cpp, bounded_queue_unittest.cpp,
// mru_cache_unittest.cpp, linked_list_unittest.cpp and
// doubly_buffered_data_unittest.cpp: load factor and growth, erase while
// probing wraps the table end, custom hashes, for_each on a const map,
// queue full/empty edges with move-only payloads, MRU overwrite/peek/erase,
// intrusive list splicing, and DoublyBufferedData modifications that
// refuse, run twice, and survive instances coming and going per thread.
#include <map>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "base/containers.h"
#include "tests/test.h"

using namespace mrpc;

namespace {
// Sends every key to the same home slot: the worst probe chain.
struct ConstHash {
    size_t operator()(int) const { return 3; }
};
// Homes near the end of the table so probe chains wrap to slot 0.
struct TailHash {
    size_t operator()(int k) const { return (size_t)(1000000 - 1 - (k % 3)); }
};
}  // namespace

TEST(ContainersMore, buckets_are_a_power_of_two_and_grow_before_the_load_factor) {
    FlatMap<int, int> m(10, 50);
    EXPECT_EQ(m.bucket_count(), 16u);
    for (int i = 0; i < 8; ++i) m[i] = i;
    EXPECT_EQ(m.bucket_count(), 16u);
    m[8] = 8;  // 9 > 16 * 50%
    EXPECT_EQ(m.bucket_count(), 32u);
    for (int i = 0; i < 9; ++i) EXPECT_EQ(*m.seek(i), i);
}

TEST(ContainersMore, tiny_initial_size_is_rounded_up) {
    FlatMap<int, int> m(1);
    EXPECT_EQ(m.bucket_count(), 8u);
    for (int i = 0; i < 1000; ++i) m[i] = -i;
    EXPECT_EQ(m.size(), 1000u);
    EXPECT_TRUE(m.bucket_count() * 70 >= 1000 * 100);
}

TEST(ContainersMore, one_home_slot_for_every_key) {
    FlatMap<int, int, ConstHash> m(64);
    for (int i = 0; i < 40; ++i) m[i] = i * 10;
    for (int i = 0; i < 40; i += 2) EXPECT_EQ(m.erase(i), 1u);
    for (int i = 0; i < 40; ++i) {
        if (i % 2) {
            ASSERT_TRUE(m.seek(i) != nullptr);
            EXPECT_EQ(*m.seek(i), i * 10);
        } else {
            EXPECT_TRUE(m.seek(i) == nullptr);
        }
    }
    EXPECT_EQ(m.size(), 20u);
}

TEST(ContainersMore, probe_chains_wrapping_the_table_end_survive_erase) {
    FlatMap<int, int, TailHash> m(32, 90);
    for (int i = 0; i < 20; ++i) m[i] = i;
    std::mt19937 rng(7);
    std::vector<int> keys;
    for (int i = 0; i < 20; ++i) keys.push_back(i);
    std::shuffle(keys.begin(), keys.end(), rng);
    std::map<int, int> oracle;
    for (int i = 0; i < 20; ++i) oracle[i] = i;
    for (int k : keys) {
        EXPECT_EQ(m.erase(k), 1u);
        oracle.erase(k);
        for (auto& kv : oracle) {
            const int* v = m.seek(kv.first);
            ASSERT_TRUE(v != nullptr);
            EXPECT_EQ(*v, kv.second);
        }
    }
    EXPECT_TRUE(m.empty());
}

TEST(ContainersMore, erase_of_a_missing_key_changes_nothing) {
    FlatMap<std::string, int> m;
    m["a"] = 1;
    EXPECT_EQ(m.erase("b"), 0u);
    EXPECT_EQ(m.size(), 1u);
    EXPECT_EQ(m.erase("a"), 1u);
    EXPECT_EQ(m.erase("a"), 0u);
    EXPECT_TRUE(m.empty());
}

TEST(ContainersMore, insert_overwrites_and_returns_the_slot) {
    FlatMap<int, std::string> m;
    std::string* p = m.insert(1, "one");
    EXPECT_EQ(*p, "one");
    p = m.insert(1, "uno");
    EXPECT_EQ(*m.seek(1), "uno");
    EXPECT_EQ(m.size(), 1u);
}

TEST(ContainersMore, const_for_each_and_iterator_agree) {
    FlatMap<int, int> m;
    for (int i = 0; i < 300; ++i) m[i * 7] = i;
    const FlatMap<int, int>& cm = m;
    long sum_a = 0, sum_b = 0;
    size_t n_a = 0, n_b = 0;
    cm.for_each([&](const int& k, const int& v) {
        sum_a += k + v;
        ++n_a;
    });
    for (auto it = m.begin(); it != m.end(); ++it) {
        sum_b += it->first + it->second;
        ++n_b;
    }
    EXPECT_EQ(n_a, 300u);
    EXPECT_EQ(n_b, 300u);
    EXPECT_EQ(sum_a, sum_b);
    EXPECT_TRUE(m.contains(7 * 299));
    EXPECT_FALSE(cm.contains(1));
}

TEST(ContainersMore, clear_then_reuse_keeps_the_buckets) {
    FlatMap<int, std::string> m;
    for (int i = 0; i < 100; ++i) m[i] = std::string(20, 'x');
    size_t buckets = m.bucket_count();
    m.clear();
    EXPECT_TRUE(m.empty());
    EXPECT_EQ(m.bucket_count(), buckets);
    EXPECT_TRUE(m.begin() == m.end());
    m[5] = "five";
    EXPECT_EQ(m.size(), 1u);
    EXPECT_EQ(*m.seek(5), "five");
}

TEST(ContainersMore, case_ignored_map_keeps_the_first_spelling) {
    CaseIgnoredFlatMap<int> m;
    m["Accept-Encoding"] = 1;
    m["ACCEPT-ENCODING"] = 2;
    EXPECT_EQ(m.size(), 1u);
    std::string key;
    m.for_each([&](const std::string& k, const int& v) {
        key = k;
        EXPECT_EQ(v, 2);
    });
    EXPECT_EQ(key, "Accept-Encoding");
    EXPECT_EQ(m.erase("accept-encoding"), 1u);
    EXPECT_TRUE(m.empty());
}

TEST(ContainersMore, bounded_queue_of_capacity_one) {
    BoundedQueue<int> q(1);
    EXPECT_TRUE(q.empty());
    EXPECT_TRUE(q.push(1));
    EXPECT_TRUE(q.full());
    EXPECT_FALSE(q.push(2));
    int v = 0;
    EXPECT_TRUE(q.pop(&v));
    EXPECT_EQ(v, 1);
    EXPECT_FALSE(q.pop(&v));
    for (int i = 0; i < 100; ++i) {
        EXPECT_TRUE(q.push(i));
        EXPECT_TRUE(q.pop(&v));
        EXPECT_EQ(v, i);
    }
}

TEST(ContainersMore, bounded_queue_fifo_against_a_model) {
    BoundedQueue<std::string> q(17);
    std::vector<std::string> model;
    std::mt19937 rng(3);
    for (int step = 0; step < 5000; ++step) {
        if (rng() % 3) {
            std::string s = std::to_string(step);
            bool ok = q.push(s);
            EXPECT_EQ(ok, model.size() < 17);
            if (ok) model.push_back(s);
        } else {
            std::string s;
            bool ok = q.pop(&s);
            EXPECT_EQ(ok, !model.empty());
            if (ok) {
                EXPECT_EQ(s, model.front());
                model.erase(model.begin());
            }
        }
        EXPECT_EQ(q.size(), model.size());
    }
    EXPECT_EQ(q.capacity(), 17u);
}

TEST(ContainersMore, mru_overwrite_refreshes_and_does_not_evict) {
    MRUCache<int, std::string> c(2);
    EXPECT_FALSE(c.Put(1, "a"));
    EXPECT_FALSE(c.Put(2, "b"));
    EXPECT_FALSE(c.Put(1, "A"));  // 1 is now the most recent
    int evicted = -1;
    EXPECT_TRUE(c.Put(3, "c", &evicted));
    EXPECT_EQ(evicted, 2);
    EXPECT_EQ(*c.Get(1), "A");
    EXPECT_TRUE(c.Get(2) == nullptr);
}

TEST(ContainersMore, mru_peek_does_not_refresh) {
    MRUCache<int, int> c(2);
    c.Put(1, 10);
    c.Put(2, 20);
    EXPECT_EQ(*c.Peek(1), 10);  // 1 stays least recent
    int evicted = -1;
    c.Put(3, 30, &evicted);
    EXPECT_EQ(evicted, 1);
    std::vector<int> order;
    c.for_each([&](const int& k, const int&) { order.push_back(k); });
    EXPECT_EQ(order.size(), 2u);
    EXPECT_EQ(order[0], 3);
    EXPECT_EQ(order[1], 2);
}

TEST(ContainersMore, mru_erase_and_clear_and_zero_capacity) {
    MRUCache<std::string, int> c(0);  // treated as 1
    EXPECT_EQ(c.capacity(), 1u);
    c.Put("x", 1);
    c.Put("y", 2);
    EXPECT_EQ(c.size(), 1u);
    EXPECT_TRUE(c.Get("x") == nullptr);
    EXPECT_TRUE(c.Erase("y"));
    EXPECT_FALSE(c.Erase("y"));
    c.Put("z", 3);
    c.clear();
    EXPECT_EQ(c.size(), 0u);
    EXPECT_TRUE(c.Peek("z") == nullptr);
}

TEST(ContainersMore, intrusive_list_insert_remove_and_walk) {
    struct Item {
        LinkNode node;
        int v;
    };
    LinkNode head;
    EXPECT_TRUE(head.empty());
    Item items[5];
    for (int i = 0; i < 5; ++i) {
        items[i].v = i;
        items[i].node.insert_before(&head);  // append at the tail
    }
    EXPECT_FALSE(head.empty());
    items[2].node.remove();
    EXPECT_TRUE(items[2].node.empty());
    items[2].node.remove();  // removing a detached node is harmless
    std::vector<int> seen;
    for (LinkNode* n = head.next; n != &head; n = n->next) {
        seen.push_back(reinterpret_cast<Item*>(n)->v);
    }
    std::vector<int> want = {0, 1, 3, 4};
    EXPECT_TRUE(seen == want);
    // walk backwards
    seen.clear();
    for (LinkNode* n = head.prev; n != &head; n = n->prev) seen.push_back(reinterpret_cast<Item*>(n)->v);
    want = {4, 3, 1, 0};
    EXPECT_TRUE(seen == want);
    items[0].node.remove();  // move 0 before 4
    items[0].node.insert_before(&items[4].node);
    seen.clear();
    for (LinkNode* n = head.next; n != &head; n = n->next) seen.push_back(reinterpret_cast<Item*>(n)->v);
    want = {1, 3, 0, 4};
    EXPECT_TRUE(seen == want);
}

TEST(ContainersMore, doubly_buffered_modify_returning_zero_changes_nothing) {
    DoublyBufferedData<std::vector<int>> d;
    d.Modify([](std::vector<int>& v) {
        v.push_back(1);
        return (size_t)1;
    });
    size_t calls = 0;
    size_t r = d.Modify([&](std::vector<int>& v) {
        ++calls;
        (void)v;
        return (size_t)0;
    });
    EXPECT_EQ(r, 0u);
    EXPECT_EQ(calls, 1u);  // the foreground is never touched
    DoublyBufferedData<std::vector<int>>::ScopedPtr p;
    d.Read(&p);
    EXPECT_EQ(p->size(), 1u);
}

TEST(ContainersMore, doubly_buffered_modify_runs_on_both_copies) {
    DoublyBufferedData<int> d;
    size_t calls = 0;
    d.Modify([&](int& v) {
        ++calls;
        v += 5;
        return (size_t)1;
    });
    EXPECT_EQ(calls, 2u);
    {
        DoublyBufferedData<int>::ScopedPtr p;
        d.Read(&p);
        EXPECT_EQ(*p, 5);
    }
    d.Modify([](int& v) {
        v *= 2;
        return (size_t)1;
    });
    DoublyBufferedData<int>::ScopedPtr p;
    d.Read(&p);
    EXPECT_EQ(*p, 10);
}

TEST(ContainersMore, doubly_buffered_instances_come_and_go_per_thread) {
    for (int round = 0; round < 20; ++round) {
        auto d = std::make_unique<DoublyBufferedData<int>>();
        d->Modify([round](int& v) {
            v = round;
            return (size_t)1;
        });
        std::thread t([&] {
            DoublyBufferedData<int>::ScopedPtr p;
            d->Read(&p);
            EXPECT_EQ(*p, round);
        });
        t.join();
        DoublyBufferedData<int>::ScopedPtr p;
        d->Read(&p);
        EXPECT_EQ(*p, round);
    }
}

TEST(ContainersMore, doubly_buffered_modify_waits_for_a_held_reader) {
    DoublyBufferedData<int> d;
    std::atomic<bool> reading{false}, release{false}, modified{false};
    std::thread reader([&] {
        DoublyBufferedData<int>::ScopedPtr p;
        d.Read(&p);
        reading = true;
        while (!release) std::this_thread::yield();
        EXPECT_EQ(*p, 0);  // the version it started on stays intact
    });
    while (!reading) std::this_thread::yield();
    std::thread writer([&] {
        d.Modify([](int& v) {
            v = 1;
            return (size_t)1;
        });
        modified = true;
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(30));
    EXPECT_FALSE(modified.load());
    release = true;
    reader.join();
    writer.join();
    EXPECT_TRUE(modified.load());
    DoublyBufferedData<int>::ScopedPtr p;
    d.Read(&p);
    EXPECT_EQ(*p, 1);
}
