// Unit tests for the base layer (spirit of reference test/iobuf_unittest.cpp,
// crc32c_unittest.cc, flat_map_unittest.cpp, endpoint_unittest.cpp).
#include <fcntl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <map>
#include <thread>

#include "base/buf.h"
#include "base/containers.h"
#include "base/crc32c.h"
#include "base/endpoint.h"
#include "base/flags.h"
#include "base/time.h"
#include "rpc/periodic_task.h"
#include "base/pool.h"
#include "base/util.h"
#include "tests/test.h"

using namespace mrpc;

DEFINE_int32(test_reloadable_flag, 5, "for tests");
MRPC_VALIDATE_FLAG(test_reloadable_flag, PositiveIntegerValidator);
DEFINE_string(test_string_flag, "abc", "for tests");

TEST(Buf, append_and_cut) {
    Buf b;
    EXPECT_TRUE(b.empty());
    b.append("hello ");
    b.append(std::string("world"));
    EXPECT_EQ(b.size(), 11u);
    EXPECT_EQ(b.to_string(), "hello world");
    Buf head;
    EXPECT_EQ(b.cutn(&head, 6), 6u);
    EXPECT_EQ(head.to_string(), "hello ");
    EXPECT_EQ(b.to_string(), "world");
    char c;
    EXPECT_TRUE(b.cut1(&c));
    EXPECT_EQ(c, 'w');
    EXPECT_EQ(b.pop_back(1), 1u);
    EXPECT_EQ(b.to_string(), "orl");
}

TEST(Buf, large_and_many_blocks) {
    std::string big(300000, 'x');
    for (size_t i = 0; i < big.size(); ++i) big[i] = (char)(i * 131 + 7);
    Buf b;
    for (size_t off = 0; off < big.size(); off += 1000) b.append(big.data() + off, std::min<size_t>(1000, big.size() - off));
    EXPECT_EQ(b.size(), big.size());
    EXPECT_TRUE(b.equals(big));
    Buf copy = b;
    EXPECT_TRUE(copy.equals(big));
    std::string out;
    b.cutn(&out, 12345);
    EXPECT_EQ(out, big.substr(0, 12345));
    EXPECT_EQ(b.size(), big.size() - 12345);
    char tmp[100];
    const char* p = (const char*)b.fetch(tmp, 100);
    EXPECT_EQ(std::string(p, 100), big.substr(12345, 100));
    Buf one;
    one.append(big.data(), big.size());  // >= 64KB: one dedicated block
    EXPECT_EQ(one.backing_block_num(), 1u);
    EXPECT_TRUE(one.equals(big));
}

TEST(Buf, user_data_and_portal) {
    static int deleted = 0;
    char* mem = (char*)malloc(64);
    memcpy(mem, "0123456789", 10);
    {
        Buf b;
        b.append_user_data(mem, 10, [](void* d, void*) { free(d); ++deleted; });
        Buf c;
        b.cutn(&c, 4);
        EXPECT_EQ(c.to_string(), "0123");
        EXPECT_EQ(b.to_string(), "456789");
    }
    EXPECT_EQ(deleted, 1);
    int fds[2];
    ASSERT_EQ(socketpair(AF_UNIX, SOCK_STREAM, 0, fds), 0);
    Buf w;
    std::string payload(50000, 'p');
    w.append(payload);
    w.append("tail");
    size_t total = w.size();
    size_t sent = 0;
    BufPortal r;
    while (sent < total || r.size() < total) {
        if (sent < total) {
            ssize_t n = w.cut_into_fd(fds[0]);
            if (n > 0) sent += n;
        }
        ssize_t m = r.append_from_fd(fds[1], 65536);
        if (m <= 0 && sent >= total && r.size() >= total) break;
    }
    EXPECT_EQ(r.size(), total);
    EXPECT_TRUE(r.equals(payload + "tail"));
    close(fds[0]);
    close(fds[1]);
}

TEST(Buf, cut_until_and_iterator) {
    Buf b;
    b.append("GET / HTTP/1.1\r\nHost: x\r\n\r\nbody");
    Buf line;
    EXPECT_EQ(b.cut_until(&line, "\r\n"), 0);
    EXPECT_EQ(line.to_string(), "GET / HTTP/1.1");
    BufBytesIterator it(b);
    std::string s;
    while (!it.done()) { s.push_back(*it); ++it; }
    EXPECT_EQ(s, "Host: x\r\n\r\nbody");
}

TEST(Buf, multi_thread_refcount) {
    Buf shared;
    shared.append(std::string(20000, 'z'));
    std::vector<std::thread> ths;
    for (int t = 0; t < 4; ++t) {
        ths.emplace_back([&shared] {
            for (int i = 0; i < 2000; ++i) {
                Buf c = shared;
                Buf d;
                c.cutn(&d, 100);
                d.append("abc");
            }
        });
    }
    for (auto& t : ths) t.join();
    EXPECT_EQ(shared.size(), 20000u);
}

TEST(Crc32c, known_values) {
    // Standard check value for "123456789"
    EXPECT_EQ(crc32c::Value("123456789", 9), 0xE3069283u);
    char zeros[32] = {0};
    EXPECT_EQ(crc32c::Value(zeros, 32), 0x8A9136AAu);
    std::string a = "hello, ", b = "world of crc";
    uint32_t whole = crc32c::Value((a + b).data(), a.size() + b.size());
    EXPECT_EQ(crc32c::Extend(crc32c::Value(a.data(), a.size()), b.data(), b.size()), whole);
    EXPECT_EQ(crc32c::Combine(crc32c::Value(a.data(), a.size()), crc32c::Value(b.data(), b.size()), b.size()), whole);
}

TEST(FlatMap, basic) {
    FlatMap<int, std::string> m;
    for (int i = 0; i < 1000; ++i) m[i] = std::to_string(i);
    EXPECT_EQ(m.size(), 1000u);
    for (int i = 0; i < 1000; i += 2) EXPECT_EQ(m.erase(i), 1u);
    EXPECT_EQ(m.size(), 500u);
    for (int i = 0; i < 1000; ++i) {
        if (i % 2) {
            ASSERT_TRUE(m.seek(i) != nullptr);
            EXPECT_EQ(*m.seek(i), std::to_string(i));
        } else {
            EXPECT_TRUE(m.seek(i) == nullptr);
        }
    }
    size_t n = 0;
    for (auto& kv : m) { (void)kv; ++n; }
    EXPECT_EQ(n, 500u);
    CaseIgnoredFlatMap<int> cm;
    cm["Content-Type"] = 3;
    EXPECT_TRUE(cm.seek("content-type") != nullptr);
}

TEST(DoublyBufferedData, read_modify) {
    DoublyBufferedData<std::vector<int>> d;
    d.Modify([](std::vector<int>& v) { v.push_back(1); return (size_t)1; });
    std::atomic<bool> stop{false};
    std::thread reader([&] {
        while (!stop) {
            DoublyBufferedData<std::vector<int>>::ScopedPtr p;
            d.Read(&p);
            EXPECT_GE(p->size(), 1u);
        }
    });
    for (int i = 0; i < 100; ++i) d.Modify([i](std::vector<int>& v) { v.push_back(i); return (size_t)1; });
    stop = true;
    reader.join();
    DoublyBufferedData<std::vector<int>>::ScopedPtr p;
    d.Read(&p);
    EXPECT_EQ(p->size(), 101u);
}

TEST(EndPoint, parse) {
    EndPoint ep;
    EXPECT_EQ(str2endpoint("127.0.0.1:8080", &ep), 0);
    EXPECT_EQ(ep.port, 8080);
    EXPECT_EQ(ep.to_string(), "127.0.0.1:8080");
    EXPECT_NE(str2endpoint("1.2.3:80", &ep), 0);
    EXPECT_EQ(str2endpoint("unix:/tmp/x.sock", &ep), 0);
    EXPECT_TRUE(ep.is_unix());
    EXPECT_EQ(hostname2endpoint("localhost:99", &ep), 0);
    EXPECT_EQ(ep.port, 99);
}

TEST(Flags, set_and_validate) {
    std::string v;
    EXPECT_TRUE(GetFlag("test_reloadable_flag", &v));
    EXPECT_EQ(v, "5");
    EXPECT_TRUE(SetFlag("test_reloadable_flag", "7", true));
    EXPECT_EQ(FLAGS_test_reloadable_flag, 7);
    EXPECT_FALSE(SetFlag("test_reloadable_flag", "-1", true));
    EXPECT_FALSE(SetFlag("test_string_flag", "x", true));  // not reloadable
    EXPECT_TRUE(SetFlag("test_string_flag", "x", false));
    EXPECT_EQ(FLAGS_test_string_flag, "x");
    EXPECT_FALSE(SetFlag("no_such_flag", "1"));
}

TEST(Util, hashing_and_strings) {
    EXPECT_EQ(murmurhash3_32("hello", 5, 0), 0x248bfa47u);
    EXPECT_EQ(base64_encode("hello", 5), "aGVsbG8=");
    std::string d;
    EXPECT_TRUE(base64_decode("aGVsbG8=", &d));
    EXPECT_EQ(d, "hello");
    auto parts = split_string("a,b,,c", ',');
    EXPECT_EQ(parts.size(), 3u);
    EXPECT_EQ(url_decode("a%20b+c"), "a b c");
    uint64_t hist[10] = {0};
    for (int i = 0; i < 10000; ++i) ++hist[fast_rand_less_than(10)];
    for (int i = 0; i < 10; ++i) EXPECT_GT(hist[i], 800u);
}

struct PoolObj {
    int v = 0;
};

TEST(ResourcePool, get_put_address) {
    uint32_t ids[100];
    for (int i = 0; i < 100; ++i) {
        PoolObj* o = get_resource<PoolObj>(&ids[i]);
        ASSERT_TRUE(o != nullptr);
        o->v = i;
    }
    for (int i = 0; i < 100; ++i) EXPECT_EQ(address_resource<PoolObj>(ids[i])->v, i);
    for (int i = 0; i < 100; ++i) return_resource<PoolObj>(ids[i]);
    uint32_t id;
    get_resource<PoolObj>(&id);
    bool reused = false;
    for (int i = 0; i < 100; ++i) reused |= (ids[i] == id);
    EXPECT_TRUE(reused);
}

TEST(Base, mru_cache_evicts_least_recent) {
    mrpc::MRUCache<std::string, int> c(3);
    c.Put("a", 1);
    c.Put("b", 2);
    c.Put("c", 3);
    ASSERT_TRUE(c.Get("a") != nullptr);  // a becomes most recent
    std::string ev;
    EXPECT_TRUE(c.Put("d", 4, &ev));
    EXPECT_EQ(ev, "b");
    EXPECT_TRUE(c.Peek("b") == nullptr);
    EXPECT_EQ(*c.Get("a"), 1);
    EXPECT_FALSE(c.Put("a", 10));
    EXPECT_EQ(*c.Peek("a"), 10);
    std::vector<std::string> order;
    c.for_each([&](const std::string& k, int) { order.push_back(k); });
    EXPECT_EQ(order.size(), 3u);
    EXPECT_EQ(order[0], "a");
    EXPECT_TRUE(c.Erase("c"));
    EXPECT_EQ(c.size(), 2u);
}

namespace {
struct CountingTask : public mrpc::PeriodicTask {
    std::atomic<int> runs{0};
    std::atomic<bool> destroyed{false};
    bool OnTriggeringTask(timespec* next) override {
        if (++runs >= 5) return false;
        *next = mrpc::realtime_after_us(2000);
        return true;
    }
    void OnDestroyingTask() override { destroyed = true; }
};
}  // namespace

TEST(Base, periodic_task_runs_until_it_stops) {
    CountingTask t;
    mrpc::PeriodicTaskManager::StartTaskAt(&t, mrpc::realtime_after_us(1000));
    for (int i = 0; i < 500 && !t.destroyed; ++i) usleep(2000);
    EXPECT_TRUE(t.destroyed.load());
    EXPECT_EQ(t.runs.load(), 5);
}
