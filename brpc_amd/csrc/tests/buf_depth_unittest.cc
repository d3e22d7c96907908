// Buf depth (base/buf.h), the rest of the reference's IOBuf suite in spirit
// (test/iobuf_unittest.cpp: appendv, reserve, copy_and_assign, compare,
// append_and_cut_it_all, cut_by_single_text_delim, cut_into_fd_tiny,
// cut_into_fd_a_lot_of_data, append_store_append_cut, own_block, swap,
// iterate_bytes, appender, copy_to_string_from_iterator,
// append_user_data_and_consume / _and_share / _with_meta, share_tls_block,
// acquire_tls_block, cut_into_fd_with_offset_multithreaded,
// append_from_fd_with_offset) plus what the MI355X design adds: memory-kind
// tags, the device copy hook, the large-block path and the block allocator.
#include <fcntl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "base/buf.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

std::string pattern(size_t n, uint32_t seed) {
    std::string s(n, '\0');
    uint32_t x = seed * 2654435761u + 1;
    for (size_t i = 0; i < n; ++i) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        s[i] = (char)x;
    }
    return s;
}

// drains a pipe/socket read end into out until `want` bytes arrived
void drain(int fd, std::string* out, size_t want) {
    char tmp[65536];
    while (out->size() < want) {
        const ssize_t r = read(fd, tmp, sizeof(tmp));
        if (r <= 0) break;
        out->append(tmp, (size_t)r);
    }
}

}  // namespace

TEST(BufDepth, appendv_many_pieces_in_order) {
    Buf b;
    std::string model;
    for (int i = 0; i < 500; ++i) {
        const std::string piece = pattern((size_t)(i * 37 % 311), (uint32_t)i);
        b.append(piece);
        model += piece;
    }
    EXPECT_EQ(b.size(), model.size());
    EXPECT_EQ(b.to_string(), model);
    // pieces packed into shared blocks, not one block per append
    EXPECT_LT(b.backing_block_num(), 500u);
}

TEST(BufDepth, append_contiguous_reserves_writable_tail) {
    Buf b;
    b.append("head:");
    char* p = b.append_contiguous(100);
    ASSERT_TRUE(p != nullptr);
    for (int i = 0; i < 100; ++i) p[i] = (char)('0' + i % 10);
    EXPECT_EQ(b.size(), 105u);
    std::string s = b.to_string();
    EXPECT_EQ(s.substr(0, 5), "head:");
    EXPECT_EQ(s[5], '0');
    EXPECT_EQ(s[104], '9');
    // a reservation larger than a default block is still contiguous
    char* big = b.append_contiguous(3 * Buf::DEFAULT_BLOCK_SIZE);
    ASSERT_TRUE(big != nullptr);
    memset(big, 'Z', 3 * Buf::DEFAULT_BLOCK_SIZE);
    EXPECT_EQ(b.size(), 105u + 3 * Buf::DEFAULT_BLOCK_SIZE);
    EXPECT_EQ(b.to_string().back(), 'Z');
}

TEST(BufDepth, copy_move_and_assign_share_blocks) {
    Buf a;
    a.append(pattern(30000, 1));
    Buf b(a);                // copy: shares blocks
    Buf c;
    c = a;                   // copy-assign
    Buf d(std::move(c));     // move: steals refs
    EXPECT_TRUE(c.empty());
    Buf e;
    e = std::move(d);
    EXPECT_TRUE(d.empty());
    EXPECT_TRUE(b.equals(a.to_string()));
    EXPECT_TRUE(e.equals(a.to_string()));
    // same blocks, not new ones
    EXPECT_EQ(b.block_data(0), a.block_data(0));
    EXPECT_EQ(e.block_data(0), a.block_data(0));
    e = e;  // self-assignment is harmless
    EXPECT_EQ(e.size(), 30000u);
    a.pop_front(100);
    EXPECT_EQ(b.size(), 30000u);  // the copies keep their view
}

TEST(BufDepth, equals_compares_bytes_not_layout) {
    const std::string s = pattern(20000, 2);
    Buf one(s), many;
    for (size_t off = 0; off < s.size(); off += 777) many.append(s.substr(off, 777));
    EXPECT_TRUE(one.equals(s));
    EXPECT_TRUE(many.equals(s));
    EXPECT_TRUE(many.equals(one.to_string()));
    std::string t = s;
    t[12345] ^= 1;
    EXPECT_FALSE(many.equals(t));
    EXPECT_FALSE(many.equals(s.substr(0, s.size() - 1)));
    EXPECT_TRUE(Buf().equals(""));
}

TEST(BufDepth, append_then_cut_it_all_in_random_chunks) {
    std::mt19937 rng(7);
    for (int round = 0; round < 20; ++round) {
        const std::string s = pattern(1 + rng() % 200000, (uint32_t)round);
        Buf b(s);
        std::string back;
        while (!b.empty()) {
            Buf piece;
            b.cutn(&piece, 1 + rng() % 9000);
            back += piece.to_string();
        }
        ASSERT_EQ(back, s);
    }
}

TEST(BufDepth, cut_by_single_char_delimiter) {
    Buf b;
    b.append("a,bb,,ccc,");
    b.append(std::string(9000, 'd'));
    b.append(",end");
    std::vector<std::string> got;
    Buf piece;
    while (b.cut_until(&piece, ",") == 0) {
        got.push_back(piece.to_string());
        piece.clear();
    }
    ASSERT_EQ(got.size(), 5u);
    EXPECT_EQ(got[0], "a");
    EXPECT_EQ(got[1], "bb");
    EXPECT_EQ(got[2], "");
    EXPECT_EQ(got[3], "ccc");
    EXPECT_EQ(got[4], std::string(9000, 'd'));
    EXPECT_EQ(b.to_string(), "end");
}

TEST(BufDepth, cut_into_fd_tiny_and_huge) {
    int fds[2];
    ASSERT_EQ(socketpair(AF_UNIX, SOCK_STREAM, 0, fds), 0);
    Buf tiny("x");
    EXPECT_EQ(tiny.cut_into_fd(fds[0]), 1);
    EXPECT_TRUE(tiny.empty());
    std::string got;
    drain(fds[1], &got, 1);
    EXPECT_EQ(got, "x");
    // a lot of data in many blocks: more regions than one writev takes
    Buf big;
    std::string model;
    for (int i = 0; i < 600; ++i) {
        const std::string p = pattern(3000, (uint32_t)i);
        char* mem = static_cast<char*>(malloc(p.size()));
        memcpy(mem, p.data(), p.size());
        big.append_user_data(mem, p.size(), [](void* d, void*) { free(d); });  // one region each
        model += p;
    }
    EXPECT_GT(big.backing_block_num(), (size_t)Buf::MAX_WRITEV_IOV);
    got.clear();
    fcntl(fds[0], F_SETFL, O_NONBLOCK);  // the writer must not block on a full socket
    fcntl(fds[1], F_SETFL, O_NONBLOCK);
    while (!big.empty()) {
        const ssize_t n = big.cut_into_fd(fds[0]);
        if (n < 0) ASSERT_TRUE(errno == EAGAIN);
        char tmp[65536];
        ssize_t r;
        while ((r = read(fds[1], tmp, sizeof(tmp))) > 0) got.append(tmp, (size_t)r);
    }
    fcntl(fds[1], F_SETFL, 0);
    drain(fds[1], &got, model.size());
    EXPECT_EQ(got.size(), model.size());
    EXPECT_TRUE(got == model);
    close(fds[0]);
    close(fds[1]);
}

TEST(BufDepth, append_store_append_cut_interleaved) {
    // a producer keeps appending while a consumer cuts and stores pieces:
    // the stored pieces stay intact after the source moved on
    Buf src;
    std::vector<Buf> stored;
    std::string model, stored_model;
    for (int i = 0; i < 300; ++i) {
        const std::string p = pattern(100 + i * 13, (uint32_t)i);
        src.append(p);
        model += p;
        Buf piece;
        src.cutn(&piece, 97 + i);
        stored_model += model.substr(0, piece.size());
        model.erase(0, piece.size());
        stored.push_back(std::move(piece));
    }
    std::string all;
    for (const Buf& b : stored) all += b.to_string();
    EXPECT_EQ(all, stored_model);
    EXPECT_EQ(src.to_string(), model);
}

TEST(BufDepth, own_block_append_block_takes_a_reference) {
    BufBlock* blk = NewBlock(4096);
    ASSERT_TRUE(blk != nullptr);
    memcpy(blk->data, "0123456789", 10);
    blk->size = 10;
    {
        Buf a;
        a.append_block(blk, 2, 5);  // "23456"
        Buf b;
        b.append_block(blk, 0, 10);
        EXPECT_EQ(a.to_string(), "23456");
        EXPECT_EQ(b.to_string(), "0123456789");
        EXPECT_EQ(blk->nshared.load(), 3);  // ours + two Bufs
    }
    EXPECT_EQ(blk->nshared.load(), 1);
    blk->dec_ref();
}

TEST(BufDepth, swap_exchanges_contents) {
    Buf a("alpha"), b;
    b.append(pattern(50000, 3));
    const std::string bs = b.to_string();
    a.swap(b);
    EXPECT_TRUE(a.equals(bs));
    EXPECT_EQ(b.to_string(), "alpha");
    Buf empty;
    empty.swap(b);
    EXPECT_TRUE(b.empty());
    EXPECT_EQ(empty.to_string(), "alpha");
}

TEST(BufDepth, bytes_iterator_forward_and_copy) {
    const std::string s = pattern(25000, 4);
    Buf b;
    for (size_t off = 0; off < s.size(); off += 1000) {
        Buf one(s.substr(off, 1000));
        b.append(one);
    }
    BufBytesIterator it(b);
    EXPECT_EQ(it.bytes_left(), s.size());
    EXPECT_EQ(it.forward(1500), 1500u);  // crosses a region
    EXPECT_EQ(*it, s[1500]);
    char out[3000];
    EXPECT_EQ(it.copy_and_forward(out, 3000), 3000u);
    EXPECT_EQ(std::string(out, 3000), s.substr(1500, 3000));
    EXPECT_EQ(it.bytes_left(), s.size() - 4500);
    EXPECT_EQ(it.forward(1u << 30), s.size() - 4500);  // clipped
    EXPECT_TRUE(it.done());
}

TEST(BufDepth, copy_to_string_at_every_offset) {
    const std::string s = pattern(9000, 5);
    Buf b;
    for (size_t off = 0; off < s.size(); off += 700) {
        Buf one(s.substr(off, 700));
        b.append(one);
    }
    for (size_t pos = 0; pos < s.size(); pos += 433) {
        std::string out;
        EXPECT_EQ(b.copy_to(&out, 1000, pos), std::min<size_t>(1000, s.size() - pos));
        ASSERT_EQ(out, s.substr(pos, 1000));
    }
}

TEST(BufDepth, appender_writes_in_order) {
    Buf b;
    BufAppender app(&b);
    std::string model;
    for (int i = 0; i < 10000; ++i) {
        if (i % 3 == 0) {
            app.push_back((char)('a' + i % 26));
            model.push_back((char)('a' + i % 26));
        } else {
            const std::string p = std::to_string(i);
            app.append(p.data(), p.size());
            model += p;
        }
    }
    EXPECT_EQ(app.buf(), &b);
    EXPECT_EQ(b.to_string(), model);
}

namespace {
std::atomic<int> g_user_frees{0};
void user_free(void* p, void* arg) {
    free(p);
    g_user_frees.fetch_add(arg ? *static_cast<int*>(arg) : 1);
}
}  // namespace

TEST(BufDepth, user_data_consumed_piecewise_then_freed_once) {
    g_user_frees = 0;
    char* mem = static_cast<char*>(malloc(100000));
    for (int i = 0; i < 100000; ++i) mem[i] = (char)(i * 7);
    Buf b;
    b.append_user_data(mem, 100000, user_free);
    size_t seen = 0;
    while (!b.empty()) {
        std::string piece;
        b.cutn(&piece, 3333);
        for (size_t i = 0; i < piece.size(); ++i) ASSERT_EQ(piece[i], (char)((seen + i) * 7));
        seen += piece.size();
        EXPECT_EQ(g_user_frees.load(), b.empty() ? 1 : 0);
    }
    EXPECT_EQ(seen, 100000u);
    EXPECT_EQ(g_user_frees.load(), 1);
}

TEST(BufDepth, user_data_shared_lives_until_the_last_view) {
    g_user_frees = 0;
    int weight = 10;
    char* mem = static_cast<char*>(malloc(5000));
    memset(mem, 'u', 5000);
    Buf a;
    a.append_user_data(mem, 5000, user_free, &weight);
    Buf views[4];
    for (int i = 0; i < 4; ++i) {
        views[i] = a;
        views[i].pop_front((size_t)i * 1000);
    }
    a.clear();
    for (int i = 0; i < 3; ++i) {
        views[i].clear();
        EXPECT_EQ(g_user_frees.load(), 0);
    }
    EXPECT_EQ(views[3].size(), 2000u);
    views[3].clear();
    EXPECT_EQ(g_user_frees.load(), 10);  // the deleter ran once, with its arg
}

TEST(BufDepth, user_data_with_meta_kind_and_device) {
    char* mem = static_cast<char*>(malloc(64));
    memcpy(mem, "pinned bytes", 12);
    Buf b;
    b.append_user_data(mem, 12, user_free, nullptr, MemKind::PINNED, -1, 0xfeedULL);
    ASSERT_EQ(b.backing_block_num(), 1u);
    const BufBlock* blk = b.ref_at(0).block;
    EXPECT_EQ(blk->meta, 0xfeedULL);
    EXPECT_TRUE(blk->kind == MemKind::PINNED);
    EXPECT_TRUE(b.all_host_accessible());
    EXPECT_EQ(b.to_string(), "pinned bytes");
    EXPECT_EQ(std::string(MemKindName(MemKind::DEVICE)).empty(), false);
}

namespace {
std::atomic<int> g_hook_calls{0};
int fake_device_copy(void* dst, const void* src, size_t n, MemKind, int) {
    g_hook_calls.fetch_add(1);
    memcpy(dst, src, n);  // the "device" block is host memory in this test
    return 0;
}
}  // namespace

TEST(BufDepth, device_blocks_copy_through_the_hook) {
    const DeviceCopyFn prev = GetDeviceCopyHook();
    SetDeviceCopyHook(fake_device_copy);
    g_hook_calls = 0;
    char* mem = static_cast<char*>(malloc(4096));
    for (int i = 0; i < 4096; ++i) mem[i] = (char)(i & 0xff);
    Buf b;
    b.append("host-prefix:");
    b.append_user_data(mem, 4096, user_free, nullptr, MemKind::DEVICE, 3, 0);
    EXPECT_FALSE(b.all_host_accessible());
    EXPECT_EQ(b.ref_at(1).block->device, 3);
    std::string out;
    EXPECT_EQ(b.copy_to(&out, 20, 10), 20u);  // straddles host and device
    EXPECT_EQ(out.substr(0, 2), "x:");
    EXPECT_EQ(out[2], (char)0);
    EXPECT_EQ(out[19], (char)17);
    EXPECT_GT(g_hook_calls.load(), 0);
    SetDeviceCopyHook(prev);
}

TEST(BufDepth, large_payloads_get_one_dedicated_block) {
    const std::string big = pattern(Buf::LARGE_BLOCK_THRESHOLD * 3, 6);
    Buf b;
    b.append("small");
    b.append(big);
    // the small head (whose block may also take the first bytes of the
    // large append) and one dedicated block for the rest
    EXPECT_LE(b.backing_block_num(), 3u);
    size_t largest = 0;
    for (size_t i = 0; i < b.backing_block_num(); ++i) largest = std::max(largest, b.block_len(i));
    EXPECT_GE(largest, big.size() - Buf::DEFAULT_BLOCK_SIZE);
    EXPECT_TRUE(b.equals("small" + big));
    Buf piece;
    b.cutn(&piece, 5 + Buf::LARGE_BLOCK_THRESHOLD);
    EXPECT_TRUE(piece.equals("small" + big.substr(0, Buf::LARGE_BLOCK_THRESHOLD)));
    EXPECT_TRUE(b.equals(big.substr(Buf::LARGE_BLOCK_THRESHOLD)));
}

TEST(BufDepth, tls_block_is_shared_by_small_appends) {
    // consecutive small appends from one thread land in the same block
    Buf a, b;
    a.append("first");
    b.append("second");
    ASSERT_EQ(a.backing_block_num(), 1u);
    ASSERT_EQ(b.backing_block_num(), 1u);
    EXPECT_EQ(a.ref_at(0).block, b.ref_at(0).block);
    EXPECT_EQ(a.to_string(), "first");
    EXPECT_EQ(b.to_string(), "second");
    // another thread gets its own block
    const BufBlock* other = nullptr;
    Buf c;
    std::thread th([&] {
        c.append("third");
        other = c.ref_at(0).block;
    });
    th.join();
    EXPECT_NE(other, a.ref_at(0).block);
    EXPECT_EQ(c.to_string(), "third");
}

TEST(BufDepth, block_accounting_returns_to_baseline) {
    const int64_t blocks0 = Buf::block_count();
    const int64_t mem0 = Buf::block_memory();
    {
        std::vector<Buf> bufs(64);
        for (size_t i = 0; i < bufs.size(); ++i) bufs[i].append(pattern(20000 + i * 100, (uint32_t)i));
        EXPECT_GT(Buf::block_count(), blocks0);
        EXPECT_GT(Buf::block_memory(), mem0);
    }
    EXPECT_LE(Buf::block_count() - blocks0, 8);  // thread caches may keep a few
}

TEST(BufDepth, portal_reads_into_its_own_blocks_across_calls) {
    int fds[2];
    ASSERT_EQ(socketpair(AF_UNIX, SOCK_STREAM, 0, fds), 0);
    const std::string msg = pattern(200000, 8);
    std::thread writer([&] {
        size_t off = 0;
        while (off < msg.size()) {
            const ssize_t n = write(fds[0], msg.data() + off, std::min<size_t>(7777, msg.size() - off));
            if (n <= 0) break;
            off += (size_t)n;
        }
    });
    BufPortal p;
    bool reads_ok = true;
    while (p.size() < msg.size()) {
        // max_count is a hint rounded up to whole blocks, as IOPortal's
        const ssize_t n = p.append_from_fd(fds[1], 10000);
        if (n <= 0 || n > (ssize_t)(10000 + Buf::DEFAULT_BLOCK_SIZE)) {
            reads_ok = false;
            break;
        }
    }
    writer.join();
    ASSERT_TRUE(reads_ok);
    EXPECT_TRUE(p.equals(msg));
    // consume from the front while the portal keeps reading: the tail block
    // is reused, and what was cut stays valid
    Buf head;
    p.cutn(&head, 123456);
    EXPECT_TRUE(head.equals(msg.substr(0, 123456)));
    p.return_cached_blocks();
    EXPECT_TRUE(p.equals(msg.substr(123456)));
    close(fds[0]);
    close(fds[1]);
}

TEST(BufDepth, concurrent_cut_into_fd_from_shared_source) {
    // threads write views of one shared Buf into their own pipes at once
    Buf shared;
    const std::string s = pattern(300000, 9);
    shared.append(s);
    const int kThreads = 4;
    std::vector<std::thread> ths;
    std::atomic<int> ok{0};
    for (int t = 0; t < kThreads; ++t) {
        ths.emplace_back([&, t] {
            int fds[2];
            if (pipe(fds) != 0) return;
            Buf mine = shared;  // shares the blocks
            mine.pop_front((size_t)t * 1000);
            const std::string want = s.substr((size_t)t * 1000);
            std::string got;
            std::thread reader([&] { drain(fds[0], &got, want.size()); });
            while (!mine.empty()) {
                if (mine.cut_into_fd(fds[1]) < 0) break;
            }
            reader.join();
            close(fds[0]);
            close(fds[1]);
            if (got == want) ok.fetch_add(1);
        });
    }
    for (auto& th : ths) th.join();
    EXPECT_EQ(ok.load(), kThreads);
    EXPECT_TRUE(shared.equals(s));
}

TEST(BufDepth, fill_iov_respects_limits) {
    Buf b;
    for (int i = 0; i < 20; ++i) {
        char* mem = static_cast<char*>(malloc(1000));
        memset(mem, 'a' + i, 1000);
        b.append_user_data(mem, 1000, [](void* d, void*) { free(d); });  // one region each
    }
    struct iovec iov[8];
    size_t nbytes = 0;
    int n = b.fill_iov(iov, 8, 1u << 30, &nbytes);  // iov-bound
    EXPECT_EQ(n, 8);
    EXPECT_EQ(nbytes, 8000u);
    EXPECT_EQ(static_cast<const char*>(iov[7].iov_base)[0], 'h');
    n = b.fill_iov(iov, 8, 2500, &nbytes);  // byte-bound: whole regions until the hint is reached
    EXPECT_EQ(n, 3);
    EXPECT_EQ(nbytes, 3000u);
    EXPECT_EQ(b.size(), 20000u);  // fill_iov does not consume
}

TEST(BufDepth, pop_back_across_blocks_and_reappend) {
    Buf b;
    std::string model;
    for (int i = 0; i < 30; ++i) {
        Buf one(pattern(500, (uint32_t)i));
        model += one.to_string();
        b.append(one);
    }
    EXPECT_EQ(b.pop_back(1234), 1234u);
    model.resize(model.size() - 1234);
    EXPECT_TRUE(b.equals(model));
    b.append("after");
    model += "after";
    EXPECT_TRUE(b.equals(model));
    EXPECT_EQ(b.pop_front(model.size() - 3), model.size() - 3);
    EXPECT_EQ(b.to_string(), "ter");
}

TEST(BufDepth, cut1_and_fetch1_walk_every_byte) {
    const std::string s = pattern(20000, 10);
    Buf b;
    for (size_t off = 0; off < s.size(); off += 333) {
        Buf one(s.substr(off, 333));
        b.append(one);
    }
    for (size_t i = 0; i < s.size(); ++i) {
        ASSERT_EQ(*b.fetch1(), s[i]);
        char c;
        ASSERT_TRUE(b.cut1(&c));
        ASSERT_EQ(c, s[i]);
    }
    EXPECT_TRUE(b.fetch1() == nullptr);
}

TEST(BufDepth, cutn_into_raw_memory_and_string) {
    Buf b(pattern(10000, 11));
    const std::string s = b.to_string();
    char raw[4000];
    EXPECT_EQ(b.cutn(raw, sizeof(raw)), sizeof(raw));
    EXPECT_EQ(std::string(raw, sizeof(raw)), s.substr(0, 4000));
    std::string rest;
    EXPECT_EQ(b.cutn(&rest, 100000), 6000u);
    EXPECT_EQ(rest, s.substr(4000));
    EXPECT_TRUE(b.empty());
}
