// More Buf cases (base/buf.h), after the reference's test/iobuf_unittest.cpp:
// self-assignment and self-append, refs that merge when appended back to
// back, appending a Buf to itself through a copy, cut_until at block seams
// and with a delimiter at the very end, fetch1 / cut1 on empty buffers,
// copy_to at and past the end, iterator forward/copy across empty refs,
// append_block slices of one block, device-kind blocks kept out of host
// reads, pop_back of whole blocks, fill_iov with max_iov 1, portal reads
// across EOF of a pipe, BufAppender through thousands of small pieces, and
// the block/memory counters returning to their baseline.
#include <fcntl.h>
#include <unistd.h>

#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "base/buf.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

std::string pattern(size_t n, unsigned seed) {
    std::string s(n, '\0');
    std::mt19937 rng(seed);
    for (auto& c : s) c = (char)('a' + rng() % 26);
    return s;
}

// A Buf made of `pieces` user blocks (distinct regions, one ref each).
struct Pieces {
    std::vector<std::string> store;
    Buf buf;
    explicit Pieces(const std::vector<std::string>& parts) : store(parts) {
        for (auto& s : store) buf.append_user_data(&s[0], s.size(), [](void*, void*) {});
    }
};

}  // namespace

TEST(BufMore, self_assignment_and_self_append_through_a_copy) {
    Buf b;
    b.append(pattern(20000, 1));
    const std::string want = b.to_string();
    Buf& alias = b;
    b = alias;  // self copy-assignment keeps the bytes
    EXPECT_TRUE(b.equals(want));
    Buf copy = b;
    b.append(copy);  // doubling through a copy
    EXPECT_EQ(b.size(), 2 * want.size());
    EXPECT_TRUE(b.equals(want + want));
    EXPECT_TRUE(copy.equals(want));
}

TEST(BufMore, adjacent_slices_of_one_block_merge_into_one_ref) {
    BufBlock* blk = NewBlock(4096);
    memset(blk->data, 'q', 4096);
    blk->size = 4096;
    Buf b;
    b.append_block(blk, 0, 1000);
    b.append_block(blk, 1000, 1000);
    b.append_block(blk, 2000, 96);
    EXPECT_EQ(b.size(), 2096u);
    EXPECT_EQ(b.backing_block_num(), 1u);  // contiguous: one ref
    b.append_block(blk, 3000, 10);          // a gap: a new ref
    EXPECT_EQ(b.backing_block_num(), 2u);
    blk->dec_ref();
    EXPECT_EQ(b.to_string(), std::string(2106, 'q'));
}

TEST(BufMore, cut_until_with_the_delimiter_across_a_seam) {
    Pieces p({"alpha\r", "\nbeta\r\n", "gamma"});
    Buf line;
    ASSERT_EQ(p.buf.cut_until(&line, "\r\n"), 0);
    EXPECT_TRUE(line.equals("alpha"));
    line.clear();
    ASSERT_EQ(p.buf.cut_until(&line, "\r\n"), 0);
    EXPECT_TRUE(line.equals("beta"));
    line.clear();
    EXPECT_EQ(p.buf.cut_until(&line, "\r\n"), -1);  // not found: nothing consumed
    EXPECT_TRUE(p.buf.equals("gamma"));
    EXPECT_TRUE(line.empty());
}

TEST(BufMore, cut_until_delimiter_at_the_end_and_at_the_front) {
    Buf b;
    b.append(",x,");
    Buf out;
    ASSERT_EQ(b.cut_until(&out, ","), 0);
    EXPECT_TRUE(out.empty());  // delimiter first: an empty piece
    ASSERT_EQ(b.cut_until(&out, ","), 0);
    EXPECT_TRUE(out.equals("x"));
    EXPECT_TRUE(b.empty());
}

TEST(BufMore, empty_buffer_reads) {
    Buf b;
    char c = 'z';
    EXPECT_FALSE(b.cut1(&c));
    EXPECT_EQ(c, 'z');
    EXPECT_TRUE(b.fetch1() == nullptr);
    char aux[4];
    EXPECT_TRUE(b.fetch(aux, 1) == nullptr);
    EXPECT_EQ(b.copy_to(aux, 4), 0u);
    EXPECT_EQ(b.pop_front(10), 0u);
    EXPECT_EQ(b.pop_back(10), 0u);
    std::string s = "keep";
    EXPECT_EQ(b.copy_to(&s), 0u);
    EXPECT_TRUE(b.equals(""));
    EXPECT_TRUE(b.all_host_accessible());
}

TEST(BufMore, copy_to_at_and_past_the_end) {
    Buf b;
    b.append("0123456789");
    char out[16] = {0};
    EXPECT_EQ(b.copy_to(out, 4, 8), 2u);  // only two bytes remain after pos 8
    EXPECT_EQ(std::string(out, 2), "89");
    EXPECT_EQ(b.copy_to(out, 4, 10), 0u);
    EXPECT_EQ(b.copy_to(out, 4, 100), 0u);
    std::string s;
    EXPECT_EQ(b.copy_to(&s, (size_t)-1, 3), 7u);
    EXPECT_EQ(s, "3456789");
    EXPECT_EQ(b.size(), 10u);  // nothing consumed
}

TEST(BufMore, fetch_returns_in_place_pointers_inside_one_block) {
    Buf b;
    b.append("abcdef");
    char aux[8];
    const void* p = b.fetch(aux, 4);
    ASSERT_TRUE(p != nullptr);
    EXPECT_TRUE(p != aux);  // no copy needed
    EXPECT_EQ(memcmp(p, "abcd", 4), 0);
    EXPECT_TRUE(b.fetch(aux, 7) == nullptr);  // more than there is
}

TEST(BufMore, bytes_iterator_forward_and_copy_across_pieces) {
    Pieces p({"ab", "cde", "f", "ghij"});
    BufBytesIterator it(p.buf);
    EXPECT_EQ(it.bytes_left(), 10u);
    EXPECT_EQ(it.forward(3), 3u);
    EXPECT_EQ(*it, 'd');
    char out[8] = {0};
    EXPECT_EQ(it.copy_and_forward(out, 4), 4u);
    EXPECT_EQ(std::string(out, 4), "defg");
    EXPECT_EQ(*it, 'h');
    EXPECT_EQ(it.forward(100), 3u);  // clipped at the end
    EXPECT_TRUE(it.done());
}

TEST(BufMore, device_blocks_are_not_host_accessible) {
    static char fake[64];
    Buf b;
    b.append("host");
    EXPECT_TRUE(b.all_host_accessible());
    b.append_user_data(fake, sizeof(fake), [](void*, void*) {}, nullptr, MemKind::DEVICE, 0, 7);
    EXPECT_FALSE(b.all_host_accessible());
    EXPECT_EQ(b.backing_block_num(), 2u);
    EXPECT_TRUE(b.ref_at(1).block->kind == MemKind::DEVICE);
    EXPECT_EQ(b.ref_at(1).block->meta, 7u);
    EXPECT_EQ(b.ref_at(1).block->device, 0);
    b.pop_back(64);
    EXPECT_TRUE(b.all_host_accessible());
    EXPECT_EQ(std::string(MemKindName(MemKind::PEER)).empty(), false);
}

TEST(BufMore, pop_back_drops_whole_and_partial_pieces) {
    Pieces p({"1111", "2222", "3333"});
    EXPECT_EQ(p.buf.pop_back(5), 5u);
    EXPECT_TRUE(p.buf.equals("1111222"));
    EXPECT_EQ(p.buf.backing_block_num(), 2u);
    EXPECT_EQ(p.buf.pop_back(3), 3u);
    EXPECT_TRUE(p.buf.equals("1111"));
    EXPECT_EQ(p.buf.backing_block_num(), 1u);
}

TEST(BufMore, fill_iov_with_a_single_slot) {
    Pieces p({"aaaa", "bbbb", "cccc"});
    struct iovec iov[1];
    size_t nbytes = 0;
    EXPECT_EQ(p.buf.fill_iov(iov, 1, 1 << 20, &nbytes), 1);
    EXPECT_EQ(nbytes, 4u);
    EXPECT_EQ(std::string((const char*)iov[0].iov_base, iov[0].iov_len), "aaaa");
}

TEST(BufMore, portal_reads_a_pipe_to_eof_in_bounded_steps) {
    int fds[2];
    ASSERT_EQ(pipe(fds), 0);
    const std::string want = pattern(100000, 5);
    size_t written = 0;
    // the pipe holds 64 KiB: write, read, write the rest, close
    BufPortal portal;
    while (written < want.size()) {
        const ssize_t w = write(fds[1], want.data() + written, std::min<size_t>(32768, want.size() - written));
        ASSERT_TRUE(w > 0);
        written += (size_t)w;
        while (portal.size() < written) {
            const ssize_t r = portal.append_from_fd(fds[0], 10000);  // bounded per call
            ASSERT_TRUE(r > 0 && r <= 10000);
        }
    }
    close(fds[1]);
    for (;;) {
        const ssize_t r = portal.append_from_fd(fds[0], 1 << 16);
        ASSERT_TRUE(r >= 0);
        if (r == 0) break;  // EOF
    }
    close(fds[0]);
    EXPECT_EQ(portal.size(), want.size());
    EXPECT_TRUE(portal.equals(want));
    portal.return_cached_blocks();
}

TEST(BufMore, appender_of_many_small_pieces) {
    Buf b;
    BufAppender app(&b);
    std::string want;
    for (int i = 0; i < 5000; ++i) {
        const std::string s = std::to_string(i) + ";";
        app.append(s.data(), s.size());
        want += s;
        if (i % 7 == 0) {
            app.push_back('|');
            want += '|';
        }
    }
    EXPECT_TRUE(app.buf() == &b);
    EXPECT_EQ(b.size(), want.size());
    EXPECT_TRUE(b.equals(want));
    // small appends share blocks: far fewer refs than appends
    EXPECT_TRUE(b.backing_block_num() < 20);
}

TEST(BufMore, move_leaves_the_source_empty_and_usable) {
    Buf a;
    a.append(pattern(30000, 9));
    const std::string want = a.to_string();
    Buf b(std::move(a));
    EXPECT_TRUE(b.equals(want));
    EXPECT_TRUE(a.empty());  // NOLINT: moved-from is specified empty
    a.append("again");
    EXPECT_TRUE(a.equals("again"));
    Buf c;
    c = std::move(b);
    EXPECT_TRUE(c.equals(want));
    EXPECT_TRUE(b.empty());  // NOLINT
}

TEST(BufMore, counters_return_to_baseline) {
    const int64_t blocks0 = Buf::block_count();
    const int64_t mem0 = Buf::block_memory();
    {
        std::vector<Buf> bufs(50);
        for (size_t i = 0; i < bufs.size(); ++i) bufs[i].append(pattern(70000 + i, (unsigned)i));  // large blocks
        EXPECT_TRUE(Buf::block_count() > blocks0);
        EXPECT_TRUE(Buf::block_memory() > mem0);
    }
    EXPECT_EQ(Buf::block_count(), blocks0);
    EXPECT_EQ(Buf::block_memory(), mem0);
}

TEST(BufMore, random_cuts_into_bufs_preserve_order) {
    const std::string want = pattern(200000, 11);
    Buf src;
    std::mt19937 rng(3);
    for (size_t o = 0; o < want.size();) {
        const size_t n = std::min<size_t>(want.size() - o, 1 + rng() % 9000);
        src.append(want.data() + o, n);
        o += n;
    }
    std::vector<Buf> parts;
    while (!src.empty()) {
        parts.emplace_back();
        src.cutn(&parts.back(), 1 + rng() % 12000);
    }
    Buf joined;
    for (auto& p : parts) joined.append(std::move(p));
    EXPECT_TRUE(joined.equals(want));
}

// A read sized for 512 KiB that finds 32 KiB keeps the untouched blocks for
// the next read instead of freeing them (BufPortal::_spare): repeated reads
// allocate no new blocks, and return_cached_blocks() gives them all back.
TEST(BufMore, portal_keeps_unfilled_blocks_for_the_next_read) {
    int fds[2];
    ASSERT_EQ(pipe(fds), 0);
    const std::string msg = pattern(32768, 21);
    const int64_t blocks0 = Buf::block_count();
    {
        BufPortal portal;
        int64_t after_first = 0;
        for (int round = 0; round < 20; ++round) {
            ASSERT_EQ(write(fds[1], msg.data(), msg.size()), (ssize_t)msg.size());
            size_t got = 0;
            while (got < msg.size()) {
                const ssize_t r = portal.append_from_fd(fds[0], 524288);
                ASSERT_TRUE(r > 0);
                got += (size_t)r;
            }
            Buf out;
            portal.cutn(&out, msg.size());
            EXPECT_TRUE(out.equals(msg));
            if (round == 0) after_first = Buf::block_count();
            // later rounds reuse the spare blocks: no growth past the first
            EXPECT_TRUE(Buf::block_count() <= after_first);
        }
        portal.return_cached_blocks();
        EXPECT_TRUE(portal.empty());
    }
    close(fds[0]);
    close(fds[1]);
    EXPECT_TRUE(Buf::block_count() <= blocks0 + 8);  // at most the thread's block cache
}
