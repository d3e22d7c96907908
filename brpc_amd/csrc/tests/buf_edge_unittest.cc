// Buf edge cases (base/buf.h): zero-length appends, over-long pops, a
// randomized queue model against std::string, multi-character delimiters,
// many tiny appends, writev of several Bufs into one fd, fetch across block
// boundaries and block accounting back to the baseline. Parity: the
// reference's test/iobuf_unittest.cpp (append_zero, pop_front/back,
// iobuf_as_queue, cut_by_multiple_text_delim, append_a_lot_and_cut_them_all,
// cut_multiple_into_fd_tiny, copy_to).
#include <fcntl.h>
#include <unistd.h>

#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "base/buf.h"
#include "tests/test.h"

using namespace mrpc;

TEST(BufEdge, append_zero_and_empty_sources) {
    Buf b;
    EXPECT_EQ(b.append("", 0), 0);
    EXPECT_EQ(b.append(std::string()), 0);
    Buf empty;
    b.append(empty);
    EXPECT_TRUE(b.empty());
    EXPECT_EQ(b.backing_block_num(), 0u);
    EXPECT_EQ(b.to_string(), "");
}

TEST(BufEdge, pops_and_cuts_longer_than_the_buf) {
    Buf b("hello world");
    EXPECT_EQ(b.pop_front(6), 6u);
    EXPECT_EQ(b.to_string(), "world");
    EXPECT_EQ(b.pop_back(100), 5u);  // only what is there
    EXPECT_TRUE(b.empty());
    EXPECT_EQ(b.pop_front(1), 0u);
    EXPECT_EQ(b.pop_back(1), 0u);
    b.append("abc");
    std::string s;
    EXPECT_EQ(b.cutn(&s, 10), 3u);
    EXPECT_EQ(s, "abc");
    char c;
    EXPECT_FALSE(b.cut1(&c));
    char raw[4];
    EXPECT_EQ(b.copy_to(raw, 4), 0u);
}

TEST(BufEdge, copy_to_past_the_end) {
    Buf b;
    for (int i = 0; i < 3; ++i) b.append(std::string(7000, (char)('a' + i)));  // several blocks
    std::string out;
    EXPECT_EQ(b.copy_to(&out, 100, 20990), 10u);  // clipped at the end
    EXPECT_EQ(out, std::string(10, 'c'));
    EXPECT_EQ(b.copy_to(&out, 5, 21000), 0u);  // at the end
    EXPECT_EQ(b.copy_to(&out, 5, 50000), 0u);  // past it
    char buf[3];
    EXPECT_EQ(b.copy_to(buf, 3, 6999), 3u);  // straddles a block boundary
    EXPECT_EQ(std::string(buf, 3), "abb");
}

TEST(BufEdge, random_queue_matches_a_string_model) {
    std::mt19937 rng(12345);
    Buf q;
    std::string model;
    size_t produced = 0;
    for (int step = 0; step < 20000; ++step) {
        const int op = (int)(rng() % 10);
        if (op < 5) {
            std::string piece(rng() % 3000, '\0');
            for (char& ch : piece) ch = (char)('A' + (produced++ % 26));
            if (rng() % 4 == 0) {
                Buf tmp(piece);  // appended by reference
                q.append(tmp);
            } else {
                q.append(piece);
            }
            model += piece;
        } else if (op < 8) {
            const size_t n = rng() % 4000;
            std::string out;
            q.cutn(&out, n);
            ASSERT_EQ(out, model.substr(0, n));
            model.erase(0, std::min(n, model.size()));
        } else if (op == 8) {
            const size_t n = rng() % 500;
            q.pop_back(n);
            model.resize(model.size() - std::min(n, model.size()));
        } else {
            Buf head;
            const size_t n = rng() % 5000;
            q.cutn(&head, n);
            ASSERT_TRUE(head.equals(model.substr(0, n)));
            model.erase(0, std::min(n, model.size()));
        }
        ASSERT_EQ(q.size(), model.size());
    }
    EXPECT_EQ(q.to_string(), model);
}

TEST(BufEdge, cut_until_multi_character_delimiters) {
    Buf b;
    // the delimiter straddles block boundaries in the second record
    b.append("key1: v1\r\n");
    b.append(std::string(8190, 'x') + "\r");
    b.append("\nkey3: v3\r\n\r\ntail");
    Buf line;
    ASSERT_EQ(b.cut_until(&line, "\r\n"), 0);
    EXPECT_EQ(line.to_string(), "key1: v1");
    line.clear();
    ASSERT_EQ(b.cut_until(&line, "\r\n"), 0);
    EXPECT_EQ(line.size(), 8190u);
    line.clear();
    ASSERT_EQ(b.cut_until(&line, "\r\n\r\n"), 0);
    EXPECT_EQ(line.to_string(), "key3: v3");
    line.clear();
    EXPECT_NE(b.cut_until(&line, "\r\n"), 0);  // no delimiter left: nothing cut
    EXPECT_EQ(b.to_string(), "tail");
}

TEST(BufEdge, a_million_tiny_appends_cut_back_exactly) {
    const int64_t blocks0 = Buf::block_count();
    {
        Buf b;
        for (int i = 0; i < 1000000; ++i) b.push_back((char)(i & 0x7f));
        EXPECT_EQ(b.size(), 1000000u);
        int64_t sum = 0;
        char c;
        size_t n = 0;
        while (b.cut1(&c)) {
            sum += c;
            ++n;
        }
        EXPECT_EQ(n, 1000000u);
        int64_t want = 0;
        for (int i = 0; i < 1000000; ++i) want += (i & 0x7f);
        EXPECT_EQ(sum, want);
    }
    // every block went back (thread-local caches may keep a few)
    EXPECT_LE(Buf::block_count() - blocks0, 8);
}

TEST(BufEdge, cut_multiple_into_one_fd) {
    int fds[2];
    ASSERT_EQ(pipe(fds), 0);
    Buf a("first|"), b, c("third");
    b.append(std::string(10000, 'm'));
    b.append("|");
    Buf* pieces[] = {&a, &b, &c};
    size_t total = a.size() + b.size() + c.size();
    size_t written = 0;
    std::string got;
    fcntl(fds[0], F_SETFL, O_NONBLOCK);
    while (written < total) {
        const ssize_t n = Buf::cut_multiple_into_fd(fds[1], pieces, 3);
        ASSERT_GT(n, 0);
        written += (size_t)n;
        char tmp[65536];
        ssize_t r;
        while ((r = read(fds[0], tmp, sizeof(tmp))) > 0) got.append(tmp, (size_t)r);
    }
    close(fds[1]);
    char tmp[65536];
    ssize_t r;
    while ((r = read(fds[0], tmp, sizeof(tmp))) > 0) got.append(tmp, (size_t)r);
    close(fds[0]);
    EXPECT_EQ(got, "first|" + std::string(10000, 'm') + "|third");
    EXPECT_TRUE(a.empty() && b.empty() && c.empty());
}

TEST(BufEdge, fetch_across_blocks_uses_the_aux_buffer) {
    Buf b;
    b.append(std::string(8190, 'p'));  // forces a block boundary soon after
    b.append("QRSTUVWX");
    b.pop_front(8186);
    char aux[12];
    const char* p = static_cast<const char*>(b.fetch(aux, 12));
    ASSERT_TRUE(p != nullptr);
    EXPECT_EQ(std::string(p, 12), "ppppQRSTUVWX");
    EXPECT_TRUE(b.fetch(aux, 13) == nullptr);  // longer than the buf
    EXPECT_EQ(*b.fetch1(), 'p');
}

TEST(BufEdge, shared_blocks_survive_the_original) {
    Buf copy;
    {
        Buf orig;
        orig.append(std::string(20000, 'z'));
        copy = orig;
        orig.pop_front(5000);
        orig.append("tail");
    }
    EXPECT_EQ(copy.size(), 20000u);
    EXPECT_EQ(copy.to_string(), std::string(20000, 'z'));
}
