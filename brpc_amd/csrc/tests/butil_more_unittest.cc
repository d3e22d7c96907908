// More base-library depth, in the spirit of the reference's butil tests
// (test/iobuf_unittest.cpp, test/recordio_unittest.cpp, test/fast_rand_test.cpp,
// test/string_printf_unittest.cpp, test/time_unittest.cpp, test/flags_unittest):
// Buf cut/pop/fetch/copy edge cases at block boundaries, the byte iterator,
// user-data deleters, the fd writer over several Bufs, record files with
// seeks and damaged tails, fast_rand ranges, string helpers, time helpers,
// and flag parsing forms.
#include <fcntl.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "base/buf.h"
#include "base/crc32c.h"
#include "base/flags.h"
#include "base/recordio.h"
#include "base/time.h"
#include "base/util.h"
#include "tests/test.h"

using namespace mrpc;

DEFINE_int32(butil_more_test_i32, 7, "test flag");
DEFINE_uint64(butil_more_test_u64, 9, "test flag");
DEFINE_double(butil_more_test_d, 0.5, "test flag");
DEFINE_bool(butil_more_test_b, false, "test flag");
DEFINE_string(butil_more_test_s, "x", "test flag");

namespace {

// A Buf made of several blocks: each piece appended as its own user block.
Buf pieces(const std::vector<std::string>& parts, std::vector<std::string>* keep) {
    Buf b;
    for (const std::string& p : parts) {
        keep->push_back(p);
        std::string& s = keep->back();
        b.append_user_data(&s[0], s.size(), [](void*, void*) {});
    }
    return b;
}

std::string tmp_path(const char* tag) {
    return string_printf("/tmp/mrpc_butil_more_%s_%d_%lld", tag, (int)getpid(), (long long)monotonic_ns());
}

}  // namespace

TEST(ButilMore, pop_back_across_blocks) {
    std::vector<std::string> keep;
    keep.reserve(8);
    Buf b = pieces({"abc", "defg", "hi"}, &keep);
    EXPECT_EQ(b.size(), 9u);
    EXPECT_EQ(b.pop_back(3), 3u);  // "hi" and "g"
    EXPECT_EQ(b.to_string(), "abcdef");
    EXPECT_EQ(b.pop_back(100), 6u);
    EXPECT_TRUE(b.empty());
    EXPECT_EQ(b.pop_back(1), 0u);
}

TEST(ButilMore, pop_front_and_cut1_across_blocks) {
    std::vector<std::string> keep;
    keep.reserve(8);
    Buf b = pieces({"ab", "c", "def"}, &keep);
    EXPECT_EQ(b.pop_front(3), 3u);
    char c = 0;
    EXPECT_TRUE(b.cut1(&c));
    EXPECT_EQ(c, 'd');
    EXPECT_EQ(b.to_string(), "ef");
    EXPECT_TRUE(b.cut1(&c));
    EXPECT_TRUE(b.cut1(&c));
    EXPECT_EQ(c, 'f');
    EXPECT_FALSE(b.cut1(&c));
}

TEST(ButilMore, cutn_into_string_buf_and_memory) {
    Buf b;
    std::string big(20000, 'x');
    for (size_t i = 0; i < big.size(); ++i) big[i] = (char)('a' + i % 26);
    b.append(big);
    std::string s;
    EXPECT_EQ(b.cutn(&s, 5), 5u);
    EXPECT_EQ(s, big.substr(0, 5));
    Buf mid;
    EXPECT_EQ(b.cutn(&mid, 9000), 9000u);
    EXPECT_TRUE(mid.equals(big.substr(5, 9000)));
    char tail[16];
    EXPECT_EQ(b.cutn(tail, 16), 16u);
    EXPECT_EQ(std::string(tail, 16), big.substr(9005, 16));
    EXPECT_EQ(b.size(), big.size() - 9021);
    std::string rest;
    EXPECT_EQ(b.cutn(&rest, 1u << 20), big.size() - 9021);  // more than left: cuts what is there
    EXPECT_TRUE(b.empty());
}

TEST(ButilMore, copy_to_with_offsets_does_not_consume) {
    std::vector<std::string> keep;
    keep.reserve(8);
    Buf b = pieces({"0123", "4567", "89"}, &keep);
    char out[8] = {0};
    EXPECT_EQ(b.copy_to(out, 5, 2), 5u);
    EXPECT_EQ(std::string(out, 5), "23456");
    std::string s;
    EXPECT_EQ(b.copy_to(&s, 100, 7), 3u);
    EXPECT_EQ(s, "789");
    EXPECT_EQ(b.copy_to(out, 4, 10), 0u);  // at the end
    EXPECT_EQ(b.size(), 10u);
}

TEST(ButilMore, fetch_spanning_blocks_uses_aux) {
    std::vector<std::string> keep;
    keep.reserve(8);
    Buf b = pieces({"ab", "cd", "ef"}, &keep);
    char aux[8];
    const char* p = (const char*)b.fetch(aux, 5);
    ASSERT_TRUE(p != nullptr);
    EXPECT_EQ(std::string(p, 5), "abcde");
    EXPECT_TRUE(p == aux);  // spanned blocks: copied
    const char* q = (const char*)b.fetch(aux, 2);
    EXPECT_EQ(std::string(q, 2), "ab");
    EXPECT_TRUE(q == keep[0].data());  // within the first block: zero copy
    EXPECT_TRUE(b.fetch(aux, 7) == nullptr);
    EXPECT_EQ(*b.fetch1(), 'a');
    Buf empty;
    EXPECT_TRUE(empty.fetch1() == nullptr);
}

TEST(ButilMore, cut_until_multi_char_delimiter_across_blocks) {
    std::vector<std::string> keep;
    keep.reserve(8);
    Buf b = pieces({"GET / HTTP/1.1\r", "\nHost: x\r\n", "\r\nbody"}, &keep);
    Buf line;
    EXPECT_EQ(b.cut_until(&line, "\r\n"), 0);
    EXPECT_EQ(line.to_string(), "GET / HTTP/1.1");
    line.clear();
    EXPECT_EQ(b.cut_until(&line, "\r\n"), 0);
    EXPECT_EQ(line.to_string(), "Host: x");
    line.clear();
    EXPECT_EQ(b.cut_until(&line, "\r\n"), 0);
    EXPECT_TRUE(line.empty());
    EXPECT_EQ(b.cut_until(&line, "\r\n"), -1);  // not found: nothing consumed
    EXPECT_EQ(b.to_string(), "body");
}

TEST(ButilMore, move_append_empties_the_source) {
    Buf a("left"), b("right");
    a.append(std::move(b));
    EXPECT_EQ(a.to_string(), "leftright");
    EXPECT_TRUE(b.empty());
    Buf c(a);  // copies share blocks
    a.pop_front(4);
    EXPECT_EQ(c.to_string(), "leftright");
    EXPECT_EQ(a.to_string(), "right");
    a.swap(c);
    EXPECT_EQ(a.to_string(), "leftright");
    EXPECT_EQ(c.to_string(), "right");
}

TEST(ButilMore, user_data_deleter_runs_once_after_last_reference) {
    static std::atomic<int> deleted{0};
    deleted = 0;
    char* mem = new char[64];
    memset(mem, 'u', 64);
    {
        Buf a;
        a.append_user_data(mem, 64, [](void* d, void*) {
            delete[] static_cast<char*>(d);
            deleted.fetch_add(1);
        });
        Buf b(a), c;
        c.append(a);
        a.clear();
        EXPECT_EQ(deleted.load(), 0);
        b.pop_front(10);
        EXPECT_EQ(deleted.load(), 0);
        EXPECT_EQ(c.size(), 64u);
    }
    EXPECT_EQ(deleted.load(), 1);
}

TEST(ButilMore, append_contiguous_is_part_of_the_buffer) {
    Buf b("head");
    char* p = b.append_contiguous(6);
    memcpy(p, "-tail!", 6);
    EXPECT_EQ(b.to_string(), "head-tail!");
    EXPECT_EQ(b.size(), 10u);
}

TEST(ButilMore, bytes_iterator_walks_every_block) {
    std::vector<std::string> keep;
    keep.reserve(8);
    Buf b = pieces({"ab", "", "cde", "f"}, &keep);
    std::string seen;
    for (BufBytesIterator it(b); !it.done(); ++it) seen.push_back(*it);
    EXPECT_EQ(seen, "abcdef");
    BufBytesIterator it(b);
    char out[4];
    EXPECT_EQ(it.copy_and_forward(out, 3), 3u);
    EXPECT_EQ(std::string(out, 3), "abc");
    EXPECT_EQ(it.forward(2), 2u);
    EXPECT_EQ(*it, 'f');
    EXPECT_EQ(it.bytes_left(), 1u);
    EXPECT_EQ(it.forward(5), 1u);
    EXPECT_TRUE(it.done());
}

TEST(ButilMore, cut_multiple_into_fd_writes_in_order) {
    int fds[2];
    ASSERT_EQ(pipe(fds), 0);
    Buf a("first,"), b("second,"), c("third");
    Buf* all[] = {&a, &b, &c};
    const ssize_t n = Buf::cut_multiple_into_fd(fds[1], all, 3);
    EXPECT_EQ(n, 18);
    EXPECT_TRUE(a.empty() && b.empty() && c.empty());
    char got[32] = {0};
    EXPECT_EQ(read(fds[0], got, sizeof(got)), 18);
    EXPECT_EQ(std::string(got, 18), "first,second,third");
    close(fds[0]);
    close(fds[1]);
}

TEST(ButilMore, portal_reads_until_eof) {
    int fds[2];
    ASSERT_EQ(pipe(fds), 0);
    std::string msg(30000, 'p');
    std::thread w([&] {
        size_t off = 0;
        while (off < msg.size()) {
            const ssize_t k = write(fds[1], msg.data() + off, msg.size() - off);
            if (k <= 0) break;
            off += (size_t)k;
        }
        close(fds[1]);
    });
    BufPortal p;
    for (;;) {
        const ssize_t k = p.append_from_fd(fds[0], 4096);
        if (k <= 0) break;
    }
    w.join();
    EXPECT_EQ(p.size(), msg.size());
    EXPECT_TRUE(p.equals(msg));
    close(fds[0]);
}

TEST(ButilMore, fill_iov_takes_whole_blocks_up_to_the_hint) {
    // max_bytes is a size hint, as the reference's cut_into_fd size_hint:
    // whole blocks until the total reaches it (writev never splits a block)
    std::vector<std::string> keep;
    keep.reserve(8);
    Buf b = pieces({"aaaa", "bbbb", "cccc"}, &keep);
    struct iovec iov[8];
    size_t nbytes = 0;
    const int n = b.fill_iov(iov, 8, 6, &nbytes);
    EXPECT_EQ(n, 2);
    EXPECT_EQ(nbytes, 8u);
    EXPECT_EQ(iov[1].iov_len, 4u);
    EXPECT_EQ(b.fill_iov(iov, 8, 4, &nbytes), 1);  // the hint reached exactly: stop
    const int m = b.fill_iov(iov, 1, 100, &nbytes);
    EXPECT_EQ(m, 1);
    EXPECT_EQ(nbytes, 4u);
}

TEST(ButilMore, record_file_seek_to_written_offsets) {
    const std::string path = tmp_path("seek");
    std::vector<uint64_t> offs;
    {
        RecordWriter w(path);
        ASSERT_TRUE(w.ok());
        for (int i = 0; i < 20; ++i) {
            Record r;
            r.MutableMeta("idx")->append(std::to_string(i));
            r.MutablePayload()->append(std::string(100 + i * 37, (char)('A' + i)));
            offs.push_back(w.offset());
            ASSERT_EQ(w.Write(r), 0);
        }
        ASSERT_EQ(w.Flush(), 0);
    }
    RecordReader rd(path);
    ASSERT_TRUE(rd.ok());
    for (int i : {13, 2, 19, 0, 7}) {
        ASSERT_TRUE(rd.SeekTo(offs[i]));
        Record r;
        ASSERT_TRUE(rd.ReadNext(&r));
        EXPECT_EQ(r.Meta("idx")->to_string(), std::to_string(i));
        EXPECT_EQ(r.Payload().size(), (size_t)(100 + i * 37));
        EXPECT_EQ(rd.last_offset(), offs[i]);
    }
    unlink(path.c_str());
}

TEST(ButilMore, record_file_truncated_tail_ends_cleanly) {
    const std::string path = tmp_path("trunc");
    {
        RecordWriter w(path);
        for (int i = 0; i < 3; ++i) {
            Record r;
            r.MutablePayload()->append(std::string(500, 'z'));
            ASSERT_EQ(w.Write(r), 0);
        }
        w.Flush();
    }
    // cut the last record in half
    FILE* f = fopen(path.c_str(), "rb");
    fseek(f, 0, SEEK_END);
    const long size = ftell(f);
    fclose(f);
    ASSERT_EQ(truncate(path.c_str(), size - 250), 0);
    RecordReader rd(path);
    Record r;
    int n = 0;
    while (rd.ReadNext(&r)) ++n;
    EXPECT_EQ(n, 2);
    unlink(path.c_str());
}

TEST(ButilMore, record_metas_add_replace_remove) {
    Record r;
    r.MutableMeta("a")->append("1");
    EXPECT_TRUE(r.MutableMeta("a", /*null_on_found=*/true) == nullptr);
    r.MutableMeta("a")->append("2");  // same meta, appended
    EXPECT_EQ(r.Meta("a")->to_string(), "12");
    r.MutableMeta("b")->append("x");
    EXPECT_EQ(r.MetaCount(), 2u);
    EXPECT_TRUE(r.RemoveMeta("a"));
    EXPECT_FALSE(r.RemoveMeta("a"));
    EXPECT_TRUE(r.Meta("a") == nullptr);
    EXPECT_EQ(r.MetaAt(0).first, "b");
    const size_t with_meta = r.ByteSize();
    r.Clear();
    EXPECT_EQ(r.MetaCount(), 0u);
    EXPECT_LT(r.ByteSize(), with_meta);
}

TEST(ButilMore, fast_rand_ranges_and_spread) {
    std::set<uint64_t> seen;
    for (int i = 0; i < 20000; ++i) {
        const uint64_t v = fast_rand_less_than(10);
        ASSERT_LT(v, 10u);
        seen.insert(v);
        const int64_t w = fast_rand_in(-3, 3);
        ASSERT_GE(w, -3);
        ASSERT_LE(w, 3);
        const double d = fast_rand_double();
        ASSERT_GE(d, 0.0);
        ASSERT_LT(d, 1.0);
    }
    EXPECT_EQ(seen.size(), 10u);
    EXPECT_EQ(fast_rand_less_than(1), 0u);
    EXPECT_EQ(fast_rand_in(5, 5), 5);
}

TEST(ButilMore, fast_rand_buckets_are_roughly_uniform) {
    int bucket[8] = {0};
    const int n = 80000;
    for (int i = 0; i < n; ++i) ++bucket[fast_rand_less_than(8)];
    for (int b : bucket) {
        EXPECT_GT(b, n / 8 * 9 / 10);
        EXPECT_LT(b, n / 8 * 11 / 10);
    }
}

TEST(ButilMore, string_appendf_and_case_helpers) {
    std::string s = "n=";
    string_appendf(&s, "%d,%s", 42, "ok");
    EXPECT_EQ(s, "n=42,ok");
    string_appendf(&s, "%s", std::string(5000, 'q').c_str());
    EXPECT_EQ(s.size(), 7u + 5000u);
    EXPECT_EQ(to_lower("MiXeD-09"), "mixed-09");
    EXPECT_TRUE(iequals("Content-Type", "content-type"));
    EXPECT_FALSE(iequals("abc", "abcd"));
    EXPECT_TRUE(starts_with("prefix-rest", "prefix"));
    EXPECT_FALSE(starts_with("pre", "prefix"));
    EXPECT_TRUE(ends_with("file.proto", ".proto"));
    EXPECT_FALSE(ends_with("o", ".proto"));
}

TEST(ButilMore, split_then_join_round_trips) {
    const std::string s = "a,b,,c,";
    const std::vector<std::string> keep = split_string(s, ',', /*skip_empty=*/false);
    ASSERT_EQ(keep.size(), 5u);
    EXPECT_EQ(join(keep, ","), s);
    const std::vector<std::string> skip = split_string(s, ',');
    EXPECT_EQ(join(skip, "|"), "a|b|c");
    EXPECT_TRUE(split_string("", ',').empty());
}

TEST(ButilMore, byte_order_helpers_round_trip) {
    unsigned char buf[8];
    pack_be16(buf, 0x1234);
    EXPECT_EQ(buf[0], 0x12);
    EXPECT_EQ(unpack_be16(buf), 0x1234);
    pack_be64(buf, 0x0102030405060708ull);
    EXPECT_EQ(buf[0], 0x01);
    EXPECT_EQ(buf[7], 0x08);
    EXPECT_EQ(unpack_be64(buf), 0x0102030405060708ull);
    pack_le32(buf, 0xA1B2C3D4);
    EXPECT_EQ(buf[0], 0xD4);
    EXPECT_EQ(unpack_le32(buf), 0xA1B2C3D4u);
}

TEST(ButilMore, md5_hash32_is_stable_and_spreads) {
    const uint32_t a = md5_hash32("key-1", 5), b = md5_hash32("key-1", 5), c = md5_hash32("key-2", 5);
    EXPECT_EQ(a, b);
    EXPECT_NE(a, c);
    std::set<uint32_t> hs;
    for (int i = 0; i < 1000; ++i) {
        const std::string k = "server-" + std::to_string(i);
        hs.insert(md5_hash32(k.data(), k.size()));
    }
    EXPECT_EQ(hs.size(), 1000u);
}

TEST(ButilMore, crc32c_extend_equals_one_shot) {
    std::string s(10000, 0);
    for (size_t i = 0; i < s.size(); ++i) s[i] = (char)(i * 131 + 7);
    const uint32_t one = crc32c::Value(s.data(), s.size());
    uint32_t inc = 0;
    for (size_t off = 0; off < s.size(); off += 777) inc = crc32c::Extend(inc, s.data() + off, std::min<size_t>(777, s.size() - off));
    EXPECT_EQ(one, inc);
    EXPECT_EQ(crc32c::Value("123456789", 9), 0xE3069283u);  // the CRC-32C check value
    // crc(A || B) from crc(A), crc(B) and |B| (no pass over A)
    const uint32_t ca = crc32c::Value(s.data(), 4000), cb = crc32c::Value(s.data() + 4000, 6000);
    EXPECT_EQ(crc32c::Combine(ca, cb, 6000), one);
}

TEST(ButilMore, time_helpers_normalise_and_advance) {
    const timespec ts = ns_to_timespec(3500000123ll);
    EXPECT_EQ(ts.tv_sec, 3);
    EXPECT_EQ(ts.tv_nsec, 500000123);
    const timespec later = realtime_after_us(1500000);
    const int64_t now_us = realtime_us();
    const int64_t later_us = (int64_t)later.tv_sec * 1000000 + later.tv_nsec / 1000;
    EXPECT_GE(later_us - now_us, 1400000);
    EXPECT_LE(later_us - now_us, 1600000);
    EXPECT_LT(later.tv_nsec, 1000000000);
    const int64_t a = monotonic_ns();
    const int64_t b = monotonic_ns();
    EXPECT_GE(b, a);
    EXPECT_EQ(monotonic_ms(), monotonic_ns() / 1000000);
}

TEST(ButilMore, flags_typed_forms) {
    EXPECT_TRUE(SetFlag("butil_more_test_i32", "0x10"));
    EXPECT_EQ(FLAGS_butil_more_test_i32, 16);
    EXPECT_FALSE(SetFlag("butil_more_test_i32", "3000000000"));  // out of int32 range
    EXPECT_FALSE(SetFlag("butil_more_test_u64", "-1"));
    EXPECT_TRUE(SetFlag("butil_more_test_u64", "18446744073709551615"));
    EXPECT_EQ(FLAGS_butil_more_test_u64, 18446744073709551615ull);
    EXPECT_TRUE(SetFlag("butil_more_test_d", "2.5e-3"));
    EXPECT_NEAR(FLAGS_butil_more_test_d, 0.0025, 1e-12);
    EXPECT_FALSE(SetFlag("butil_more_test_d", "1.0x"));
    EXPECT_TRUE(SetFlag("butil_more_test_s", "a=b=c"));
    EXPECT_EQ(FLAGS_butil_more_test_s, "a=b=c");
    for (const char* v : {"yes", "on", "1", "true"}) {
        EXPECT_TRUE(SetFlag("butil_more_test_b", "false"));
        EXPECT_TRUE(SetFlag("butil_more_test_b", v));
        EXPECT_TRUE(FLAGS_butil_more_test_b);
    }
    EXPECT_FALSE(SetFlag("butil_more_test_b", "maybe"));
    std::string cur;
    EXPECT_TRUE(GetFlag("butil_more_test_d", &cur));
    EXPECT_EQ(cur, "0.0025");
    EXPECT_FALSE(GetFlag("no_such_flag_here", &cur));
}

TEST(ButilMore, command_line_negation_and_separate_values) {
    std::vector<std::string> args = {"prog", "--nobutil_more_test_b", "-butil_more_test_i32", "21", "rest",
                                     "--butil_more_test_s=hello"};
    std::vector<char*> argv;
    for (std::string& a : args) argv.push_back(&a[0]);
    FLAGS_butil_more_test_b = true;
    int argc = (int)argv.size();
    char** av = argv.data();
    EXPECT_EQ(ParseCommandLineFlags(&argc, &av, true), 3);
    EXPECT_FALSE(FLAGS_butil_more_test_b);
    EXPECT_EQ(FLAGS_butil_more_test_i32, 21);
    EXPECT_EQ(FLAGS_butil_more_test_s, "hello");
    ASSERT_EQ(argc, 2);
    EXPECT_EQ(std::string(av[1]), "rest");
}

TEST(ButilMore, list_flags_is_sorted_and_has_defaults) {
    const std::vector<FlagInfo> all = ListFlags();
    ASSERT_GT(all.size(), 10u);
    for (size_t i = 1; i < all.size(); ++i) EXPECT_LT(all[i - 1].name, all[i].name);
    FlagInfo fi;
    ASSERT_TRUE(GetFlagInfo("butil_more_test_i32", &fi));
    EXPECT_EQ(fi.default_value, "7");
    EXPECT_EQ(fi.type, "int32");
}
