// Focused unit tests of the base layer (spirit of the reference's
// test/iobuf_unittest.cpp, flat_map_unittest.cpp, bounded_queue_unittest.cpp,
// crc32c_unittest.cpp, snappy_unittest.cpp, string_printf_unittest.cpp,
// endpoint_unittest.cpp, recordio_unittest.cpp): one behaviour per case.
#include <fcntl.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "base/buf.h"
#include "base/containers.h"
#include "base/crc32c.h"
#include "base/endpoint.h"
#include "base/recordio.h"
#include "base/snappy.h"
#include "base/util.h"
#include "json/json.h"
#include "tests/test.h"

using namespace mrpc;

namespace {
std::string RandomBytes(size_t n, uint32_t seed) {
    std::mt19937 g(seed);
    std::string s(n, '\0');
    for (auto& c : s) c = (char)(g() & 0xff);
    return s;
}
}  // namespace

// ------------------------------------------------------------------ Buf
TEST(BufUnit, empty_buf_properties) {
    Buf b;
    EXPECT_TRUE(b.empty());
    EXPECT_EQ(b.size(), 0u);
    EXPECT_EQ(b.backing_block_num(), 0u);
    EXPECT_EQ(b.to_string(), "");
    char c;
    EXPECT_FALSE(b.cut1(&c));
    EXPECT_EQ(b.pop_front(10), 0u);
    EXPECT_EQ(b.pop_back(10), 0u);
}

TEST(BufUnit, pop_back_across_blocks) {
    Buf b;
    const std::string s = RandomBytes(20000, 1);
    b.append(s);
    EXPECT_EQ(b.pop_back(12345), 12345u);
    EXPECT_TRUE(b.equals(s.substr(0, s.size() - 12345)));
    EXPECT_EQ(b.pop_back(100000), s.size() - 12345);
    EXPECT_TRUE(b.empty());
}

TEST(BufUnit, copy_to_with_offset) {
    Buf b;
    const std::string s = RandomBytes(30000, 2);
    b.append(s);
    std::string out;
    EXPECT_EQ(b.copy_to(&out, 1000, 12000), 1000u);
    EXPECT_EQ(out, s.substr(12000, 1000));
    char raw[64];
    EXPECT_EQ(b.copy_to(raw, 64, s.size() - 10), 10u);  // clipped at the end
    EXPECT_EQ(memcmp(raw, s.data() + s.size() - 10, 10), 0);
    EXPECT_EQ(b.size(), s.size());  // copy_to does not consume
}

TEST(BufUnit, cutn_into_string_and_raw) {
    Buf b("hello world");
    std::string head;
    EXPECT_EQ(b.cutn(&head, 5), 5u);
    EXPECT_EQ(head, "hello");
    char rest[16] = {0};
    EXPECT_EQ(b.cutn(rest, 100), 6u);
    EXPECT_EQ(std::string(rest), " world");
    EXPECT_TRUE(b.empty());
}

TEST(BufUnit, copies_share_blocks_and_are_independent) {
    Buf a;
    a.append(RandomBytes(10000, 3));
    const int64_t blocks = Buf::block_count();
    Buf b(a);  // shares blocks: no new memory
    EXPECT_EQ(Buf::block_count(), blocks);
    EXPECT_TRUE(b.equals(a.to_string()));
    b.pop_front(100);
    a.append("tail");
    EXPECT_EQ(a.size(), 10004u);
    EXPECT_EQ(b.size(), 9900u);
}

TEST(BufUnit, move_leaves_source_empty) {
    Buf a("payload");
    Buf b(std::move(a));
    EXPECT_TRUE(a.empty());
    EXPECT_EQ(b.to_string(), "payload");
    Buf c;
    c = std::move(b);
    EXPECT_TRUE(b.empty());
    EXPECT_EQ(c.to_string(), "payload");
}

TEST(BufUnit, swap_exchanges_contents) {
    Buf a("aaa"), b("bbbbbb");
    a.swap(b);
    EXPECT_EQ(a.to_string(), "bbbbbb");
    EXPECT_EQ(b.to_string(), "aaa");
}

TEST(BufUnit, append_buf_concatenates) {
    Buf a("12"), b("345");
    a.append(b);
    EXPECT_EQ(a.to_string(), "12345");
    EXPECT_EQ(b.to_string(), "345");  // copy-append keeps the source
    a.append(std::move(b));
    EXPECT_EQ(a.to_string(), "12345345");
    EXPECT_TRUE(b.empty());
}

TEST(BufUnit, fetch_contiguous_or_aux) {
    Buf b;
    b.append("abc");
    Buf big;
    big.append(RandomBytes(9000, 4));  // likely spans blocks
    b.append(big);
    char aux[16];
    const char* p = static_cast<const char*>(b.fetch(aux, 3));
    EXPECT_EQ(std::string(p, 3), "abc");
    EXPECT_EQ(*b.fetch1(), 'a');
    EXPECT_TRUE(b.fetch(aux, b.size() + 1) == nullptr);
}

TEST(BufUnit, cut_until_delimiter) {
    Buf b("k1=v1&k2=v2&tail");
    Buf out;
    ASSERT_EQ(b.cut_until(&out, "&"), 0);
    EXPECT_EQ(out.to_string(), "k1=v1");
    out.clear();
    ASSERT_EQ(b.cut_until(&out, "&"), 0);
    EXPECT_EQ(out.to_string(), "k2=v2");
    out.clear();
    EXPECT_NE(b.cut_until(&out, "&"), 0);  // no delimiter left
    EXPECT_EQ(b.to_string(), "tail");
}

TEST(BufUnit, bytes_iterator_walks_every_byte) {
    const std::string s = RandomBytes(17000, 5);
    Buf b;
    b.append(s);
    BufBytesIterator it(b);
    size_t i = 0;
    bool same = true;
    for (; !it.done(); ++it, ++i) same = same && (*it == s[i]);
    EXPECT_TRUE(same);
    EXPECT_EQ(i, s.size());
    BufBytesIterator it2(b);
    EXPECT_EQ(it2.forward(1000), 1000u);
    char tmp[8];
    EXPECT_EQ(it2.copy_and_forward(tmp, 8), 8u);
    EXPECT_EQ(memcmp(tmp, s.data() + 1000, 8), 0);
    EXPECT_EQ(it2.bytes_left(), s.size() - 1008);
}

TEST(BufUnit, fill_iov_covers_blocks) {
    Buf b;
    const std::string s = RandomBytes(50000, 6);
    b.append(s);
    struct iovec iov[64];
    size_t n = 0;
    const int k = b.fill_iov(iov, 64, (size_t)-1, &n);
    EXPECT_GT(k, 0);
    EXPECT_EQ(n, s.size());
    std::string joined;
    for (int i = 0; i < k; ++i) joined.append((const char*)iov[i].iov_base, iov[i].iov_len);
    EXPECT_EQ(joined, s);
    size_t m = 0;
    // the byte budget is a hint in whole blocks: stop after the block that reaches it
    EXPECT_EQ(b.fill_iov(iov, 64, 100, &m), 1);
    EXPECT_EQ(m, b.block_len(0));
    EXPECT_EQ(b.fill_iov(iov, 2, (size_t)-1, &m), 2);  // iov budget
}

TEST(BufUnit, cut_into_fd_and_portal_read_back) {
    int fds[2];
    ASSERT_EQ(pipe(fds), 0);
    fcntl(fds[0], F_SETFL, O_NONBLOCK);
    const std::string s = RandomBytes(4000, 7);
    Buf b;
    b.append(s);
    EXPECT_EQ(b.cut_into_fd(fds[1]), (ssize_t)s.size());
    EXPECT_TRUE(b.empty());
    BufPortal in;
    EXPECT_EQ(in.append_from_fd(fds[0], 1 << 20), (ssize_t)s.size());
    EXPECT_TRUE(in.equals(s));
    close(fds[0]);
    close(fds[1]);
}

TEST(BufUnit, append_contiguous_reserves_in_place) {
    Buf b;
    char* p = b.append_contiguous(100);
    ASSERT_TRUE(p != nullptr);
    memset(p, 'z', 100);
    EXPECT_EQ(b.size(), 100u);
    EXPECT_EQ(b.to_string(), std::string(100, 'z'));
}

// ------------------------------------------------------------ containers
TEST(FlatMapUnit, erase_keeps_probe_chains) {
    FlatMap<int, int> m(8);
    for (int i = 0; i < 1000; ++i) m[i * 64] = i;  // many collisions in a small table
    for (int i = 0; i < 1000; i += 2) EXPECT_EQ(m.erase(i * 64), 1u);
    EXPECT_EQ(m.size(), 500u);
    bool ok = true;
    for (int i = 0; i < 1000; ++i) {
        const int* v = m.seek(i * 64);
        ok = ok && ((i % 2) ? (v && *v == i) : v == nullptr);
    }
    EXPECT_TRUE(ok);
    EXPECT_EQ(m.erase(12345), 0u);
}

TEST(FlatMapUnit, iteration_visits_every_entry_once) {
    FlatMap<std::string, int> m;
    for (int i = 0; i < 300; ++i) m["k" + std::to_string(i)] = i;
    int sum = 0, n = 0;
    for (auto& kv : m) {
        sum += kv.second;
        ++n;
    }
    EXPECT_EQ(n, 300);
    EXPECT_EQ(sum, 299 * 300 / 2);
    m.clear();
    EXPECT_TRUE(m.empty());
    EXPECT_TRUE(m.begin() == m.end());
}

TEST(BoundedQueueUnit, fifo_and_capacity) {
    BoundedQueue<int> q(3);
    EXPECT_TRUE(q.empty());
    EXPECT_TRUE(q.push(1));
    EXPECT_TRUE(q.push(2));
    EXPECT_TRUE(q.push(3));
    EXPECT_TRUE(q.full());
    EXPECT_FALSE(q.push(4));
    int v = 0;
    EXPECT_TRUE(q.pop(&v));
    EXPECT_EQ(v, 1);
    EXPECT_TRUE(q.push(4));  // wraps around
    std::vector<int> got;
    while (q.pop(&v)) got.push_back(v);
    EXPECT_EQ(got.size(), 3u);
    EXPECT_EQ(got[0], 2);
    EXPECT_EQ(got[2], 4);
}

TEST(MRUCacheUnit, get_refreshes_recency) {
    MRUCache<int, std::string> c(2);
    c.Put(1, "one");
    c.Put(2, "two");
    ASSERT_TRUE(c.Get(1) != nullptr);  // 1 becomes most recent
    int evicted = -1;
    c.Put(3, "three", &evicted);
    EXPECT_EQ(evicted, 2);
    EXPECT_TRUE(c.Peek(2) == nullptr);
    EXPECT_EQ(*c.Peek(1), "one");
    EXPECT_TRUE(c.Erase(1));
    EXPECT_FALSE(c.Erase(1));
}

TEST(DoublyBufferedDataUnit, readers_never_see_torn_updates) {
    DoublyBufferedData<std::vector<int>> d;
    d.Modify([](std::vector<int>& v) {
        v.assign(64, 0);
        return (size_t)1;
    });
    std::atomic<bool> stop{false}, torn{false};
    std::vector<std::thread> readers;
    for (int t = 0; t < 4; ++t) {
        readers.emplace_back([&] {
            while (!stop.load()) {
                DoublyBufferedData<std::vector<int>>::ScopedPtr p;
                if (d.Read(&p) != 0) continue;
                const std::vector<int>& v = *p;
                for (int x : v) {
                    if (x != v[0]) torn = true;
                }
            }
        });
    }
    for (int gen = 1; gen <= 200; ++gen) {
        d.Modify([gen](std::vector<int>& v) {
            for (int& x : v) x = gen;
            return (size_t)1;
        });
    }
    stop = true;
    for (auto& t : readers) t.join();
    EXPECT_FALSE(torn.load());
}

// ------------------------------------------------------------------ crc
TEST(Crc32cUnit, extend_equals_one_shot) {
    const std::string s = RandomBytes(100003, 8);
    const uint32_t whole = crc32c::Value(s.data(), s.size());
    uint32_t c = 0;
    for (size_t off = 0; off < s.size(); off += 977) {
        c = crc32c::Extend(c, s.data() + off, std::min<size_t>(977, s.size() - off));
    }
    EXPECT_EQ(c, whole);
}

TEST(Crc32cUnit, combine_matches_concatenation) {
    const std::string a = RandomBytes(3000, 9), b = RandomBytes(12345, 10);
    const uint32_t ca = crc32c::Value(a.data(), a.size()), cb = crc32c::Value(b.data(), b.size());
    const std::string ab = a + b;
    EXPECT_EQ(crc32c::Combine(ca, cb, b.size()), crc32c::Value(ab.data(), ab.size()));
    EXPECT_EQ(crc32c::Combine(ca, crc32c::Value("", 0), 0), ca);
}

TEST(Crc32cUnit, rfc3720_vectors) {
    char zeros[32] = {0}, ones[32], inc[32], dec[32];
    memset(ones, 0xff, 32);
    for (int i = 0; i < 32; ++i) {
        inc[i] = (char)i;
        dec[i] = (char)(31 - i);
    }
    EXPECT_EQ(crc32c::Value(zeros, 32), 0x8a9136aau);
    EXPECT_EQ(crc32c::Value(ones, 32), 0x62a8ab43u);
    EXPECT_EQ(crc32c::Value(inc, 32), 0x46dd794eu);
    EXPECT_EQ(crc32c::Value(dec, 32), 0x113fdb5cu);
}

// ---------------------------------------------------------------- snappy
TEST(SnappyUnit, roundtrip_many_shapes) {
    std::vector<std::string> inputs = {"", "a", std::string(100000, 'x'), RandomBytes(70000, 11)};
    std::string text;
    for (int i = 0; i < 5000; ++i) text += "word" + std::to_string(i % 97) + " ";
    inputs.push_back(text);
    for (const std::string& in : inputs) {
        std::string c, d;
        ASSERT_TRUE(snappy::Compress(in.data(), in.size(), &c));
        EXPECT_LE(c.size(), snappy::MaxCompressedLength(in.size()));
        size_t ulen = 0;
        ASSERT_TRUE(snappy::GetUncompressedLength(c.data(), c.size(), &ulen));
        EXPECT_EQ(ulen, in.size());
        EXPECT_TRUE(snappy::IsValidCompressedBuffer(c.data(), c.size()));
        ASSERT_TRUE(snappy::Uncompress(c.data(), c.size(), &d));
        EXPECT_TRUE(d == in);
    }
}

// Hand-built streams of every copy shape (offsets 1..70, lengths 1..64,
// copies ending at the very end of the output where the word-at-a-time path
// has no room) against a byte-by-byte reference decoder.
TEST(SnappyUnit, copy_paths_match_a_naive_decoder) {
    std::mt19937 rng(9);
    for (int trial = 0; trial < 3000; ++trial) {
        std::string stream, want;
        // a literal first so every offset has history
        const size_t lit = 1 + rng() % 60;  // one-byte literal tag
        std::string l = RandomBytes(lit, trial);
        std::string body;
        body.push_back((char)((lit - 1) << 2));
        body += l;
        want += l;
        const int ncopies = 1 + (int)(rng() % 12);
        for (int c = 0; c < ncopies; ++c) {
            const size_t off = 1 + rng() % std::min<size_t>(70, want.size());
            const size_t len = 1 + rng() % 64;
            body.push_back((char)(((len - 1) << 2) | 2));  // copy with a 2-byte offset
            body.push_back((char)(off & 0xff));
            body.push_back((char)(off >> 8));
            for (size_t i = 0; i < len; ++i) want.push_back(want[want.size() - off]);
        }
        size_t n = want.size();
        do {  // varint of the uncompressed length
            stream.push_back((char)((n & 0x7f) | (n >= 0x80 ? 0x80 : 0)));
            n >>= 7;
        } while (n);
        stream += body;
        std::string got;
        ASSERT_TRUE(snappy::Uncompress(stream.data(), stream.size(), &got));
        ASSERT_TRUE(got == want);
    }
}

TEST(SnappyUnit, compressible_input_shrinks) {
    const std::string in(1 << 20, 'q');
    std::string c;
    ASSERT_TRUE(snappy::Compress(in.data(), in.size(), &c));
    EXPECT_LT(c.size(), in.size() / 20);
}

TEST(SnappyUnit, corrupted_streams_are_rejected) {
    std::string text;
    for (int i = 0; i < 2000; ++i) text += "abcdefgh" + std::to_string(i);
    std::string c, d;
    ASSERT_TRUE(snappy::Compress(text.data(), text.size(), &c));
    EXPECT_FALSE(snappy::Uncompress(c.data(), c.size() / 2, &d));  // truncated
    std::string bad = c;
    bad[0] = (char)0xff;  // length varint runs past the end / too large
    bad[1] = (char)0xff;
    bad[2] = (char)0xff;
    bad[3] = (char)0xff;
    bad[4] = (char)0xff;
    EXPECT_FALSE(snappy::Uncompress(bad.data(), bad.size(), &d));
    // a copy whose offset points before the start of the output
    const char evil[] = {10, (char)0x01 | (char)(1 << 2), 100};  // len 10; copy-1 of 5 at offset 100
    EXPECT_FALSE(snappy::IsValidCompressedBuffer(evil, sizeof(evil)));
}

// ------------------------------------------------------------------ util
TEST(UtilUnit, split_trim_join) {
    EXPECT_EQ(split_string("a,,b,c", ',').size(), 3u);
    EXPECT_EQ(split_string("a,,b,c", ',', false).size(), 4u);
    EXPECT_EQ(split_string_any("a b;c", " ;").size(), 3u);
    EXPECT_EQ(trim("  x y \t\n"), "x y");
    EXPECT_EQ(join({"a", "b", "c"}, "-"), "a-b-c");
    EXPECT_TRUE(starts_with("prefix_rest", "prefix"));
    EXPECT_FALSE(starts_with("pre", "prefix"));
    EXPECT_TRUE(ends_with("file.proto", ".proto"));
    EXPECT_TRUE(iequals("Content-Type", "content-type"));
    EXPECT_EQ(to_lower("MiXeD"), "mixed");
}

TEST(UtilUnit, parse_int64_strict) {
    int64_t v = 0;
    EXPECT_TRUE(parse_int64("-9223372036854775808", &v));
    EXPECT_EQ(v, INT64_MIN);
    EXPECT_TRUE(parse_int64("42", &v));
    EXPECT_EQ(v, 42);
    EXPECT_FALSE(parse_int64("42x", &v));
    EXPECT_FALSE(parse_int64("", &v));
    EXPECT_FALSE(parse_int64("99999999999999999999", &v));
}

TEST(UtilUnit, url_and_base64_roundtrips) {
    const std::string raw = "a b&c=d/é?";
    EXPECT_EQ(url_decode(url_encode(raw)), raw);
    EXPECT_EQ(url_decode("a%20b+c"), "a b c");
    const std::string bin = RandomBytes(1000, 12);
    std::string back;
    ASSERT_TRUE(base64_decode(base64_encode(bin.data(), bin.size()), &back));
    EXPECT_TRUE(back == bin);
    EXPECT_EQ(base64_encode("foobar", 6), "Zm9vYmFy");
    EXPECT_EQ(base64_encode("fo", 2), "Zm8=");
    EXPECT_FALSE(base64_decode("Zm9v!", &back));
}

TEST(UtilUnit, hashes_known_values) {
    unsigned char d[16];
    md5("", 0, d);
    EXPECT_EQ(hex_dump(d, 16, 16).find("d41d8cd9") != std::string::npos ||
                  string_printf("%02x%02x%02x%02x", d[0], d[1], d[2], d[3]) == "d41d8cd9",
              true);
    EXPECT_EQ(sha1_hex("abc", 3), "a9993e364706816aba3e25717850c26c9cd0d89d");
    EXPECT_EQ(murmurhash3_32("", 0, 0), 0u);
    EXPECT_NE(murmurhash3_32("a", 1, 0), murmurhash3_32("b", 1, 0));
}

TEST(UtilUnit, html_escape_and_printf) {
    EXPECT_EQ(html_escape("<a href=\"x\">&</a>"), "&lt;a href=&quot;x&quot;&gt;&amp;&lt;/a&gt;");
    std::string s = string_printf("%d-%s", 7, "x");
    string_appendf(&s, "+%05.1f", 2.5);
    EXPECT_EQ(s, "7-x+002.5");
    const std::string big(5000, 'b');
    EXPECT_EQ(string_printf("%s", big.c_str()).size(), 5000u);
}

TEST(UtilUnit, fast_rand_ranges) {
    bool ok = true;
    for (int i = 0; i < 10000; ++i) {
        ok = ok && fast_rand_less_than(7) < 7;
        const int64_t v = fast_rand_in(-3, 3);
        ok = ok && v >= -3 && v <= 3;
        const double d = fast_rand_double();
        ok = ok && d >= 0 && d < 1;
    }
    EXPECT_TRUE(ok);
}

TEST(UtilUnit, big_endian_packing) {
    char b[8];
    pack_be32(b, 0x01020304);
    EXPECT_EQ((int)b[0], 1);
    EXPECT_EQ(unpack_be32(b), 0x01020304u);
    pack_be64(b, 0x0102030405060708ULL);
    EXPECT_EQ((int)b[7], 8);
    EXPECT_EQ(unpack_be64(b), 0x0102030405060708ULL);
    pack_be16(b, 0xabcd);
    EXPECT_EQ(unpack_be16(b), 0xabcd);
}

// -------------------------------------------------------------- endpoint
TEST(EndPointUnit, parse_and_format) {
    EndPoint ep;
    ASSERT_EQ(str2endpoint("127.0.0.1:8080", &ep), 0);
    EXPECT_EQ(ep.port, 8080);
    EXPECT_EQ(ep.to_string(), "127.0.0.1:8080");
    EXPECT_NE(str2endpoint("127.0.0.1", &ep), 0);
    EXPECT_NE(str2endpoint("127.0.0.1:99999", &ep), 0);
    EXPECT_NE(str2endpoint("not-an-ip:80", &ep), 0);
    EndPoint a, b;
    str2endpoint("10.0.0.1:1", &a);
    str2endpoint("10.0.0.1:2", &b);
    EXPECT_TRUE(a < b);
    EXPECT_FALSE(a == b);
}

// -------------------------------------------------------------- recordio
TEST(RecordIOUnit, metas_payload_and_offsets) {
    char path[] = "/tmp/mrpc_recordio_XXXXXX";
    const int fd = mkstemp(path);
    ASSERT_GE(fd, 0);
    close(fd);
    std::vector<uint64_t> offsets;
    {
        RecordWriter w(path);
        ASSERT_TRUE(w.ok());
        for (int i = 0; i < 50; ++i) {
            Record r;
            r.MutableMeta("idx")->append(std::to_string(i));
            r.MutablePayload()->append(RandomBytes(100 + i * 37, i));
            offsets.push_back(w.offset());
            ASSERT_EQ(w.Write(r), 0);
        }
        w.Flush();
    }
    RecordReader rd(path);
    Record r;
    // random access through the offsets
    ASSERT_TRUE(rd.SeekTo(offsets[31]));
    ASSERT_TRUE(rd.ReadNext(&r));
    EXPECT_EQ(rd.last_offset(), offsets[31]);
    EXPECT_EQ(r.Meta("idx")->to_string(), "31");
    EXPECT_EQ(r.Payload().to_string(), RandomBytes(100 + 31 * 37, 31));
    ASSERT_TRUE(rd.SeekTo(0));
    int n = 0;
    while (rd.ReadNext(&r)) ++n;
    EXPECT_EQ(n, 50);
    EXPECT_EQ(rd.last_error(), 0);
    unlink(path);
}

TEST(RecordIOUnit, corruption_skips_one_record) {
    char path[] = "/tmp/mrpc_recordio_XXXXXX";
    const int fd = mkstemp(path);
    ASSERT_GE(fd, 0);
    close(fd);
    uint64_t second = 0;
    {
        RecordWriter w(path);
        for (int i = 0; i < 3; ++i) {
            Record r;
            r.MutablePayload()->append("record-" + std::to_string(i));
            if (i == 1) second = w.offset();
            w.Write(r);
        }
    }
    // flip a payload byte of the second record
    FILE* f = fopen(path, "r+b");
    ASSERT_TRUE(f != nullptr);
    fseek(f, (long)second + 14, SEEK_SET);
    fputc('X', f);
    fclose(f);
    RecordReader rd(path);
    Record r;
    std::vector<std::string> got;
    while (rd.ReadNext(&r)) got.push_back(r.Payload().to_string());
    ASSERT_EQ(got.size(), 2u);
    EXPECT_EQ(got[0], "record-0");
    EXPECT_EQ(got[1], "record-2");
    EXPECT_GT(rd.skipped_bytes(), 0u);
    unlink(path);
}

// ------------------------------------------------------------------ json
TEST(JsonUnit, parse_types_and_serialize) {
    json::Value v;
    std::string err;
    ASSERT_TRUE(json::Parse(R"({"a":1,"b":-2,"c":1.5,"d":"xé\n","e":[true,false,null],"f":{"g":18446744073709551615}})",
                            &v, &err));
    EXPECT_TRUE(v.is_object());
    EXPECT_EQ(v.find("a")->as_int(), 1);
    EXPECT_EQ(v.find("b")->as_int(), -2);
    EXPECT_EQ(v.find("c")->as_double(), 1.5);
    EXPECT_EQ(v.find("d")->as_string(), "x\xc3\xa9\n");
    EXPECT_EQ(v.find("e")->size(), 3u);
    EXPECT_TRUE(v.find("e")->array()[2].is_null());
    EXPECT_TRUE(v.find("f")->find("g")->uint_overflows_int());
    EXPECT_EQ(v.find("f")->find("g")->as_uint(), 18446744073709551615ULL);
    json::Value back;
    ASSERT_TRUE(json::Parse(v.ToString(), &back));
    EXPECT_EQ(back.ToString(), v.ToString());
    EXPECT_TRUE(v.find("missing") == nullptr);
}

// EscapeString copies plain runs a word at a time: every special byte at
// every offset of an 8-byte word must still be escaped, and every string
// must come back from the parser unchanged (runs split by the memchr scan).
TEST(JsonUnit, escape_specials_at_every_word_offset_and_round_trip) {
    const char specials[] = {'"', '\\', '\n', '\r', '\t', '\b', '\f', '\x01', '\x1f', '\x7f', (char)0x80, (char)0xff};
    for (char sp : specials) {
        for (size_t at = 0; at < 19; ++at) {
            std::string raw(19, 'a');
            raw[at] = sp;
            std::string esc;
            json::EscapeString(raw, &esc);
            const unsigned char u = (unsigned char)sp;
            if (u < 0x20 || sp == '"' || sp == '\\') {
                EXPECT_TRUE(esc.size() > raw.size() + 2);  // escaped
            } else {
                EXPECT_EQ(esc, "\"" + raw + "\"");  // 0x7f and high bytes pass through
            }
            json::Value v;
            ASSERT_TRUE(json::Parse(esc, &v));
            EXPECT_EQ(v.as_string(), raw);
        }
    }
    std::mt19937 rng(17);
    for (int t = 0; t < 200; ++t) {
        std::string raw(rng() % 300, '\0');
        for (auto& c : raw) c = (rng() % 10 == 0) ? (char)(rng() % 0x22) : (char)('a' + rng() % 26);
        std::string esc = "prefix";  // appends after existing content
        json::EscapeString(raw, &esc);
        ASSERT_EQ(esc.compare(0, 6, "prefix"), 0);
        json::Value v;
        ASSERT_TRUE(json::Parse(esc.substr(6), &v));
        EXPECT_EQ(v.as_string(), raw);
    }
}

// Host int arrays stay packed (no Value per element); anything that is not
// a plain int64 turns the array into Values with the same contents.
TEST(JsonUnit, packed_int_arrays_and_fallbacks) {
    json::Value v;
    ASSERT_TRUE(json::Parse("[1, -2 ,3,9223372036854775807,-9223372036854775808, 0]", &v));
    ASSERT_TRUE(v.packed_ints() != nullptr);
    const std::vector<int64_t> want = {1, -2, 3, INT64_MAX, INT64_MIN, 0};
    EXPECT_TRUE(*v.packed_ints() == want);
    EXPECT_EQ(v.size(), 6u);
    EXPECT_EQ(v.array()[3].as_int(), INT64_MAX);  // the const view
    EXPECT_EQ(v.ToString(), "[1,-2,3,9223372036854775807,-9223372036854775808,0]");
    const json::Value copy = v;  // copies do not share the view
    EXPECT_EQ(copy.array().size(), 6u);
    // a uint64 beyond int64, a float, a string: element-wise Values
    ASSERT_TRUE(json::Parse("[1,2,18446744073709551615]", &v));
    EXPECT_TRUE(v.packed_ints() == nullptr);
    ASSERT_EQ(v.array().size(), 3u);
    EXPECT_EQ(v.array()[1].as_int(), 2);
    EXPECT_TRUE(v.array()[2].uint_overflows_int());
    ASSERT_TRUE(json::Parse("[1,2.5,\"x\",[3]]", &v));
    EXPECT_TRUE(v.packed_ints() == nullptr);
    ASSERT_EQ(v.array().size(), 4u);
    EXPECT_EQ(v.array()[1].as_double(), 2.5);
    EXPECT_EQ(v.array()[2].as_string(), "x");
    EXPECT_TRUE(v.array()[3].packed_ints() != nullptr);
    ASSERT_TRUE(json::Parse("[1e3, 7]", &v));
    EXPECT_EQ(v.array()[0].as_double(), 1000.0);
    // 20 digits: not an int64 literal
    ASSERT_TRUE(json::Parse("[-92233720368547758080]", &v));
    EXPECT_TRUE(v.array()[0].type() == json::Value::DOUBLE);
    // the packed path still rejects what the element path rejects
    EXPECT_FALSE(json::Parse("[1,2", &v));
    EXPECT_FALSE(json::Parse("[1 2]", &v));
    EXPECT_FALSE(json::Parse("[1,]", &v));
    EXPECT_FALSE(json::Parse("[1.2.3]", &v));
}

TEST(JsonUnit, malformed_inputs) {
    json::Value v;
    std::string err;
    EXPECT_FALSE(json::Parse("{\"a\":}", &v, &err));
    EXPECT_FALSE(err.empty());
    EXPECT_FALSE(json::Parse("[1,2", &v));
    EXPECT_FALSE(json::Parse("{\"a\" 1}", &v));
    EXPECT_FALSE(json::Parse("\"unterminated", &v));
    EXPECT_FALSE(json::Parse("tru", &v));
    EXPECT_FALSE(json::Parse("{} trailing", &v));
    EXPECT_TRUE(json::Parse("  [ ]  ", &v));
    EXPECT_TRUE(v.is_array());
}

// Host structural index with the kernel's semantics (gpu/json_kernels.hip).
static std::vector<uint32_t> json_index_ref(const std::string& t) {
    std::vector<uint32_t> out;
    bool in_str = false, esc = false;
    for (size_t i = 0; i < t.size(); ++i) {
        const char c = t[i];
        const bool escaped = esc;
        esc = c == '\\' && !esc;
        if (c == '"' && !escaped) {
            in_str = !in_str;
            out.push_back((uint32_t)i);
        } else if (!in_str && strchr("{}[]:,", c) && c) {
            out.push_back((uint32_t)i);
        }
    }
    return out;
}

TEST(JsonUnit, parse_with_structural_index) {
    std::string doc = "{\"k\":[";
    for (int i = 0; i < 300; ++i) {
        if (i) doc += ",";
        doc += "{\"s\":\"" + std::string(i % 50, 'x') + (i % 7 == 0 ? "\\\"q\\\\" : "") + "\",\"n\":" +
               std::to_string(i * 1.5) + ",\"b\":" + (i % 2 ? "true" : "null") + "}";
    }
    doc += "],\"t\":\"tail \\u00e9\"}";
    json::Value plain, indexed, wrong;
    std::string err;
    ASSERT_TRUE(json::Parse(doc, &plain, &err));
    const std::vector<uint32_t> idx = json_index_ref(doc);
    ASSERT_TRUE(json::ParseWithIndex(doc.data(), doc.size(), idx.data(), idx.size(), &indexed, &err));
    EXPECT_EQ(indexed.ToString(), plain.ToString());
    EXPECT_EQ(indexed.find("k")->size(), 300u);
    // a wrong index never changes the result: shifted positions, dropped ones
    std::vector<uint32_t> bad = idx;
    for (size_t i = 5; i < bad.size(); i += 3) bad[i] += 1;
    ASSERT_TRUE(json::ParseWithIndex(doc.data(), doc.size(), bad.data(), bad.size(), &wrong, &err));
    EXPECT_EQ(wrong.ToString(), plain.ToString());
    std::vector<uint32_t> sparse;
    for (size_t i = 0; i < idx.size(); i += 2) sparse.push_back(idx[i]);
    ASSERT_TRUE(json::ParseWithIndex(doc.data(), doc.size(), sparse.data(), sparse.size(), &wrong, &err));
    EXPECT_EQ(wrong.ToString(), plain.ToString());
    // malformed input is still reported
    const std::string broken = doc.substr(0, doc.size() - 3);
    const std::vector<uint32_t> bidx = json_index_ref(broken);
    EXPECT_FALSE(json::ParseWithIndex(broken.data(), broken.size(), bidx.data(), bidx.size(), &wrong, &err));
}

TEST(JsonUnit, object_order_and_escaping) {
    json::Value o = json::Value::Object();
    o.set("z", json::Value(1));
    o.set("a", json::Value("q\"uote"));
    o["m"] = json::Value(true);
    const std::string s = o.ToString();
    EXPECT_LT(s.find("\"z\""), s.find("\"a\""));  // insertion order kept
    EXPECT_TRUE(s.find("q\\\"uote") != std::string::npos);
    std::string esc;
    json::EscapeString("\t\x01", &esc);
    EXPECT_TRUE(esc.find("\\t") != std::string::npos);
    EXPECT_TRUE(esc.find("\\u0001") != std::string::npos);
}
