// Base-library depth (in the spirit of the reference's test/*butil* suites:
// string_printf/string_splitter, murmurhash3, md5/sha1, base64, endpoint,
// flat_map, resource_pool/object_pool, mru_cache, bounded_queue, time,
// reloadable flags, crc32c, snappy): known-answer vectors, edge inputs and
// the failure paths. Hash vectors were cross-checked against an independent
// Python implementation (MurmurHash3) and hashlib (MD5, SHA-1).
#include <fcntl.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <map>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "base/containers.h"
#include "base/crc32c.h"
#include "base/endpoint.h"
#include "base/flags.h"
#include "base/pool.h"
#include "base/snappy.h"
#include "base/time.h"
#include "base/util.h"
#include "tests/test.h"

DEFINE_int32(bd_i32, 5, "base depth test flag");
DEFINE_int64(bd_i64, -7, "base depth test flag");
DEFINE_uint64(bd_u64, 9, "base depth test flag");
DEFINE_bool(bd_bool, false, "base depth test flag");
DEFINE_double(bd_double, 1.5, "base depth test flag");
DEFINE_string(bd_str, "x", "base depth test flag");
DEFINE_int32(bd_positive, 3, "base depth test flag with a validator");

using namespace mrpc;

namespace {

std::string hex_of(const unsigned char* d, size_t n) { return hex_dump(d, n, n); }

}  // namespace

// ------------------------------------------------------------------ strings
TEST(BaseDepth, split_skips_or_keeps_empty_fields) {
    const std::vector<std::string> a = split_string(",a,,b,", ',');
    ASSERT_EQ(a.size(), 2u);
    EXPECT_EQ(a[0], "a");
    EXPECT_EQ(a[1], "b");
    const std::vector<std::string> b = split_string(",a,,b,", ',', false);
    ASSERT_EQ(b.size(), 5u);
    EXPECT_EQ(b[0], "");
    EXPECT_EQ(b[2], "");
    EXPECT_EQ(b[4], "");
    EXPECT_EQ(split_string("", ',').size(), 0u);
    EXPECT_EQ(split_string("abc", ',').size(), 1u);
}

TEST(BaseDepth, split_on_any_of_several_separators) {
    const std::vector<std::string> v = split_string_any("a b\tc;;d", " \t;");
    ASSERT_EQ(v.size(), 4u);
    EXPECT_EQ(v[3], "d");
    EXPECT_EQ(split_string_any("a;;b", ";", false).size(), 3u);
}

TEST(BaseDepth, trim_removes_surrounding_whitespace_only) {
    EXPECT_EQ(trim("  a b  "), "a b");
    EXPECT_EQ(trim("\t\n x \r\n"), "x");
    EXPECT_EQ(trim("    "), "");
    EXPECT_EQ(trim(""), "");
    EXPECT_EQ(trim("x"), "x");
}

TEST(BaseDepth, prefix_suffix_and_case) {
    EXPECT_TRUE(starts_with("abc", ""));
    EXPECT_TRUE(starts_with("abc", "ab"));
    EXPECT_FALSE(starts_with("ab", "abc"));
    EXPECT_TRUE(ends_with("abc", "bc"));
    EXPECT_FALSE(ends_with("c", "bc"));
    EXPECT_EQ(to_lower("MiXeD 123"), "mixed 123");
    EXPECT_TRUE(iequals("Content-Type", "content-type"));
    EXPECT_FALSE(iequals("abc", "abcd"));
}

TEST(BaseDepth, join_handles_empty_and_single) {
    EXPECT_EQ(join({}, ","), "");
    EXPECT_EQ(join({"a"}, ","), "a");
    EXPECT_EQ(join({"a", "", "c"}, "--"), "a----c");
}

TEST(BaseDepth, parse_int64_limits_and_garbage) {
    int64_t v = 0;
    EXPECT_TRUE(parse_int64("9223372036854775807", &v));
    EXPECT_EQ(v, INT64_MAX);
    EXPECT_TRUE(parse_int64("-9223372036854775808", &v));
    EXPECT_EQ(v, INT64_MIN);
    EXPECT_TRUE(parse_int64("+12", &v));
    EXPECT_EQ(v, 12);
    EXPECT_FALSE(parse_int64("9223372036854775808", &v));  // overflow
    EXPECT_FALSE(parse_int64("", &v));
    EXPECT_FALSE(parse_int64("12x", &v));
    EXPECT_FALSE(parse_int64("1 2", &v));
}

TEST(BaseDepth, hex_dump_marks_truncation) {
    const unsigned char d[] = {0x00, 0xab, 0x10, 0xff};
    EXPECT_EQ(hex_dump(d, 4), "00ab10ff");
    EXPECT_EQ(hex_dump(d, 4, 2), "00ab...");
    EXPECT_EQ(hex_dump(d, 0), "");
}

TEST(BaseDepth, url_codec_round_trips_every_byte) {
    std::string all;
    for (int c = 0; c < 256; ++c) all.push_back((char)c);
    EXPECT_EQ(url_decode(url_encode(all)), all);
    EXPECT_EQ(url_encode("a b/c~"), "a%20b%2Fc~");
    EXPECT_EQ(url_decode("a+b%2f%2F"), "a b//");
    // malformed escapes pass through unchanged
    EXPECT_EQ(url_decode("%zz%4"), "%zz%4");
}

TEST(BaseDepth, html_escape_covers_the_specials) {
    EXPECT_EQ(html_escape("<a href=\"x\">&'</a>"), html_escape("<a href=\"x\">&'</a>"));
    const std::string e = html_escape("<&>\"");
    EXPECT_EQ(e.find('<'), std::string::npos);
    EXPECT_EQ(e.find('>'), std::string::npos);
    EXPECT_NE(e.find("&amp;"), std::string::npos);
    EXPECT_EQ(html_escape("plain"), "plain");
}

TEST(BaseDepth, string_printf_grows_past_any_stack_buffer) {
    const std::string big(5000, 'q');
    const std::string s = string_printf("<%s|%d>", big.c_str(), 42);
    EXPECT_EQ(s.size(), big.size() + 5);
    EXPECT_TRUE(ends_with(s, "|42>"));
    std::string acc = "x";
    string_appendf(&acc, "%03d", 7);
    string_appendf(&acc, "%s", big.c_str());
    EXPECT_EQ(acc.size(), 4 + big.size());
    EXPECT_TRUE(starts_with(acc, "x007q"));
}

// ------------------------------------------------------------------ hashes
TEST(BaseDepth, murmurhash3_32_known_answers) {
    EXPECT_EQ(murmurhash3_32("", 0, 0), 0u);
    EXPECT_EQ(murmurhash3_32("", 0, 1), 0x514e28b7u);
    EXPECT_EQ(murmurhash3_32("", 0, 0xffffffffu), 0x81f16f39u);
    EXPECT_EQ(murmurhash3_32("\0\0\0\0", 4, 0), 0x2362f9deu);
    EXPECT_EQ(murmurhash3_32("aaaa", 4, 0x9747b28cu), 0x5a97808au);
    EXPECT_EQ(murmurhash3_32("abc", 3, 0), 0xb3dd93fau);
    EXPECT_EQ(murmurhash3_32("Hello, world!", 13, 0x9747b28cu), 0x24884cbau);
    const char* fox = "The quick brown fox jumps over the lazy dog";
    EXPECT_EQ(murmurhash3_32(fox, strlen(fox), 0x9747b28cu), 0x2fa826cdu);
}

TEST(BaseDepth, murmurhash3_x64_128_known_answers) {
    uint64_t h[2];
    murmurhash3_x64_128("", 0, 0, h);
    EXPECT_EQ(h[0], 0u);
    EXPECT_EQ(h[1], 0u);
    murmurhash3_x64_128("hello", 5, 0, h);
    EXPECT_EQ(h[0], 0xcbd8a7b341bd9b02ull);
    EXPECT_EQ(h[1], 0x5b1e906a48ae1d19ull);
    const char* fox = "The quick brown fox jumps over the lazy dog";
    murmurhash3_x64_128(fox, strlen(fox), 0, h);
    EXPECT_EQ(h[0], 0xe34bbc7bbc071b6cull);
    EXPECT_EQ(h[1], 0x7a433ca9c49a9347ull);
    murmurhash3_x64_128("0123456789abcdefXYZ", 19, 42, h);  // a 16-byte block plus a tail
    EXPECT_EQ(h[0], 0x3fa90146b0ef7bc6ull);
    EXPECT_EQ(h[1], 0x71a710817d54ea00ull);
}

TEST(BaseDepth, md5_rfc1321_vectors) {
    struct V {
        std::string in;
        const char* hex;
    } vs[] = {
        {"", "d41d8cd98f00b204e9800998ecf8427e"},
        {"a", "0cc175b9c0f1b6a831c399e269772661"},
        {"abc", "900150983cd24fb0d6963f7d28e17f72"},
        {"message digest", "f96b697d7cb7938d525a2f31aaf161d0"},
        {"abcdefghijklmnopqrstuvwxyz", "c3fcd3d76192e4007dfb496cca67e13b"},
        {std::string(8 * 10, '0'), nullptr},
    };
    std::string digits;
    for (int i = 0; i < 8; ++i) digits += "1234567890";
    vs[5] = {digits, "57edf4a22be3c955ac49da2e2107b67a"};
    for (const V& v : vs) {
        unsigned char d[16];
        md5(v.in.data(), v.in.size(), d);
        EXPECT_EQ(hex_of(d, 16), std::string(v.hex));
    }
    EXPECT_EQ(md5_hash32("abc", 3), 0x98500190u);  // the digest's first four bytes, little endian
}

TEST(BaseDepth, sha1_fips180_vectors) {
    EXPECT_EQ(sha1_hex("", 0), "da39a3ee5e6b4b0d3255bfef95601890afd80709");
    EXPECT_EQ(sha1_hex("abc", 3), "a9993e364706816aba3e25717850c26c9cd0d89d");
    const char* m = "abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq";
    EXPECT_EQ(sha1_hex(m, strlen(m)), "84983e441c3bd26ebaae4aa1f95129e5e54670f1");
}

// ------------------------------------------------------------------ base64
TEST(BaseDepth, base64_rfc4648_vectors) {
    const char* in[] = {"", "f", "fo", "foo", "foob", "fooba", "foobar"};
    const char* out[] = {"", "Zg==", "Zm8=", "Zm9v", "Zm9vYg==", "Zm9vYmE=", "Zm9vYmFy"};
    for (int i = 0; i < 7; ++i) {
        EXPECT_EQ(base64_encode(in[i], strlen(in[i])), std::string(out[i]));
        std::string back;
        EXPECT_TRUE(base64_decode(out[i], &back));
        EXPECT_EQ(back, std::string(in[i]));
    }
}

TEST(BaseDepth, base64_decode_refuses_malformed_input) {
    std::string out;
    EXPECT_FALSE(base64_decode("Zm9v!", &out));     // bad symbol
    EXPECT_FALSE(base64_decode("Zg==Zg==", &out));  // data after padding
    EXPECT_FALSE(base64_decode("Z", &out));         // a lone symbol carries no byte
    EXPECT_FALSE(base64_decode("Zm9=v", &out));
    EXPECT_FALSE(base64_decode("Zg===", &out));     // too much padding
    EXPECT_TRUE(base64_decode("Zm9vYg", &out));     // unpadded is accepted
    EXPECT_EQ(out, "foob");
    EXPECT_TRUE(base64_decode("Zm9v\r\nYmFy", &out));  // line breaks are skipped
    EXPECT_EQ(out, "foobar");
}

TEST(BaseDepth, base64_round_trips_binary_of_every_length) {
    std::string s;
    for (int n = 0; n < 70; ++n) {
        std::string back;
        EXPECT_TRUE(base64_decode(base64_encode(s.data(), s.size()), &back));
        EXPECT_EQ(back, s);
        s.push_back((char)(n * 37 + 11));
    }
}

// ------------------------------------------------------------------ packing
TEST(BaseDepth, big_and_little_endian_packing) {
    unsigned char b[8];
    pack_be16(b, 0x1234);
    EXPECT_EQ((int)b[0], 0x12);
    EXPECT_EQ(unpack_be16(b), 0x1234);
    pack_be32(b, 0xdeadbeefu);
    EXPECT_EQ((int)b[0], 0xde);
    EXPECT_EQ((int)b[3], 0xef);
    EXPECT_EQ(unpack_be32(b), 0xdeadbeefu);
    pack_be64(b, 0x0102030405060708ull);
    EXPECT_EQ((int)b[0], 1);
    EXPECT_EQ((int)b[7], 8);
    EXPECT_EQ(unpack_be64(b), 0x0102030405060708ull);
    pack_le32(b, 0x11223344u);
    EXPECT_EQ((int)b[0], 0x44);
    EXPECT_EQ(unpack_le32(b), 0x11223344u);
}

// ------------------------------------------------------------------ status
TEST(BaseDepth, status_and_error_text) {
    EXPECT_TRUE(Status::OK().ok());
    EXPECT_EQ(Status::OK().to_string(), "OK");
    Status s(42, "nope");
    EXPECT_FALSE(s.ok());
    EXPECT_EQ(s.error_code(), 42);
    EXPECT_EQ(s.to_string(), "[42] nope");
    RegisterErrorText(987654, "base depth error");
    EXPECT_EQ(std::string(ErrorText(987654)), "base depth error");
    EXPECT_TRUE(ErrorText(987655) != nullptr);  // unknown codes still get a text
}

// ------------------------------------------------------------------ time
TEST(BaseDepth, clocks_are_consistent) {
    int64_t prev = monotonic_ns();
    for (int i = 0; i < 1000; ++i) {
        const int64_t now = monotonic_ns();
        EXPECT_GE(now, prev);
        prev = now;
    }
    const int64_t us = monotonic_us(), ms = monotonic_ms();
    EXPECT_LE(ms, us / 1000 + 1);
    EXPECT_GE(realtime_ms(), 1600000000000LL);  // after 2020
    const timespec t = ns_to_timespec(3500000123LL);
    EXPECT_EQ((int64_t)t.tv_sec, 3);
    EXPECT_EQ((int64_t)t.tv_nsec, 500000123);
    const timespec due = realtime_after_us(2000000);
    EXPECT_GT((int64_t)due.tv_sec * 1000000 + due.tv_nsec / 1000, realtime_us() + 1000000);
}

TEST(BaseDepth, timer_measures_a_sleep) {
    Timer t;
    t.start();
    usleep(20000);
    t.stop();
    EXPECT_GE(t.u_elapsed(), 19000);
    EXPECT_LT(t.m_elapsed(), 2000 * mtest::kSlowdown);
    EXPECT_NEAR(t.s_elapsed(), t.n_elapsed() / 1e9, 1e-9);
}

// ------------------------------------------------------------------ flags
TEST(BaseDepth, flags_parse_typed_values_and_refuse_bad_ones) {
    std::string err;
    EXPECT_TRUE(SetFlag("bd_i32", "0x10", false, &err));
    EXPECT_EQ(FLAGS_bd_i32, 16);
    EXPECT_FALSE(SetFlag("bd_i32", "4294967296", false, &err));  // out of int32
    EXPECT_FALSE(SetFlag("bd_i32", "12abc", false, &err));
    EXPECT_EQ(FLAGS_bd_i32, 16);
    EXPECT_TRUE(SetFlag("bd_i64", "-9223372036854775808"));
    EXPECT_EQ(FLAGS_bd_i64, INT64_MIN);
    EXPECT_FALSE(SetFlag("bd_u64", "-1"));
    EXPECT_TRUE(SetFlag("bd_u64", "18446744073709551615"));
    EXPECT_EQ(FLAGS_bd_u64, UINT64_MAX);
    for (const char* t : {"true", "1", "yes", "on"}) {
        EXPECT_TRUE(SetFlag("bd_bool", "false"));
        EXPECT_TRUE(SetFlag("bd_bool", t));
        EXPECT_TRUE(FLAGS_bd_bool);
    }
    EXPECT_FALSE(SetFlag("bd_bool", "maybe"));
    EXPECT_TRUE(SetFlag("bd_double", "2.25e1"));
    EXPECT_EQ(FLAGS_bd_double, 22.5);
    EXPECT_FALSE(SetFlag("bd_double", "abc"));
    EXPECT_TRUE(SetFlag("bd_str", "hello world"));
    EXPECT_EQ(FLAGS_bd_str, "hello world");
    EXPECT_FALSE(SetFlag("bd_no_such_flag", "1"));
    std::string v;
    EXPECT_TRUE(GetFlag("bd_i32", &v));
    EXPECT_EQ(v, "16");
    SetFlag("bd_i32", "5");
}

TEST(BaseDepth, flag_info_default_reloadable_and_validator) {
    FlagInfo info;
    ASSERT_TRUE(GetFlagInfo("bd_positive", &info));
    EXPECT_EQ(info.default_value, "3");
    EXPECT_FALSE(info.reloadable);
    std::string err;
    EXPECT_FALSE(SetFlag("bd_positive", "4", /*require_reloadable=*/true, &err));  // not reloadable yet
    ASSERT_TRUE(RegisterFlagValidator("bd_positive", PositiveIntegerValidator));
    ASSERT_TRUE(GetFlagInfo("bd_positive", &info));
    EXPECT_TRUE(info.reloadable);
    EXPECT_TRUE(SetFlag("bd_positive", "4", true, &err));
    EXPECT_FALSE(SetFlag("bd_positive", "0", true, &err));  // the validator refuses
    EXPECT_FALSE(SetFlag("bd_positive", "-3", true, &err));
    EXPECT_EQ(FLAGS_bd_positive, 4);
    ASSERT_TRUE(GetFlagInfo("bd_positive", &info));
    EXPECT_EQ(info.current_value, "4");
    bool listed = false;
    for (const FlagInfo& f : ListFlags()) listed |= f.name == "bd_positive";
    EXPECT_TRUE(listed);
}

TEST(BaseDepth, command_line_forms_and_unknown_arguments) {
    std::vector<std::string> args = {"prog", "--bd_i32=7", "-bd_str=two words", "--bd_i64", "-99",
                                     "--nobd_bool", "--unknown_thing=1", "positional"};
    std::vector<char*> argv;
    for (std::string& a : args) argv.push_back(&a[0]);
    int argc = (int)argv.size();
    char** av = argv.data();
    SetFlag("bd_bool", "true");
    const int n = ParseCommandLineFlags(&argc, &av, true);
    EXPECT_EQ(n, 4);
    EXPECT_EQ(FLAGS_bd_i32, 7);
    EXPECT_EQ(FLAGS_bd_str, "two words");
    EXPECT_EQ(FLAGS_bd_i64, -99);
    EXPECT_FALSE(FLAGS_bd_bool);
    ASSERT_EQ(argc, 3);  // the program name and what was not a flag stay
    EXPECT_EQ(std::string(av[1]), "--unknown_thing=1");
    EXPECT_EQ(std::string(av[2]), "positional");
    SetFlag("bd_i32", "5");
}

TEST(BaseDepth, flags_from_a_file) {
    char path[] = "/tmp/bd_flagsXXXXXX";
    const int fd = mkstemp(path);
    ASSERT_TRUE(fd >= 0);
    SetFlag("bd_bool", "false");
    const std::string body =
        "# comment\nbd_i32 = 11 \n\nbd_str = spaced \nbd_double=0.5\n\tbd_bool\t=\ttrue\t\nbd_i64 =  -8\n";
    ASSERT_EQ((size_t)write(fd, body.data(), body.size()), body.size());
    close(fd);
    const int n = LoadFlagsFromFile(path);
    unlink(path);
    EXPECT_EQ(n, 5);  // every line applied, blanks around '=' and at the end included
    EXPECT_EQ(FLAGS_bd_i32, 11);
    EXPECT_EQ(FLAGS_bd_double, 0.5);
    EXPECT_EQ(FLAGS_bd_str, "spaced");
    EXPECT_TRUE(FLAGS_bd_bool);
    EXPECT_EQ(FLAGS_bd_i64, -8);
    SetFlag("bd_i32", "5");
}

// ------------------------------------------------------------------ pools
namespace {
struct PoolItem {
    int v = 0;
    char pad[40];
};
}  // namespace

TEST(BaseDepth, resource_pool_recycles_ids_and_keeps_addresses) {
    std::vector<uint32_t> ids;
    std::set<PoolItem*> addrs;
    for (int i = 0; i < 1000; ++i) {
        uint32_t id;
        PoolItem* p = get_resource<PoolItem>(&id);
        ASSERT_TRUE(p != nullptr);
        EXPECT_TRUE(address_resource<PoolItem>(id) == p);
        p->v = (int)id;
        ids.push_back(id);
        addrs.insert(p);
    }
    EXPECT_EQ(addrs.size(), 1000u);
    EXPECT_EQ(std::set<uint32_t>(ids.begin(), ids.end()).size(), 1000u);
    for (uint32_t id : ids) return_resource<PoolItem>(id);
    // a freed id comes back (LIFO per thread) at the same address
    uint32_t again;
    PoolItem* p = get_resource<PoolItem>(&again);
    EXPECT_TRUE(std::find(ids.begin(), ids.end(), again) != ids.end());
    EXPECT_TRUE(address_resource<PoolItem>(again) == p);
    return_resource<PoolItem>(again);
    EXPECT_TRUE(address_resource<PoolItem>(0xFFFFFF00u) == nullptr);  // never allocated
}

TEST(BaseDepth, resource_pool_ids_are_unique_across_threads) {
    std::vector<std::vector<uint32_t>> got(4);
    std::vector<std::thread> th;
    for (int t = 0; t < 4; ++t) {
        th.emplace_back([&got, t] {
            for (int i = 0; i < 2000; ++i) {
                uint32_t id;
                get_resource<PoolItem>(&id);
                got[t].push_back(id);
            }
        });
    }
    for (auto& x : th) x.join();
    std::set<uint32_t> all;
    for (auto& v : got) all.insert(v.begin(), v.end());
    EXPECT_EQ(all.size(), 8000u);
    for (auto& v : got)
        for (uint32_t id : v) return_resource<PoolItem>(id);
}

TEST(BaseDepth, object_pool_reuses_returned_objects) {
    PoolItem* a = get_object<PoolItem>();
    a->v = 77;
    return_object(a);
    PoolItem* b = get_object<PoolItem>();
    EXPECT_TRUE(a == b);  // the thread's cache hands it back
    EXPECT_EQ(b->v, 77);  // objects are not reset: callers do it
    return_object(b);
}

// ------------------------------------------------------------------ containers
TEST(BaseDepth, flat_map_with_string_keys_and_custom_hash) {
    FlatMap<std::string, int, CaseIgnoredHash, CaseIgnoredEqual> m;
    m["Accept"] = 1;
    m.insert("HOST", 2);
    EXPECT_TRUE(m.contains("accept"));
    EXPECT_TRUE(m.seek("host") != nullptr);
    EXPECT_EQ(*m.seek("Host"), 2);
    EXPECT_EQ(m.erase("ACCEPT"), 1u);
    EXPECT_EQ(m.erase("ACCEPT"), 0u);
    EXPECT_EQ(m.size(), 1u);
    EXPECT_TRUE(m.seek("missing") == nullptr);
}

TEST(BaseDepth, flat_map_survives_heavy_churn) {
    FlatMap<uint64_t, uint64_t> m;
    std::map<uint64_t, uint64_t> ref;
    uint64_t x = 88172645463325252ull;
    for (int i = 0; i < 20000; ++i) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        const uint64_t k = x % 3000;
        if (x & 1) {
            m[k] = x;
            ref[k] = x;
        } else {
            EXPECT_EQ(m.erase(k), ref.erase(k));
        }
    }
    EXPECT_EQ(m.size(), ref.size());
    for (auto& kv : ref) {
        const uint64_t* v = m.seek(kv.first);
        ASSERT_TRUE(v != nullptr);
        EXPECT_EQ(*v, kv.second);
    }
    size_t n = 0;
    m.for_each([&n](const uint64_t&, const uint64_t&) { ++n; });
    EXPECT_EQ(n, ref.size());
    m.clear();
    EXPECT_TRUE(m.empty());
}

TEST(BaseDepth, bounded_queue_refuses_past_capacity) {
    BoundedQueue<int> q(3);
    EXPECT_TRUE(q.empty());
    EXPECT_EQ(q.capacity(), 3u);
    EXPECT_TRUE(q.push(1));
    EXPECT_TRUE(q.push(2));
    EXPECT_TRUE(q.push(3));
    EXPECT_TRUE(q.full());
    EXPECT_FALSE(q.push(4));
    int v = 0;
    EXPECT_TRUE(q.pop(&v));
    EXPECT_EQ(v, 1);
    EXPECT_TRUE(q.push(4));
    for (int want : {2, 3, 4}) {
        EXPECT_TRUE(q.pop(&v));
        EXPECT_EQ(v, want);
    }
    EXPECT_FALSE(q.pop(&v));
}

TEST(BaseDepth, mru_cache_capacity_one_and_peek) {
    MRUCache<int, std::string> c(1);
    EXPECT_FALSE(c.Put(1, "a"));
    int evicted = 0;
    EXPECT_TRUE(c.Put(2, "b", &evicted));
    EXPECT_EQ(evicted, 1);
    EXPECT_TRUE(c.Get(1) == nullptr);
    EXPECT_EQ(*c.Peek(2), "b");
    EXPECT_FALSE(c.Put(2, "c"));  // overwrite, no eviction
    EXPECT_EQ(*c.Get(2), "c");
    EXPECT_TRUE(c.Erase(2));
    EXPECT_EQ(c.size(), 0u);
    MRUCache<int, int> z(0);  // capacity 0 is clamped to 1
    EXPECT_EQ(z.capacity(), 1u);
}

TEST(BaseDepth, mru_cache_iterates_most_recent_first) {
    MRUCache<int, int> c(3);
    c.Put(1, 10);
    c.Put(2, 20);
    c.Put(3, 30);
    c.Get(1);
    std::vector<int> order;
    c.for_each([&order](const int& k, const int&) { order.push_back(k); });
    ASSERT_EQ(order.size(), 3u);
    EXPECT_EQ(order[0], 1);
    EXPECT_EQ(order[1], 3);
    EXPECT_EQ(order[2], 2);
}

TEST(BaseDepth, link_nodes_form_a_ring) {
    LinkNode head, a, b;
    EXPECT_TRUE(head.empty());
    a.insert_before(&head);
    b.insert_before(&head);
    EXPECT_TRUE(head.next == &a);
    EXPECT_TRUE(a.next == &b);
    EXPECT_TRUE(b.next == &head);
    EXPECT_TRUE(head.prev == &b);
    a.remove();
    EXPECT_TRUE(a.empty());
    EXPECT_TRUE(head.next == &b);
    b.remove();
    EXPECT_TRUE(head.empty());
}

// ------------------------------------------------------------------ endpoints
TEST(BaseDepth, endpoint_forms_parse_and_print) {
    EndPoint ep;
    ASSERT_EQ(str2endpoint("10.1.2.3:8080", &ep), 0);
    EXPECT_EQ(ep.port, 8080);
    EXPECT_EQ(ep.to_string(), "10.1.2.3:8080");
    EXPECT_EQ(ip2str(ep.ip), "10.1.2.3");
    ASSERT_EQ(str2endpoint("[::1]:53", &ep), 0);
    EXPECT_TRUE(ep.is_ipv6());
    EXPECT_EQ(ep.port, 53);
    ASSERT_EQ(str2endpoint("unix:/tmp/bd.sock", &ep), 0);
    EXPECT_TRUE(ep.is_unix());
    EXPECT_EQ(ep.path, "/tmp/bd.sock");
    EXPECT_NE(str2endpoint("10.1.2.3:70000", &ep), 0);
    EXPECT_NE(str2endpoint("10.1.2.3", &ep), 0);
    EXPECT_NE(str2endpoint("300.1.2.3:80", &ep), 0);
    EXPECT_NE(str2endpoint("", &ep), 0);
    ASSERT_EQ(str2endpoint("127.0.0.1", 99, &ep), 0);
    EXPECT_EQ(ep.to_string(), "127.0.0.1:99");
    uint32_t ip = 0;
    EXPECT_EQ(str2ip("192.168.0.1", &ip), 0);
    EXPECT_EQ(ip2str(ip), "192.168.0.1");
    EXPECT_NE(str2ip("192.168.0", &ip), 0);
}

TEST(BaseDepth, endpoint_order_equality_and_hash) {
    EndPoint a, b, c;
    str2endpoint("1.1.1.1:80", &a);
    str2endpoint("1.1.1.1:81", &b);
    str2endpoint("[::1]:80", &c);
    EXPECT_TRUE(a < b);
    EXPECT_FALSE(b < a);
    EXPECT_TRUE(a < c);  // IPv4 before IPv6
    EXPECT_TRUE(a != b);
    EndPoint a2;
    str2endpoint("1.1.1.1:80", &a2);
    EXPECT_TRUE(a == a2);
    EXPECT_EQ(EndPointHash()(a), EndPointHash()(a2));
}

TEST(BaseDepth, hostname_resolution_of_localhost) {
    EndPoint ep;
    ASSERT_EQ(hostname2endpoint("localhost:1234", &ep), 0);
    EXPECT_EQ(ep.port, 1234);
    EXPECT_NE(hostname2endpoint("no-such-host.invalid:1", &ep), 0);
}

TEST(BaseDepth, loopback_listen_connect_and_sides) {
    EndPoint any;
    str2endpoint("127.0.0.1:0", &any);
    const int lfd = tcp_listen(any);
    ASSERT_TRUE(lfd >= 0);
    EndPoint bound;
    ASSERT_EQ(get_local_side(lfd, &bound), 0);
    EXPECT_GT(bound.port, 0);
    const int cfd = tcp_connect(bound, 2000);
    ASSERT_TRUE(cfd >= 0);
    const int afd = accept(lfd, nullptr, nullptr);
    ASSERT_TRUE(afd >= 0);
    EndPoint peer, local;
    EXPECT_EQ(get_remote_side(cfd, &peer), 0);
    EXPECT_EQ(peer, bound);
    EXPECT_EQ(get_local_side(afd, &local), 0);
    EXPECT_EQ(local, bound);
    EXPECT_EQ(make_non_blocking(cfd), 0);
    EXPECT_TRUE(fcntl(cfd, F_GETFL) & O_NONBLOCK);
    EXPECT_EQ(make_blocking(cfd), 0);
    EXPECT_FALSE(fcntl(cfd, F_GETFL) & O_NONBLOCK);
    EXPECT_EQ(make_close_on_exec(cfd), 0);
    EXPECT_TRUE(fcntl(cfd, F_GETFD) & FD_CLOEXEC);
    EXPECT_EQ(make_no_delay(cfd), 0);
    close(afd);
    close(cfd);
    close(lfd);
    // nothing listens there any more
    EXPECT_LT(tcp_connect(bound, 500), 0);
}

// ------------------------------------------------------------------ crc32c
TEST(BaseDepth, crc32c_unaligned_and_split_inputs_agree) {
    std::string buf(4096 + 64, '\0');
    for (size_t i = 0; i < buf.size(); ++i) buf[i] = (char)(i * 131 + 7);
    for (size_t off = 0; off < 16; ++off) {
        const uint32_t whole = crc32c::Value(buf.data() + off, 4096);
        uint32_t part = 0;
        for (size_t at = 0; at < 4096; at += 13 + off) {
            const size_t n = std::min<size_t>(13 + off, 4096 - at);
            part = crc32c::Extend(part, buf.data() + off + at, n);
        }
        EXPECT_EQ(part, whole);
        const uint32_t a = crc32c::Value(buf.data() + off, 1000);
        const uint32_t b = crc32c::Value(buf.data() + off + 1000, 3096);
        EXPECT_EQ(crc32c::Combine(a, b, 3096), whole);
    }
    EXPECT_EQ(crc32c::Value("", 0), 0u);
    EXPECT_EQ(crc32c::Value("123456789", 9), 0xe3069283u);  // the CRC-32C check value
    const uint32_t c = crc32c::Value("abc", 3);
    EXPECT_EQ(crc32c::Combine(c, 0, 0), c);
}

// ------------------------------------------------------------------ snappy
TEST(BaseDepth, snappy_edge_inputs) {
    std::string out, back;
    ASSERT_TRUE(snappy::Compress("", 0, &out));
    size_t len = 99;
    EXPECT_TRUE(snappy::GetUncompressedLength(out.data(), out.size(), &len));
    EXPECT_EQ(len, 0u);
    EXPECT_TRUE(snappy::Uncompress(out.data(), out.size(), &back));
    EXPECT_EQ(back, "");
    for (size_t n : {1u, 2u, 3u, 4u, 15u, 16u, 17u, 59u, 60u, 61u, 65535u, 65536u, 65537u, 300000u}) {
        std::string in(n, 'a');
        for (size_t i = 0; i < n; i += 7) in[i] = (char)('a' + i % 26);
        ASSERT_TRUE(snappy::Compress(in.data(), in.size(), &out));
        EXPECT_LE(out.size(), snappy::MaxCompressedLength(n));
        EXPECT_TRUE(snappy::IsValidCompressedBuffer(out.data(), out.size()));
        ASSERT_TRUE(snappy::Uncompress(out.data(), out.size(), &back));
        EXPECT_EQ(back, in);
        // any truncation is refused
        if (out.size() > 2) {
            EXPECT_FALSE(snappy::Uncompress(out.data(), out.size() - 1, &back));
        }
    }
}

TEST(BaseDepth, snappy_refuses_random_garbage) {
    uint64_t x = 0x9e3779b97f4a7c15ull;
    int refused = 0;
    for (int t = 0; t < 300; ++t) {
        std::string g(1 + t % 97, '\0');
        for (char& ch : g) {
            x ^= x << 13;
            x ^= x >> 7;
            x ^= x << 17;
            ch = (char)x;
        }
        std::string back;
        const bool valid = snappy::IsValidCompressedBuffer(g.data(), g.size());
        const bool ok = snappy::Uncompress(g.data(), g.size(), &back);
        EXPECT_EQ(valid, ok);  // the validator and the decoder agree
        refused += !ok;
        if (ok) {
            size_t len = 0;
            EXPECT_TRUE(snappy::GetUncompressedLength(g.data(), g.size(), &len));
            EXPECT_EQ(len, back.size());
        }
    }
    EXPECT_GT(refused, 250);
}
