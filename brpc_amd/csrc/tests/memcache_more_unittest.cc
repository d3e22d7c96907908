// More memcache binary-protocol cases (redis/memcache.h), after the
// reference's test/brpc_memcache_unittest.cpp and the protocol's wire
// layout: the opcodes and extras of every request kind, the 250-byte key
// limit for each keyed op, Clear(), GET results with flags and cas, counter
// values, error statuses with their text, result counting across partial
// reads, malformed bodies, and popping past the end.
#include <string>

#include "redis/memcache.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

std::string be(uint64_t v, int n) {
    std::string s;
    for (int i = n - 1; i >= 0; --i) s.push_back((char)(v >> (8 * i)));
    return s;
}

std::string hdr(uint8_t magic, uint8_t op, uint16_t keylen, uint8_t extlen, uint16_t status, uint32_t body,
                uint64_t cas) {
    return std::string(1, (char)magic) + std::string(1, (char)op) + be(keylen, 2) + std::string(1, (char)extlen) +
           std::string(1, '\0') + be(status, 2) + be(body, 4) + be(0, 4) + be(cas, 8);
}

std::string resp(uint8_t op, uint16_t status, const std::string& ext, const std::string& key, const std::string& val,
                 uint64_t cas = 0) {
    return hdr(0x81, op, (uint16_t)key.size(), (uint8_t)ext.size(), status,
               (uint32_t)(ext.size() + key.size() + val.size()), cas) +
           ext + key + val;
}

int consume_all(MemcacheResponse* r, const std::string& wire, int count) {
    Buf in;
    in.append(wire);
    return r->ConsumePartial(&in, count);
}

}  // namespace

TEST(MemcacheMore, get_delete_and_version_wire) {
    MemcacheRequest req;
    ASSERT_TRUE(req.Get("key"));
    ASSERT_TRUE(req.Delete("gone"));
    ASSERT_TRUE(req.Version());
    std::string want = hdr(0x80, 0x00, 3, 0, 0, 3, 0) + "key";
    want += hdr(0x80, 0x04, 4, 0, 0, 4, 0) + "gone";
    want += hdr(0x80, 0x0b, 0, 0, 0, 0, 0);
    EXPECT_TRUE(req.raw().to_string() == want);
    EXPECT_EQ(req.op_count(), 3);
}

TEST(MemcacheMore, storage_ops_carry_extras_only_where_the_protocol_has_them) {
    MemcacheRequest req;
    ASSERT_TRUE(req.Add("a", "1", 5, 6, 0));
    ASSERT_TRUE(req.Replace("b", "22", 7, 8, 9));
    ASSERT_TRUE(req.Append("c", "333", 1, 1, 0));   // no extras: flags/exptime not sent
    ASSERT_TRUE(req.Prepend("d", "4444", 1, 1, 3));
    std::string want = hdr(0x80, 0x02, 1, 8, 0, 8 + 1 + 1, 0) + be(5, 4) + be(6, 4) + "a1";
    want += hdr(0x80, 0x03, 1, 8, 0, 8 + 1 + 2, 9) + be(7, 4) + be(8, 4) + "b22";
    want += hdr(0x80, 0x0e, 1, 0, 0, 1 + 3, 0) + "c333";
    want += hdr(0x80, 0x0f, 1, 0, 0, 1 + 4, 3) + "d4444";
    EXPECT_TRUE(req.raw().to_string() == want);
    EXPECT_EQ(req.op_count(), 4);
}

TEST(MemcacheMore, increment_wire_and_key_limits) {
    MemcacheRequest req;
    ASSERT_TRUE(req.Increment(std::string(250, 'k'), 1, 2, 3));
    const std::string w = req.raw().to_string();
    EXPECT_EQ(w.size(), 24u + 20 + 250);
    EXPECT_TRUE(w.substr(0, 24) == hdr(0x80, 0x05, 250, 20, 0, 270, 0));
    EXPECT_TRUE(w.substr(24, 20) == be(1, 8) + be(2, 8) + be(3, 4));
    const std::string too_long(251, 'k');
    EXPECT_FALSE(req.Get(too_long));
    EXPECT_FALSE(req.Set(too_long, "v", 0, 0, 0));
    EXPECT_FALSE(req.Add(too_long, "v", 0, 0, 0));
    EXPECT_FALSE(req.Replace(too_long, "v", 0, 0, 0));
    EXPECT_FALSE(req.Append(too_long, "v", 0, 0, 0));
    EXPECT_FALSE(req.Prepend(too_long, "v", 0, 0, 0));
    EXPECT_FALSE(req.Delete(too_long));
    EXPECT_FALSE(req.Increment(too_long, 1, 1, 0));
    EXPECT_FALSE(req.Decrement(too_long, 1, 1, 0));
    EXPECT_FALSE(req.Touch(too_long, 1));
    EXPECT_EQ(req.op_count(), 1);
}

TEST(MemcacheMore, clear_empties_the_request) {
    MemcacheRequest req;
    req.Get("x");
    req.Flush(10);
    EXPECT_EQ(req.op_count(), 2);
    req.Clear();
    EXPECT_EQ(req.op_count(), 0);
    EXPECT_TRUE(req.raw().empty());
    req.Version();
    EXPECT_EQ(req.raw().size(), 24u);
}

TEST(MemcacheMore, get_result_with_flags_and_cas) {
    MemcacheResponse r;
    ASSERT_EQ(consume_all(&r, resp(0x00, 0, be(0xabcd, 4), "", "payload", 77), 1), 1);
    std::string v;
    uint32_t flags = 0;
    uint64_t cas = 0;
    ASSERT_TRUE(r.PopGet(&v, &flags, &cas));
    EXPECT_EQ(v, "payload");
    EXPECT_EQ(flags, 0xabcdu);
    EXPECT_EQ(cas, 77u);
    MemcacheResponse r2;
    ASSERT_EQ(consume_all(&r2, resp(0x00, 0, be(1, 4), "", "v"), 1), 1);
    EXPECT_TRUE(r2.PopGet(nullptr, nullptr, nullptr));  // every output is optional
}

TEST(MemcacheMore, counter_results_are_big_endian_u64) {
    MemcacheResponse r;
    std::string wire = resp(0x05, 0, "", "", be(0x0102030405060708ull, 8), 5);
    wire += resp(0x06, 0, "", "", be(0, 8), 6);
    ASSERT_EQ(consume_all(&r, wire, 2), 1);
    uint64_t v = 0, cas = 0;
    ASSERT_TRUE(r.PopIncrement(&v, &cas));
    EXPECT_EQ(v, 0x0102030405060708ull);
    EXPECT_EQ(cas, 5u);
    ASSERT_TRUE(r.PopDecrement(&v, nullptr));
    EXPECT_EQ(v, 0u);
}

TEST(MemcacheMore, error_status_carries_the_server_text) {
    MemcacheResponse r;
    std::string wire = resp(0x04, MC_STATUS_KEY_ENOENT, "", "", "Not found");
    wire += resp(0x05, MC_STATUS_DELTA_BADVAL, "", "", "Non-numeric server-side value for incr or decr");
    wire += resp(0x1c, 0, "", "", "");
    ASSERT_EQ(consume_all(&r, wire, 3), 1);
    EXPECT_FALSE(r.PopDelete());
    EXPECT_TRUE(r.LastError().find("Not found") != std::string::npos);
    EXPECT_FALSE(r.PopIncrement(nullptr, nullptr));
    EXPECT_TRUE(r.LastError().find("Non-numeric") != std::string::npos);
    EXPECT_TRUE(r.PopTouch());
}

TEST(MemcacheMore, results_are_counted_across_partial_reads) {
    MemcacheResponse r;
    const std::string a = resp(0x01, 0, "", "", "", 1), b = resp(0x08, 0, "", "", "");
    Buf in;
    in.append(a);
    in.append(b.substr(0, 10));
    EXPECT_EQ(r.ConsumePartial(&in, 2), 0);
    EXPECT_EQ(r.result_count(), 1);
    EXPECT_EQ(in.size(), 10u);  // the incomplete header stays
    in.append(b.substr(10));
    EXPECT_EQ(r.ConsumePartial(&in, 2), 1);
    EXPECT_EQ(r.result_count(), 2);
    EXPECT_TRUE(in.empty());
    uint64_t cas = 0;
    EXPECT_TRUE(r.PopSet(&cas));
    EXPECT_TRUE(r.PopFlush());
    EXPECT_EQ(r.result_count(), 0);
}

TEST(MemcacheMore, body_shorter_than_key_and_extras_is_malformed) {
    MemcacheResponse r;
    std::string bad = hdr(0x81, 0x00, 5, 4, 0, 6, 0) + "123456";  // 5 + 4 > 6
    EXPECT_LT(consume_all(&r, bad, 1), 0);
}

TEST(MemcacheMore, popping_past_the_end_and_clear) {
    MemcacheResponse r;
    ASSERT_EQ(consume_all(&r, resp(0x0b, 0, "", "", "1.0"), 1), 1);
    std::string v;
    EXPECT_TRUE(r.PopVersion(&v));
    EXPECT_FALSE(r.PopVersion(&v));
    EXPECT_EQ(r.LastError(), std::string("no more results"));
    r.Clear();
    EXPECT_TRUE(r.LastError().empty());
    EXPECT_EQ(r.result_count(), 0);
    ASSERT_EQ(consume_all(&r, resp(0x02, 0, "", "", "", 3) + resp(0x03, 0, "", "", "", 4) +
                                  resp(0x0e, 0, "", "", "", 5) + resp(0x0f, 0, "", "", "", 6),
                          4),
              1);
    uint64_t c = 0;
    EXPECT_TRUE(r.PopAdd(&c));
    EXPECT_EQ(c, 3u);
    EXPECT_TRUE(r.PopReplace(&c));
    EXPECT_TRUE(r.PopAppend(&c));
    EXPECT_TRUE(r.PopPrepend(&c));
    EXPECT_EQ(c, 6u);
}
