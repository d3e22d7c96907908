// Protobuf codec depth: merge semantics, varint and zigzag boundaries,
// wire-type mismatches, last-one-wins, nesting limits, malformed input.
// Expected bytes are derived from the protobuf encoding rules (the
// reference's brpc_protobuf_json_unittest / brpc_proto_unittest exercise
// the same codec through google protobuf; here the codec is our own).
#include <cstring>
#include <memory>
#include <vector>
#include <string>

#include "mrpc/proto/echo.pb.h"
#include "pb/dynamic.h"
#include "pb/parser.h"
#include "pb/wire.h"
#include "tests/test.h"

using namespace mrpc;
using namespace mrpc::pb;

namespace {

const char* kProto = R"(
syntax = "proto2";
package d;
message Leaf { optional int32 v = 1; repeated int32 r = 2; optional string s = 3; }
message Node {
  optional int32 i32 = 1;
  optional int64 i64 = 2;
  optional uint32 u32 = 3;
  optional uint64 u64 = 4;
  optional sint32 s32 = 5;
  optional sint64 s64 = 6;
  optional fixed32 fx32 = 7;
  optional fixed64 fx64 = 8;
  optional bool b = 9;
  optional string str = 10;
  optional Leaf leaf = 11;
  repeated Leaf leaves = 12;
  repeated int32 ints = 13;
  oneof pick { string a = 14; Leaf l = 15; }
  optional Node child = 16;
  optional float f = 17;
  optional double dd = 18;
  repeated sint64 packed_s64 = 19 [packed = true];
}
)";

struct Env {
    Importer imp{{}};
    const Descriptor* node = nullptr;
    const Descriptor* leaf = nullptr;
    Env() {
        std::string err;
        if (imp.ImportFromString("d.proto", kProto, &err)) {
            node = imp.FindMessageTypeByName("d.Node");
            leaf = imp.FindMessageTypeByName("d.Leaf");
        }
    }
    const FieldDescriptor* f(const char* name) const { return node->FindFieldByName(name); }
    const FieldDescriptor* lf(const char* name) const { return leaf->FindFieldByName(name); }
};

std::string hex(const std::string& s) {
    static const char* d = "0123456789abcdef";
    std::string o;
    for (unsigned char c : s) {
        o += d[c >> 4];
        o += d[c & 15];
    }
    return o;
}

std::string wire_of(const Env& e, void (*fill)(const Env&, Message*)) {
    Message* m = e.node->prototype->New();
    fill(e, m);
    std::string w = m->SerializeAsString();
    delete m;
    return w;
}

}  // namespace

TEST(PbDepth, varint_and_zigzag_boundaries) {
    Env e;
    ASSERT_TRUE(e.node != nullptr);
    struct Case {
        const char* field;
        int64_t v;
        const char* want;  // hex of the whole message
    };
    // tag (field << 3 | wire) then the value
    const Case cases[] = {
        {"i32", -1, "08ffffffffffffffffff01"},       // negative int32: 10-byte varint
        {"i32", 2147483647, "08ffffffff07"},
        {"i64", INT64_MIN, "10808080808080808080" "01"},
        {"u32", 0xFFFFFFFFLL, "18ffffffff0f"},
        {"s32", -1, "2801"},                          // zigzag(-1) = 1
        {"s32", 2147483647, "28feffffff0f"},          // zigzag(max) = 0xfffffffe
        {"s32", -2147483647 - 1, "28ffffffff0f"},     // zigzag(min) = 0xffffffff
        {"s64", -64, "307f"},
        {"s64", 64, "308001"},
        {"fx32", 0xDEADBEEF, "3defbeadde"},
        {"b", 1, "4801"},
    };
    for (const Case& c : cases) {
        Message* m = e.node->prototype->New();
        const FieldDescriptor* fd = e.f(c.field);
        switch (fd->type) {
        case FieldType::INT32:
        case FieldType::SINT32: Reflection::SetInt32(m, fd, (int32_t)c.v); break;
        case FieldType::INT64:
        case FieldType::SINT64: Reflection::SetInt64(m, fd, c.v); break;
        case FieldType::UINT32:
        case FieldType::FIXED32: Reflection::SetUInt32(m, fd, (uint32_t)c.v); break;
        case FieldType::BOOL: Reflection::SetBool(m, fd, c.v != 0); break;
        default: break;
        }
        const std::string w = m->SerializeAsString();
        EXPECT_EQ(hex(w), std::string(c.want));
        EXPECT_EQ(m->ByteSizeLong(), w.size());
        Message* back = e.node->prototype->New();
        ASSERT_TRUE(back->ParseFromString(w));
        EXPECT_EQ(back->SerializeAsString(), w);
        delete m;
        delete back;
    }
    // u64 max and fixed64
    Message* m = e.node->prototype->New();
    Reflection::SetUInt64(m, e.f("u64"), ~0ull);
    Reflection::SetUInt64(m, e.f("fx64"), 0x0102030405060708ull);
    EXPECT_EQ(hex(m->SerializeAsString()), "20ffffffffffffffffff01" "410807060504030201");
    delete m;
}

TEST(PbDepth, merge_from_semantics) {
    Env e;
    Message* a = e.node->prototype->New();
    Message* b = e.node->prototype->New();
    Reflection::SetInt32(a, e.f("i32"), 1);
    Reflection::SetString(a, e.f("str"), "a");
    Reflection::AddInt32(a, e.f("ints"), 1);
    Message* la = Reflection::MutableMessage(a, e.f("leaf"));
    Reflection::SetInt32(la, e.lf("v"), 10);
    Reflection::AddInt32(la, e.lf("r"), 100);
    Reflection::SetString(a, e.f("a"), "oneof-a");
    // b overwrites scalars it has, appends repeated, merges the nested message
    Reflection::SetInt32(b, e.f("i32"), 2);
    Reflection::AddInt32(b, e.f("ints"), 2);
    Message* lb = Reflection::MutableMessage(b, e.f("leaf"));
    Reflection::SetString(lb, e.lf("s"), "from-b");
    Reflection::AddInt32(lb, e.lf("r"), 200);
    Message* ol = Reflection::MutableMessage(b, e.f("l"));  // the other oneof member
    Reflection::SetInt32(ol, e.lf("v"), 7);
    a->MergeFrom(*b);
    EXPECT_EQ(Reflection::GetInt32(*a, e.f("i32")), 2);
    EXPECT_EQ(Reflection::GetString(*a, e.f("str")), "a");  // untouched
    EXPECT_EQ(Reflection::FieldSize(*a, e.f("ints")), 2);
    const Message& leaf = Reflection::GetMessage(*a, e.f("leaf"));
    EXPECT_EQ(Reflection::GetInt32(leaf, e.lf("v")), 10);
    EXPECT_EQ(Reflection::GetString(leaf, e.lf("s")), "from-b");
    EXPECT_EQ(Reflection::FieldSize(leaf, e.lf("r")), 2);
    // the merged-in oneof member replaces the other
    EXPECT_FALSE(Reflection::HasField(*a, e.f("a")));
    EXPECT_TRUE(Reflection::HasField(*a, e.f("l")));
    // wire-level merge (concatenation) gives the same message
    Message* c = e.node->prototype->New();
    Message* a0 = e.node->prototype->New();
    Reflection::SetInt32(a0, e.f("i32"), 1);
    Reflection::SetString(a0, e.f("str"), "a");
    Reflection::AddInt32(a0, e.f("ints"), 1);
    Message* la0 = Reflection::MutableMessage(a0, e.f("leaf"));
    Reflection::SetInt32(la0, e.lf("v"), 10);
    Reflection::AddInt32(la0, e.lf("r"), 100);
    Reflection::SetString(a0, e.f("a"), "oneof-a");
    ASSERT_TRUE(c->ParseFromString(a0->SerializeAsString() + b->SerializeAsString()));
    EXPECT_EQ(c->SerializeAsString(), a->SerializeAsString());
    delete a;
    delete b;
    delete c;
    delete a0;
}

TEST(PbDepth, last_one_wins_and_repeated_occurrences) {
    Env e;
    // i32 twice on the wire: the last value wins; a nested message twice:
    // the occurrences merge
    std::string w;
    w += std::string("\x08\x05", 2);
    w += std::string("\x08\x07", 2);
    w += std::string("\x5a\x02\x08\x01", 4);  // leaf{v:1}
    w += std::string("\x5a\x02\x10\x02", 4);  // leaf{r:2}
    Message* m = e.node->prototype->New();
    ASSERT_TRUE(m->ParseFromString(w));
    EXPECT_EQ(Reflection::GetInt32(*m, e.f("i32")), 7);
    const Message& leaf = Reflection::GetMessage(*m, e.f("leaf"));
    EXPECT_EQ(Reflection::GetInt32(leaf, e.lf("v")), 1);
    EXPECT_EQ(Reflection::FieldSize(leaf, e.lf("r")), 1);
    // a packed run and single elements of the same repeated field append
    std::string p;
    p += std::string("\x68\x01", 2);          // ints: 1 (unpacked)
    p += std::string("\x6a\x03\x02\x03\x04", 5);  // ints: [2,3,4] (packed)
    p += std::string("\x68\x05", 2);          // ints: 5
    Message* r = e.node->prototype->New();
    ASSERT_TRUE(r->ParseFromString(p));
    ASSERT_EQ(Reflection::FieldSize(*r, e.f("ints")), 5);
    for (int i = 0; i < 5; ++i) EXPECT_EQ(Reflection::GetRepeatedInt32(*r, e.f("ints"), i), i + 1);
    delete m;
    delete r;
}

TEST(PbDepth, wire_type_mismatch_goes_to_unknown_fields) {
    Env e;
    // field 1 (i32, a varint) sent as fixed32: kept as an unknown field
    std::string w("\x0d\x01\x00\x00\x00", 5);
    Message* m = e.node->prototype->New();
    ASSERT_TRUE(m->ParseFromString(w));
    EXPECT_FALSE(Reflection::HasField(*m, e.f("i32")));
    EXPECT_EQ(m->SerializeAsString(), w);  // round-trips untouched
    delete m;
}

TEST(PbDepth, malformed_input_rejected) {
    Env e;
    const std::string bad[] = {
        std::string("\x08", 1),                                       // tag without value
        std::string("\x08\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff\x01", 12),  // 11-byte varint
        std::string("\x52\x05" "abc", 5),                             // length past the end
        std::string("\x5a\x03\x08", 3),                               // nested message cut short
        std::string("\x00\x01", 2),                                   // field number 0
        std::string("\x0f", 1),                                       // wire type 7
        std::string("\x3d\x01\x02", 3),                               // fixed32 cut short
    };
    for (size_t i = 0; i < sizeof(bad) / sizeof(bad[0]); ++i) {
        Message* m = e.node->prototype->New();
        const bool ok = m->ParseFromString(bad[i]);
        if (ok) fprintf(stderr, "malformed case %zu parsed\n", i);
        EXPECT_FALSE(ok);
        delete m;
    }
}

TEST(PbDepth, nesting_limit) {
    Env e;
    // child { child { ... } } nested deeper than the limit: refused, no
    // stack exhaustion; within the limit: fine
    auto nested = [](int depth) {
        std::string inner;
        for (int i = 0; i < depth; ++i) {
            std::string w;
            w += (char)0x82;  // field 16, wire 2: tag 0x82 0x01
            w += (char)0x01;
            size_t n = inner.size();
            do {
                w += (char)((n & 0x7f) | (n >= 0x80 ? 0x80 : 0));
                n >>= 7;
            } while (n);
            inner = w + inner;
        }
        return inner;
    };
    Message* ok = e.node->prototype->New();
    EXPECT_TRUE(ok->ParseFromString(nested(50)));
    Message* deep = e.node->prototype->New();
    EXPECT_FALSE(deep->ParseFromString(nested(5000)));
    delete ok;
    delete deep;
}

TEST(PbDepth, clear_resets_presence_and_defaults) {
    Env e;
    Message* m = e.node->prototype->New();
    Reflection::SetInt32(m, e.f("i32"), 3);
    Reflection::SetString(m, e.f("a"), "x");
    Reflection::AddInt32(m, e.f("ints"), 1);
    Reflection::MutableMessage(m, e.f("leaf"));
    EXPECT_TRUE(Reflection::HasField(*m, e.f("leaf")));
    m->Clear();
    EXPECT_FALSE(Reflection::HasField(*m, e.f("i32")));
    EXPECT_FALSE(Reflection::HasField(*m, e.f("a")));
    EXPECT_FALSE(Reflection::HasField(*m, e.f("leaf")));
    EXPECT_EQ(Reflection::FieldSize(*m, e.f("ints")), 0);
    EXPECT_EQ(m->ByteSizeLong(), 0u);
    EXPECT_EQ(m->SerializeAsString(), std::string());
    delete m;
}

TEST(PbDepth, floats_and_packed_zigzag_round_trip) {
    Env e;
    Message* m = e.node->prototype->New();
    Reflection::SetFloat(m, e.f("f"), -0.0f);
    Reflection::SetDouble(m, e.f("dd"), 1e308);
    const int64_t vals[] = {0, -1, 1, INT64_MIN, INT64_MAX, -300};
    for (int64_t v : vals) Reflection::AddInt64(m, e.f("packed_s64"), v);
    const std::string w = m->SerializeAsString();
    EXPECT_EQ(m->ByteSizeLong(), w.size());
    Message* b = e.node->prototype->New();
    ASSERT_TRUE(b->ParseFromString(w));
    const float f = Reflection::GetFloat(*b, e.f("f"));
    EXPECT_TRUE(f == 0.0f && std::signbit(f));
    EXPECT_EQ(Reflection::GetDouble(*b, e.f("dd")), 1e308);
    ASSERT_EQ(Reflection::FieldSize(*b, e.f("packed_s64")), 6);
    for (int i = 0; i < 6; ++i) EXPECT_EQ(Reflection::GetRepeatedInt64(*b, e.f("packed_s64"), i), vals[i]);
    // packed zigzag: tag (19 << 3 | 2) = 9a 01, 25 payload bytes, then the
    // zigzag varints 0, 1, 2, 2^64-1, 2^64-2, 599
    const std::string want = "9a0119" "000102" "ffffffffffffffffff01" "feffffffffffffffff01" "d704";
    EXPECT_TRUE(hex(w).find(want) != std::string::npos);
    delete m;
    delete b;
}

TEST(PbDepth, generated_and_dynamic_agree) {
    // the generated EchoRequest and a dynamic message built from the same
    // .proto text produce the same bytes
    example::EchoRequest g;
    g.set_message(std::string(300, 'q'));
    g.set_sleep_us(-2);
    g.set_server_fail(false);
    const std::string gw = g.SerializeAsString();
    const Descriptor* d = example::EchoRequest::descriptor();
    Message* dyn = d->prototype->New();
    ASSERT_TRUE(dyn->ParseFromString(gw));
    EXPECT_EQ(dyn->SerializeAsString(), gw);
    EXPECT_EQ(dyn->ByteSizeLong(), gw.size());
    delete dyn;
}

// The device-pack contract: with a PackedRunSink installed the
// serializer writes tag + length of large packed varint runs, skips their
// payload and hands the runs over; filling them (here with the host
// encoder the device path falls back to) gives the ordinary encoding.
namespace {
struct CollectRuns : public PackedRunSink {
    size_t min = 1;
    std::vector<PackedRun> runs;
    size_t min_elems() const override { return min; }
    void Take(PackedRun&& r) override { runs.push_back(std::move(r)); }
};
}  // namespace

TEST(PbDepth, packed_run_sink_skips_and_host_fill_matches) {
    example::EchoRequest req;
    req.set_message("hdr");
    const int64_t vals[] = {0, 1, 127, 128, -1, (int64_t)1 << 62, -((int64_t)1 << 40), 300};
    for (int rep = 0; rep < 700; ++rep) {
        for (int64_t v : vals) req.add_ids(v * (rep + 1));
    }
    const std::string want = req.SerializeAsString();
    const size_t n = req.ByteSizeLong();
    ASSERT_TRUE(n == want.size());
    std::string got(n, '\xAA');
    CollectRuns sink;
    sink.min = 4096;
    PackedRunSink* prev = SetThreadPackedRunSink(&sink);
    uint8_t* e = req.SerializeWithCachedSizesToArray(reinterpret_cast<uint8_t*>(&got[0]));
    SetThreadPackedRunSink(prev);
    EXPECT_EQ((size_t)(e - reinterpret_cast<uint8_t*>(&got[0])), n);
    ASSERT_TRUE(sink.runs.size() == 1u);
    const PackedRun& r = sink.runs[0];
    EXPECT_EQ(r.n, (size_t)5600);
    EXPECT_EQ(r.elem_bytes, (size_t)8);
    EXPECT_EQ(r.chunk_bytes.size(), (size_t)3);  // 2048 + 2048 + 1504 elements
    size_t sum = 0;
    for (uint32_t c : r.chunk_bytes) sum += c;
    EXPECT_EQ(sum, r.bytes);
    // the payload was skipped (still the fill pattern), the rest is final
    const size_t off = (size_t)(r.dst - reinterpret_cast<uint8_t*>(&got[0]));
    EXPECT_EQ(got.substr(0, off), want.substr(0, off));
    EXPECT_EQ(got.substr(off, 4), std::string(4, '\xAA'));
    EXPECT_EQ(got.substr(off + r.bytes), want.substr(off + r.bytes));
    EncodePackedRunOnHost(r);
    EXPECT_EQ(got, want);
    // below the threshold nothing is handed over
    CollectRuns high;
    high.min = 100000;
    prev = SetThreadPackedRunSink(&high);
    std::string plain(n, '\0');
    req.SerializeWithCachedSizesToArray(reinterpret_cast<uint8_t*>(&plain[0]));
    SetThreadPackedRunSink(prev);
    EXPECT_TRUE(high.runs.empty());
    EXPECT_EQ(plain, want);
}

TEST(PbDepth, packed_run_sink_every_varint_type) {
    // dynamic message with one packed field per varint type: the host fill
    // reproduces the ordinary bytes for each (negative int32 -> 10 bytes,
    // zigzag for sint, 0/1 for bool)
    const char* proto = R"(
syntax = "proto2";
package pr;
message All {
  repeated int32 a = 1 [packed = true];
  repeated uint32 b = 2 [packed = true];
  repeated sint32 c = 3 [packed = true];
  repeated int64 d = 4 [packed = true];
  repeated uint64 e = 5 [packed = true];
  repeated sint64 f = 6 [packed = true];
  repeated bool g = 7 [packed = true];
  repeated fixed32 h = 8 [packed = true];
}
)";
    Importer imp{{}};
    std::string err;
    ASSERT_TRUE(imp.ImportFromString("pr.proto", proto, &err) != nullptr);
    const Descriptor* d = imp.FindMessageTypeByName("pr.All");
    ASSERT_TRUE(d != nullptr);
    std::unique_ptr<Message> m(d->prototype->New());
    for (int i = 0; i < 3000; ++i) {
        const int64_t x = (int64_t)i * 2654435761LL * ((i & 1) ? -1 : 1);
        Reflection::AddInt32(m.get(), d->FindFieldByName("a"), (int32_t)x);
        Reflection::AddUInt32(m.get(), d->FindFieldByName("b"), (uint32_t)x);
        Reflection::AddInt32(m.get(), d->FindFieldByName("c"), (int32_t)x);
        Reflection::AddInt64(m.get(), d->FindFieldByName("d"), x << (i % 20));
        Reflection::AddUInt64(m.get(), d->FindFieldByName("e"), (uint64_t)x << (i % 30));
        Reflection::AddInt64(m.get(), d->FindFieldByName("f"), x);
        Reflection::AddBool(m.get(), d->FindFieldByName("g"), (i % 3) == 0);
        Reflection::AddUInt32(m.get(), d->FindFieldByName("h"), (uint32_t)i);
    }
    const std::string want = m->SerializeAsString();
    std::string got(want.size(), '\0');
    CollectRuns sink;
    sink.min = 2000;
    m->ByteSizeLong();
    PackedRunSink* prev = SetThreadPackedRunSink(&sink);
    m->SerializeWithCachedSizesToArray(reinterpret_cast<uint8_t*>(&got[0]));
    SetThreadPackedRunSink(prev);
    EXPECT_EQ(sink.runs.size(), (size_t)7);  // every varint type; fixed32 stays on the host
    for (const PackedRun& r : sink.runs) EncodePackedRunOnHost(r);
    EXPECT_EQ(got, want);
}

// The parse half: MergeFromFieldTable hands large packed runs to a decoder
// in one call and appends what it decoded; runs it leaves (values null)
// and small runs are parsed on the host. Host stand-in decoder here.
namespace {
struct HostRunDecoder : public PackedRunDecoder {
    size_t min = 64;
    int calls = 0;
    size_t runs_seen = 0;
    bool skip_second = false;
    std::vector<std::vector<int64_t>> keep;
    size_t min_bytes() const override { return min; }
    void Decode(std::vector<PackedRunIn>* runs) override {
        ++calls;
        for (size_t k = 0; k < runs->size(); ++k) {
            PackedRunIn& r = (*runs)[k];
            ++runs_seen;
            if (skip_second && k == 1) continue;
            CodedInput in(r.p, r.len);
            keep.emplace_back();
            while (!in.at_limit()) {
                uint64_t x;
                if (!in.read_varint(&x)) return;
                keep.back().push_back((int64_t)x);
            }
            r.values = keep.back().data();
            r.count = keep.back().size();
        }
    }
};

// pb_scan-style table of a wire buffer (host walk)
std::vector<uint64_t> field_table(const std::string& w) {
    std::vector<uint64_t> t;
    CodedInput in(w.data(), w.size());
    const uint8_t* base = reinterpret_cast<const uint8_t*>(w.data());
    size_t pos = 0;
    while (pos < w.size()) {
        CodedInput c(base + pos, w.size() - pos);
        const uint32_t tag = c.read_tag();
        uint64_t v = 0;
        const size_t hdr = w.size() - pos - c.bytes_left();
        if ((tag & 7) == 2) {
            uint64_t len;
            c.read_varint(&len);
            const size_t lh = w.size() - pos - c.bytes_left();
            v = ((uint64_t)(pos + lh) << 32) | len;
            pos += lh + len;
        } else {
            c.read_varint(&v);
            pos += w.size() - pos - c.bytes_left();
        }
        (void)hdr;
        t.push_back(tag);
        t.push_back(v);
    }
    return t;
}
}  // namespace

TEST(PbDepth, field_table_merge_with_run_decoder) {
    example::EchoRequest req;
    req.set_message("m");
    for (int i = 0; i < 3000; ++i) req.add_ids((int64_t)i * 1000003 - 7);
    const std::string w = req.SerializeAsString();
    const std::vector<uint64_t> t = field_table(w);
    example::EchoRequest a, b;
    HostRunDecoder dec;
    ASSERT_TRUE(a.MergeFromFieldTable(reinterpret_cast<const uint8_t*>(w.data()), w.size(), t.data(),
                                      (int)t.size() / 2, &dec));
    EXPECT_EQ(dec.calls, 1);
    EXPECT_EQ(dec.runs_seen, (size_t)1);
    EXPECT_EQ(a.SerializeAsString(), w);
    // runs below min_bytes never reach the decoder
    HostRunDecoder big;
    big.min = 1 << 20;
    ASSERT_TRUE(b.MergeFromFieldTable(reinterpret_cast<const uint8_t*>(w.data()), w.size(), t.data(),
                                      (int)t.size() / 2, &big));
    EXPECT_EQ(big.calls, 0);
    EXPECT_EQ(b.SerializeAsString(), w);
    // a wire with the field split in two runs: the decoder declines the
    // second, the host parses it, order is kept
    example::EchoRequest h1, h2;
    for (int i = 0; i < 100; ++i) h1.add_ids(i);
    for (int i = 0; i < 100; ++i) h2.add_ids(1000 + i);
    const std::string w2 = h1.SerializeAsString() + h2.SerializeAsString();
    const std::vector<uint64_t> t2 = field_table(w2);
    example::EchoRequest c;
    HostRunDecoder part;
    part.min = 16;
    part.skip_second = true;
    ASSERT_TRUE(c.MergeFromFieldTable(reinterpret_cast<const uint8_t*>(w2.data()), w2.size(), t2.data(),
                                      (int)t2.size() / 2, &part));
    EXPECT_EQ(part.calls, 1);
    EXPECT_EQ(part.runs_seen, (size_t)2);
    ASSERT_EQ(c.ids_size(), 200);
    for (int i = 0; i < 100; ++i) {
        EXPECT_EQ(c.ids(i), (int64_t)i);
        EXPECT_EQ(c.ids(100 + i), (int64_t)(1000 + i));
    }
}

TEST(PbDepth, repeated_scalar_data_views_the_vectors) {
    Env e;
    ASSERT_TRUE(e.node != nullptr);
    std::unique_ptr<Message> m(e.node->prototype->New());
    for (int i = 0; i < 5; ++i) Reflection::AddInt32(m.get(), e.f("ints"), i * 3);
    size_t n = 0, eb = 0;
    const void* p = Reflection::RepeatedScalarData(*m, e.f("ints"), &n, &eb);
    ASSERT_TRUE(p != nullptr);
    EXPECT_EQ(n, (size_t)5);
    EXPECT_EQ(eb, (size_t)4);
    EXPECT_EQ(static_cast<const int32_t*>(p)[4], 12);
    // strings, messages and singular fields have no scalar array
    EXPECT_TRUE(Reflection::RepeatedScalarData(*m, e.f("leaves"), &n, &eb) == nullptr);
    EXPECT_EQ(n, (size_t)0);
    EXPECT_TRUE(Reflection::RepeatedScalarData(*m, e.f("i32"), &n, &eb) == nullptr);
    // the bulk packed parser fills the same vector the element path would
    const std::string w = m->SerializeAsString();
    std::unique_ptr<Message> back(e.node->prototype->New());
    ASSERT_TRUE(back->ParseFromString(w));
    EXPECT_EQ(back->SerializeAsString(), w);
    EXPECT_EQ(Reflection::FieldSize(*back, e.f("ints")), 5);
}
