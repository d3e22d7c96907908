// json2pb depth (json/json2pb.h), in the spirit of the reference's
// test/brpc_protobuf_json_unittest.cpp: unicode and control characters both
// ways, maps, edge cases, the expected failures (malformed documents, wrong
// kinds, out-of-range numbers), 64-bit numbers as strings, camelCase names
// and bodies spread over many Buf blocks.
#include <cmath>
#include <limits>
#include <string>

#include "base/buf.h"
#include "json/json.h"
#include "json/json2pb.h"
#include "mrpc/proto/test_services.pb.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

bool to_pb(const std::string& json, pb::Message* m, std::string* err = nullptr,
           const json2pb::Json2PbOptions& o = json2pb::Json2PbOptions()) {
    std::string e;
    const bool ok = json2pb::JsonToProtoMessage(json, m, o, err ? err : &e);
    return ok;
}

std::string to_json(const pb::Message& m, const json2pb::Pb2JsonOptions& o = json2pb::Pb2JsonOptions()) {
    std::string out, err;
    if (!json2pb::ProtoMessageToJson(m, &out, o, &err)) return "<error: " + err + ">";
    return out;
}

bool has(const std::string& hay, const std::string& needle) { return hay.find(needle) != std::string::npos; }

}  // namespace

TEST(Json2pbDepth, unicode_escapes_decode_to_utf8) {
    test::Rich r;
    // BMP escape, a surrogate pair (U+1F600), raw UTF-8 passed through
    ASSERT_TRUE(to_pb("{\"must\":\"\\u4e2d\\u6587\",\"s\":\"\\ud83d\\ude00 caf\xc3\xa9\"}", &r));
    EXPECT_EQ(r.must(), "\xe4\xb8\xad\xe6\x96\x87");
    EXPECT_EQ(r.s(), "\xf0\x9f\x98\x80 caf\xc3\xa9");
}

TEST(Json2pbDepth, unicode_survives_a_round_trip) {
    test::Rich r;
    r.set_must("\xe4\xb8\xad\xe6\x96\x87");
    r.set_s("\xf0\x9f\x98\x80");
    const std::string j = to_json(r);
    test::Rich back;
    ASSERT_TRUE(to_pb(j, &back));
    EXPECT_EQ(back.must(), r.must());
    EXPECT_EQ(back.s(), r.s());
}

TEST(Json2pbDepth, control_characters_are_escaped_on_output) {
    test::Rich r;
    r.set_must(std::string("a\x01" "b\tc\nd\"e\\f\x1f", 13));
    const std::string j = to_json(r);
    EXPECT_TRUE_M(has(j, "\\u0001"), std::string(j));
    EXPECT_TRUE_M(has(j, "\\t"), std::string(j));
    EXPECT_TRUE_M(has(j, "\\n"), std::string(j));
    EXPECT_TRUE_M(has(j, "\\\""), std::string(j));
    EXPECT_TRUE_M(has(j, "\\\\"), std::string(j));
    EXPECT_TRUE_M(has(j, "\\u001f") || has(j, "\\u001F"), std::string(j));
    for (char c : j) EXPECT_TRUE((unsigned char)c >= 0x20);
    test::Rich back;
    ASSERT_TRUE(to_pb(j, &back));
    EXPECT_EQ(back.must(), r.must());
}

TEST(Json2pbDepth, string_escapes_on_input) {
    test::Rich r;
    ASSERT_TRUE(to_pb("{\"must\":\"q\\\"b\\\\s\\/f\\bn\\fr\\rt\\t\"}", &r));
    EXPECT_EQ(r.must(), "q\"b\\s/f\bn\fr\rt\t");
}

TEST(Json2pbDepth, map_fields_are_json_objects_both_ways) {
    test::Rich r;
    ASSERT_TRUE(to_pb("{\"must\":\"m\",\"counts\":{\"a\":1,\"b\":-2,\"\":3}}", &r));
    ASSERT_EQ(r.counts_size(), 3);
    int32_t a = 0, b = 0, empty = 0;
    for (int i = 0; i < r.counts_size(); ++i) {
        if (r.counts(i).key() == "a") a = r.counts(i).value();
        if (r.counts(i).key() == "b") b = r.counts(i).value();
        if (r.counts(i).key().empty()) empty = r.counts(i).value();
    }
    EXPECT_EQ(a, 1);
    EXPECT_EQ(b, -2);
    EXPECT_EQ(empty, 3);
    const std::string j = to_json(r);
    EXPECT_TRUE_M(has(j, "\"counts\":{"), std::string(j));
    EXPECT_TRUE_M(has(j, "\"a\":1"), std::string(j));
    // a map whose value has the wrong kind is reported
    test::Rich bad;
    std::string err;
    to_pb("{\"must\":\"m\",\"counts\":{\"a\":\"x\"}}", &bad, &err);
    EXPECT_FALSE(err.empty());
}

TEST(Json2pbDepth, nested_and_repeated_messages) {
    test::Rich r;
    ASSERT_TRUE(to_pb("{\"must\":\"m\",\"inner\":{\"x\":5,\"tags\":[\"p\",\"q\"]},"
                      "\"inners\":[{\"x\":1},{},{\"tags\":[]}]}", &r));
    EXPECT_EQ(r.inner().x(), 5);
    ASSERT_EQ(r.inner().tags_size(), 2);
    EXPECT_EQ(r.inner().tags(1), "q");
    ASSERT_EQ(r.inners_size(), 3);
    EXPECT_EQ(r.inners(0).x(), 1);
    EXPECT_FALSE(r.inners(1).has_x());
    EXPECT_EQ(r.inners(2).tags_size(), 0);
}

TEST(Json2pbDepth, edge_documents) {
    test::Rich r;
    // whitespace everywhere, an empty nested object, an empty array
    ASSERT_TRUE(to_pb(" \n\t{ \"must\" : \"m\" , \"inner\" : { } , \"nums\" : [ ] } \n", &r));
    EXPECT_TRUE(r.has_inner());
    EXPECT_EQ(r.nums_size(), 0);
    // extreme numbers of every width
    test::Rich n;
    ASSERT_TRUE(to_pb("{\"must\":\"m\",\"i32\":-2147483648,\"i64\":-9223372036854775808,"
                      "\"u64\":18446744073709551615,\"d\":1.7976931348623157e308}", &n));
    EXPECT_EQ(n.i32(), std::numeric_limits<int32_t>::min());
    EXPECT_EQ(n.i64(), std::numeric_limits<int64_t>::min());
    EXPECT_EQ(n.u64(), std::numeric_limits<uint64_t>::max());
    EXPECT_EQ(n.d(), std::numeric_limits<double>::max());
    // a long packed array
    std::string big = "{\"must\":\"m\",\"nums\":[";
    for (int i = 0; i < 5000; ++i) big += (i ? "," : "") + std::to_string(i * 7 - 100);
    big += "]}";
    test::Rich a;
    ASSERT_TRUE(to_pb(big, &a));
    ASSERT_EQ(a.nums_size(), 5000);
    EXPECT_EQ(a.nums(4999), 4999 * 7 - 100);
}

TEST(Json2pbDepth, malformed_documents_fail) {
    const char* bad[] = {
        "",
        "{",
        "{\"must\":\"m\"",
        "{\"must\":\"m\",}",
        "{\"must\" \"m\"}",
        "{\"must\":\"unterminated}",
        "[{\"must\":\"m\"}]",
        "\"must\"",
        "{\"must\":\"m\"} trailing",
        "{'must':'m'}",
        "{\"must\":\"\\x41\"}",
        "{\"must\":\"m\",\"nums\":[1,2,]}",
    };
    for (const char* j : bad) {
        test::Rich r;
        std::string err;
        EXPECT_FALSE_M(to_pb(j, &r, &err), std::string("accepted: ") + std::string(j));
    }
}

TEST(Json2pbDepth, wrong_kinds_are_reported) {
    struct Case {
        const char* json;
        const char* field;
    } cases[] = {
        {"{\"must\":\"m\",\"i32\":5000000000}", "i32"},   // out of range
        {"{\"must\":\"m\",\"u64\":-1}", "u64"},           // negative into unsigned
        {"{\"must\":\"m\",\"i32\":1.5}", "i32"},          // fraction into an integer
        {"{\"must\":\"m\",\"flag\":\"yes\"}", "flag"},    // string into bool
        {"{\"must\":\"m\",\"inner\":[1]}", "inner"},      // array into a message
        {"{\"must\":\"m\",\"nums\":{\"a\":1}}", "nums"},  // object into a repeated scalar
        {"{\"must\":\"m\",\"color\":\"PURPLE\"}", "color"},  // unknown enum name
        {"{\"must\":7}", "must"},                         // number into a string
    };
    for (const Case& c : cases) {
        test::Rich r;
        std::string err;
        const bool ok = to_pb(c.json, &r, &err);
        // either refused outright or accepted with the field left unset and
        // the problem named (the reference's soft-error semantics)
        EXPECT_FALSE_M(err.empty(), std::string(c.json));
        if (ok) EXPECT_TRUE_M(has(err, c.field), std::string(c.json) + std::string(" -> ") + std::string(err));
    }
}

TEST(Json2pbDepth, required_fields_are_enforced_in_nested_messages_too) {
    test::Rich r;
    std::string err;
    EXPECT_FALSE(to_pb("{\"i32\":1}", &r, &err));
    EXPECT_TRUE_M(has(err, "must"), std::string(err));
    // a message with every required field present but an unknown key
    json2pb::Json2PbOptions strict;
    strict.allow_unknown_fields = false;
    EXPECT_FALSE(to_pb("{\"must\":\"m\",\"zzz\":{\"deep\":[1,2]}}", &r, &err, strict));
    EXPECT_TRUE(to_pb("{\"must\":\"m\",\"zzz\":{\"deep\":[1,2]}}", &r, &err));
}

TEST(Json2pbDepth, int64_as_strings_both_ways) {
    test::Rich r;
    ASSERT_TRUE(to_pb("{\"must\":\"m\",\"i64\":\"-9223372036854775808\",\"u64\":\"12345678901234567890\"}", &r));
    EXPECT_EQ(r.i64(), std::numeric_limits<int64_t>::min());
    EXPECT_EQ(r.u64(), 12345678901234567890ULL);
    test::Rich bad;
    std::string err;
    to_pb("{\"must\":\"m\",\"i64\":\"12abc\"}", &bad, &err);
    EXPECT_FALSE(bad.has_i64());
    EXPECT_FALSE(err.empty());
    // printed values parse back exactly
    const std::string j = to_json(r);
    test::Rich back;
    ASSERT_TRUE(to_pb(j, &back));
    EXPECT_EQ(back.i64(), r.i64());
    EXPECT_EQ(back.u64(), r.u64());
}

TEST(Json2pbDepth, doubles_round_trip_exactly) {
    const double vals[] = {0.1, -2.5e-300, 1e21, 123456789.125, 5e-324, 0.0};
    for (double v : vals) {
        test::Rich r;
        r.set_must("m");
        r.set_d(v);
        test::Rich back;
        ASSERT_TRUE(to_pb(to_json(r), &back));
        EXPECT_EQ(back.d(), v);
    }
    test::Rich nan;
    ASSERT_TRUE(to_pb("{\"must\":\"m\",\"d\":\"NaN\"}", &nan));
    EXPECT_TRUE(std::isnan(nan.d()));
}

TEST(Json2pbDepth, json_names_in_camel_case) {
    test::Inner in;
    in.set_x(3);
    in.add_tags("t");
    json2pb::Pb2JsonOptions o;
    o.use_json_name = true;
    const std::string j = to_json(in, o);
    EXPECT_TRUE_M(has(j, "\"x\":3"), std::string(j));
    EXPECT_TRUE_M(has(j, "\"tags\":[\"t\"]"), std::string(j));
}

TEST(Json2pbDepth, pretty_output_parses_back) {
    test::Rich r;
    r.set_must("m");
    r.mutable_inner()->set_x(1);
    r.add_nums(1);
    r.add_nums(2);
    json2pb::Pb2JsonOptions o;
    o.pretty_json = true;
    const std::string j = to_json(r, o);
    EXPECT_TRUE_M(has(j, "\n"), std::string(j));
    test::Rich back;
    ASSERT_TRUE(to_pb(j, &back));
    EXPECT_EQ(back.inner().x(), 1);
    EXPECT_EQ(back.nums_size(), 2);
}

TEST(Json2pbDepth, body_spread_over_many_buf_blocks) {
    std::string j = "{\"must\":\"m\",\"s\":\"";
    j += std::string(20000, 'z');
    j += "\",\"nums\":[";
    for (int i = 0; i < 2000; ++i) j += (i ? "," : "") + std::to_string(i);
    j += "]}";
    Buf b;
    // small user blocks so tokens straddle block boundaries
    for (size_t i = 0; i < j.size(); i += 7) b.append(j.data() + i, std::min<size_t>(7, j.size() - i));
    test::Rich r;
    std::string err;
    ASSERT_TRUE_M(json2pb::JsonToProtoMessage(b, &r, json2pb::Json2PbOptions(), &err), std::string(err));
    EXPECT_EQ(r.s().size(), 20000u);
    ASSERT_EQ(r.nums_size(), 2000);
    EXPECT_EQ(r.nums(1999), 1999);
}

TEST(Json2pbDepth, enums_by_name_and_number) {
    test::Rich r;
    ASSERT_TRUE(to_pb("{\"must\":\"m\",\"color\":\"GREEN\"}", &r));
    EXPECT_EQ(r.color(), test::GREEN);
    test::Rich n;
    ASSERT_TRUE(to_pb("{\"must\":\"m\",\"color\":2}", &n));
    EXPECT_EQ(n.color(), test::BLUE);
    EXPECT_TRUE(has(to_json(n), "\"color\":\"BLUE\""));
}

TEST(Json2pbDepth, bytes_are_base64_both_ways_by_default) {
    test::Rich r;
    r.set_must("m");
    r.set_raw(std::string("\x00\xff\x10" "binary" "\x80", 10));
    const std::string j = to_json(r);
    EXPECT_TRUE_M(has(j, "\"raw\":\"AP8QYmluYXJ5gA==\""), std::string(j));
    test::Rich back;
    ASSERT_TRUE(to_pb(j, &back));
    EXPECT_EQ(back.raw(), r.raw());
    // both directions switched off: the bytes travel as a JSON string
    json2pb::Pb2JsonOptions po;
    po.bytes_to_base64 = false;
    test::Rich t;
    t.set_must("m");
    t.set_raw("plain text");
    const std::string jt = to_json(t, po);
    EXPECT_TRUE_M(has(jt, "\"raw\":\"plain text\""), std::string(jt));
    json2pb::Json2PbOptions jo;
    jo.base64_to_bytes = false;
    test::Rich tb;
    ASSERT_TRUE(to_pb(jt, &tb, nullptr, jo));
    EXPECT_EQ(tb.raw(), "plain text");
}

TEST(Json2pbDepth, invalid_base64_is_refused) {
    const char* bad[] = {"{\"must\":\"m\",\"raw\":\"@@@@\"}", "{\"must\":\"m\",\"raw\":\"QUJD=\"}",
                         "{\"must\":\"m\",\"raw\":12}"};
    for (const char* j : bad) {
        test::Rich r;
        std::string err;
        const bool ok = to_pb(j, &r, &err);
        EXPECT_FALSE_M(err.empty(), std::string(j));
        if (ok) EXPECT_FALSE_M(r.has_raw(), std::string(j));
    }
}

TEST(Json2pbDepth, always_print_primitive_fields) {
    test::Rich r;
    r.set_must("m");
    json2pb::Pb2JsonOptions o;
    EXPECT_FALSE(has(to_json(r, o), "\"i32\""));
    o.always_print_primitive_fields = true;
    const std::string j = to_json(r, o);
    EXPECT_TRUE_M(has(j, "\"i32\":0"), std::string(j));
    EXPECT_TRUE_M(has(j, "\"flag\":false"), std::string(j));
    EXPECT_TRUE_M(has(j, "\"s\":\"\""), std::string(j));
    // the defaults parse back to equal values
    test::Rich back;
    ASSERT_TRUE(to_pb(j, &back));
    EXPECT_EQ(back.i32(), 0);
    EXPECT_EQ(back.s(), "");
}

TEST(Json2pbDepth, empty_repeated_fields_on_request) {
    test::Rich r;
    r.set_must("m");
    EXPECT_FALSE(has(to_json(r), "\"nums\""));
    json2pb::Pb2JsonOptions o;
    o.jsonify_empty_array = true;
    const std::string j = to_json(r, o);
    EXPECT_TRUE_M(has(j, "\"nums\":[]"), std::string(j));
    EXPECT_TRUE_M(has(j, "\"inners\":[]"), std::string(j));
    test::Rich back;
    ASSERT_TRUE(to_pb(j, &back));
    EXPECT_EQ(back.nums_size(), 0);
}

TEST(Json2pbDepth, enums_printed_as_numbers_on_request) {
    test::Rich r;
    r.set_must("m");
    r.set_color(test::BLUE);
    EXPECT_TRUE(has(to_json(r), "\"color\":\"BLUE\""));
    json2pb::Pb2JsonOptions o;
    o.enum_option_as_string = false;
    const std::string j = to_json(r, o);
    EXPECT_TRUE_M(has(j, "\"color\":2"), std::string(j));
    test::Rich back;
    ASSERT_TRUE(to_pb(j, &back));
    EXPECT_EQ(back.color(), test::BLUE);
}

TEST(Json2pbDepth, repeated_messages_and_strings_round_trip) {
    test::Rich r;
    r.set_must("m");
    for (int i = 0; i < 40; ++i) {
        test::Inner* in = r.add_inners();
        in->set_x(i * i - 7);
        for (int k = 0; k < i % 4; ++k) in->add_tags("t" + std::to_string(i) + "\"q\\" + std::to_string(k));
    }
    const std::string j = to_json(r);
    test::Rich back;
    ASSERT_TRUE(to_pb(j, &back));
    ASSERT_EQ(back.inners_size(), 40);
    for (int i = 0; i < 40; ++i) {
        EXPECT_EQ(back.inners(i).x(), i * i - 7);
        ASSERT_EQ(back.inners(i).tags_size(), i % 4);
        for (int k = 0; k < i % 4; ++k) EXPECT_EQ(back.inners(i).tags(k), r.inners(i).tags(k));
    }
}

TEST(Json2pbDepth, infinities_both_ways) {
    test::Rich r;
    r.set_must("m");
    r.set_d(std::numeric_limits<double>::infinity());
    const std::string j = to_json(r);
    test::Rich back;
    ASSERT_TRUE_M(to_pb(j, &back), std::string(j));
    EXPECT_TRUE(std::isinf(back.d()) && back.d() > 0);
    test::Rich neg;
    ASSERT_TRUE(to_pb("{\"must\":\"m\",\"d\":\"-Infinity\"}", &neg));
    EXPECT_TRUE(std::isinf(neg.d()) && neg.d() < 0);
}

TEST(Json2pbDepth, missing_required_field_on_output_is_reported) {
    test::Rich r;  // `must` unset
    r.set_i32(3);
    std::string out, err;
    const bool ok = json2pb::ProtoMessageToJson(r, &out, json2pb::Pb2JsonOptions(), &err);
    // refused, or printed with the problem named (either keeps the caller
    // from shipping a message its peer cannot parse without knowing)
    EXPECT_TRUE_M(!ok || has(err, "must"), std::string(out) + " / " + std::string(err));
}

TEST(Json2pbDepth, unknown_nested_keys_of_every_kind_are_skipped) {
    test::Rich r;
    ASSERT_TRUE(to_pb("{\"zz0\":null,\"must\":\"m\",\"zz1\":[{},[],null,true,-1.5e3,\"s\"],"
                      "\"inner\":{\"x\":5,\"unknown\":{\"deep\":[{\"a\":{\"b\":[1]}}]}},\"zz2\":false}", &r));
    EXPECT_EQ(r.must(), "m");
    EXPECT_EQ(r.inner().x(), 5);
    // the same document is refused by a strict parser, naming the key
    json2pb::Json2PbOptions strict;
    strict.allow_unknown_fields = false;
    test::Rich s2;
    std::string err;
    EXPECT_FALSE(to_pb("{\"must\":\"m\",\"inner\":{\"x\":5,\"unknown\":1}}", &s2, &err, strict));
    EXPECT_TRUE_M(has(err, "unknown"), std::string(err));
}
