// protobuf codec tests (spirit of reference test/brpc_proto_unittest.cpp,
// brpc_repeated_field_unittest.cpp). Wire compatibility with the python
// protobuf runtime is checked from pytest (tests/test_pb_wire_compat.py).
#include "base/buf.h"
#include "mrpc/proto/echo.pb.h"
#include "mrpc/proto/rpc_meta.pb.h"
#include "pb/dynamic.h"
#include "pb/parser.h"
#include "tests/test.h"

using namespace mrpc;
using namespace mrpc::pb;

TEST(Pb, generated_roundtrip) {
    example::EchoRequest req;
    EXPECT_FALSE(req.IsInitialized());
    req.set_message("hello world");
    req.set_sleep_us(-5);
    req.set_server_fail(true);
    EXPECT_TRUE(req.IsInitialized());
    std::string wire = req.SerializeAsString();
    // field1: 0a 0b "hello world"; field2 varint -5 (10 bytes); field3 bool
    EXPECT_EQ((int)(unsigned char)wire[0], 0x0a);
    EXPECT_EQ(wire.size(), 2u + 11u + 1u + 10u + 2u);
    example::EchoRequest back;
    ASSERT_TRUE(back.ParseFromString(wire));
    EXPECT_EQ(back.message(), "hello world");
    EXPECT_EQ(back.sleep_us(), -5);
    EXPECT_TRUE(back.server_fail());
    EXPECT_FALSE(back.has_close_fd());
    EXPECT_EQ(back.ShortDebugString(), "message: \"hello world\" sleep_us: -5 server_fail: true");
    Buf b;
    ASSERT_TRUE(req.SerializeToBuf(&b));
    example::EchoRequest fromb;
    ASSERT_TRUE(fromb.ParseFromBuf(b));
    EXPECT_EQ(fromb.message(), "hello world");
}

TEST(Pb, nested_meta) {
    policy::RpcMeta meta;
    meta.mutable_request()->set_service_name("example.EchoService");
    meta.mutable_request()->set_method_name("Echo");
    meta.mutable_request()->set_log_id(123456789012LL);
    meta.set_correlation_id(0x1234567800000001LL);
    meta.set_attachment_size(64);
    auto* dp = meta.add_device_payload();
    dp->set_ring_offset(4096);
    dp->set_length(65536);
    std::string wire = meta.SerializeAsString();
    policy::RpcMeta back;
    ASSERT_TRUE(back.ParseFromString(wire));
    EXPECT_EQ(back.request().service_name(), "example.EchoService");
    EXPECT_EQ(back.request().log_id(), 123456789012LL);
    EXPECT_EQ(back.correlation_id(), 0x1234567800000001LL);
    ASSERT_EQ(back.device_payload_size(), 1);
    EXPECT_EQ(back.device_payload(0).length(), 65536);
    EXPECT_FALSE(back.has_response());
    // missing required field in nested message -> not initialized
    policy::RpcMeta bad;
    bad.mutable_request()->set_service_name("x");
    EXPECT_FALSE(bad.IsInitialized());
    EXPECT_EQ(bad.InitializationErrorString(), "request.method_name");
}

static const char* kTestProto = R"(
syntax = "proto2";
package t;
enum Color { RED = 0; GREEN = 1; BLUE = 2; }
message Inner { optional int32 a = 1; repeated string tags = 2; }
message All {
  optional double d = 1;
  optional float f = 2;
  optional int64 i64 = 3 [default = -7];
  optional uint64 u64 = 4;
  optional int32 i32 = 5;
  optional fixed64 f64 = 6;
  optional fixed32 f32 = 7;
  optional bool b = 8;
  optional string s = 9 [default = "dflt"];
  optional Inner inner = 11;
  optional bytes by = 12;
  optional uint32 u32 = 13;
  optional Color color = 14 [default = BLUE];
  optional sfixed32 sf32 = 15;
  optional sfixed64 sf64 = 16;
  optional sint32 si32 = 17;
  optional sint64 si64 = 18;
  repeated int32 packed_i32 = 19 [packed = true];
  repeated int32 unpacked_i32 = 20;
  repeated Inner inners = 21;
  map<string, int32> counts = 22;
  oneof choice { string name = 23; int32 id = 24; }
  repeated Color colors = 25;
}
)";

TEST(Pb, dynamic_all_types) {
    Importer imp({});
    std::string err;
    const FileDescriptor* fd = imp.ImportFromString("t.proto", kTestProto, &err);
    ASSERT_TRUE(fd != nullptr);
    const Descriptor* d = imp.FindMessageTypeByName("t.All");
    ASSERT_TRUE(d != nullptr);
    Message* m = d->prototype->New();
    // defaults
    EXPECT_EQ(Reflection::GetInt64(*m, d->FindFieldByName("i64")), -7);
    EXPECT_EQ(Reflection::GetString(*m, d->FindFieldByName("s")), "dflt");
    EXPECT_EQ(Reflection::GetEnumValue(*m, d->FindFieldByName("color")), 2);
    Reflection::SetDouble(m, d->FindFieldByName("d"), 3.5);
    Reflection::SetFloat(m, d->FindFieldByName("f"), -1.25f);
    Reflection::SetUInt64(m, d->FindFieldByName("u64"), 0xFFFFFFFFFFFFFFFFull);
    Reflection::SetInt32(m, d->FindFieldByName("i32"), -1);
    Reflection::SetInt32(m, d->FindFieldByName("si32"), -100);
    Reflection::SetInt64(m, d->FindFieldByName("si64"), -1000000000000LL);
    Reflection::SetBool(m, d->FindFieldByName("b"), true);
    Reflection::SetString(m, d->FindFieldByName("by"), std::string("\0\1\2", 3));
    for (int i = 0; i < 5; ++i) {
        Reflection::AddInt32(m, d->FindFieldByName("packed_i32"), i * 300);
        Reflection::AddInt32(m, d->FindFieldByName("unpacked_i32"), -i);
    }
    Message* in = Reflection::MutableMessage(m, d->FindFieldByName("inner"));
    Reflection::SetInt32(in, in->GetDescriptor()->FindFieldByName("a"), 9);
    Reflection::AddString(in, in->GetDescriptor()->FindFieldByName("tags"), "x");
    Message* e = Reflection::AddMessage(m, d->FindFieldByName("counts"));
    Reflection::SetString(e, e->GetDescriptor()->FindFieldByName("key"), "k");
    Reflection::SetInt32(e, e->GetDescriptor()->FindFieldByName("value"), 5);
    Reflection::SetString(m, d->FindFieldByName("name"), "nm");
    Reflection::SetInt32(m, d->FindFieldByName("id"), 77);  // clears name (oneof)
    EXPECT_FALSE(Reflection::HasField(*m, d->FindFieldByName("name")));
    Reflection::AddEnumValue(m, d->FindFieldByName("colors"), 1);
    std::string wire = m->SerializeAsString();
    Message* m2 = d->prototype->New();
    ASSERT_TRUE(m2->ParseFromString(wire));
    EXPECT_EQ(m2->SerializeAsString(), wire);
    EXPECT_EQ(Reflection::GetDouble(*m2, d->FindFieldByName("d")), 3.5);
    EXPECT_EQ(Reflection::GetUInt64(*m2, d->FindFieldByName("u64")), 0xFFFFFFFFFFFFFFFFull);
    EXPECT_EQ(Reflection::GetInt32(*m2, d->FindFieldByName("si32")), -100);
    EXPECT_EQ(Reflection::FieldSize(*m2, d->FindFieldByName("packed_i32")), 5);
    EXPECT_EQ(Reflection::GetRepeatedInt32(*m2, d->FindFieldByName("packed_i32"), 4), 1200);
    EXPECT_EQ(Reflection::GetInt32(*m2, d->FindFieldByName("id")), 77);
    EXPECT_EQ(Reflection::GetString(*m2, d->FindFieldByName("by")), std::string("\0\1\2", 3));
    // packed and unpacked encodings are accepted interchangeably
    Message* m3 = d->prototype->New();
    ASSERT_TRUE(m3->ParseFromString(wire));
    delete m;
    delete m2;
    delete m3;
}

TEST(Pb, unknown_fields_preserved) {
    // An RpcMeta with a field the (older) EchoRequest does not know.
    example::EchoRequest r;
    r.set_message("m");
    std::string wire = r.SerializeAsString();
    wire += std::string("\xa0\x06\x01", 3);  // field 100 varint 1
    example::EchoRequest back;
    ASSERT_TRUE(back.ParseFromString(wire));
    EXPECT_EQ(back.unknown_fields().size(), 3u);
    EXPECT_EQ(back.SerializeAsString(), wire);
    // truncated input fails
    example::EchoRequest t;
    EXPECT_FALSE(t.ParseFromString(wire.substr(0, 2)));
}

TEST(Pb, service_descriptor) {
    const ServiceDescriptor* sd = example::EchoService::descriptor();
    ASSERT_TRUE(sd != nullptr);
    EXPECT_EQ(sd->full_name, "example.EchoService");
    ASSERT_EQ(sd->method_count(), 1);
    EXPECT_EQ(sd->method(0)->input_type, example::EchoRequest::descriptor());
    EXPECT_TRUE(DescriptorPool::generated_pool()->FindMethodByName("example.EchoService.Echo") != nullptr);
}

// Host construction of the GPU pb_scan table ({tag, value} pairs; wire 2
// values are (offset << 32) | length) for MergeFromFieldTable.
static std::vector<uint64_t> scan_fields(const std::string& wire) {
    std::vector<uint64_t> t;
    CodedInput in(wire.data(), wire.size());
    for (;;) {
        const uint32_t tag = in.read_tag();
        if (tag == 0) break;
        uint64_t v = 0;
        switch (tag & 7) {
        case 0: in.read_varint(&v); break;
        case 1: in.read_fixed64(&v); break;
        case 5: {
            uint32_t x = 0;
            in.read_fixed32(&x);
            v = x;
            break;
        }
        case 2: {
            uint64_t len = 0;
            const uint8_t* d = nullptr;
            in.read_varint(&len);
            in.read_bytes((size_t)len, &d);
            v = ((uint64_t)(d - (const uint8_t*)wire.data()) << 32) | len;
            break;
        }
        }
        t.push_back(tag);
        t.push_back(v);
    }
    return t;
}

TEST(Pb, merge_from_field_table) {
    Importer imp({});
    std::string err;
    ASSERT_TRUE(imp.ImportFromString("t.proto", kTestProto, &err) != nullptr);
    const Descriptor* d = imp.FindMessageTypeByName("t.All");
    Message* m = d->prototype->New();
    Reflection::SetDouble(m, d->FindFieldByName("d"), -2.5);
    Reflection::SetFloat(m, d->FindFieldByName("f"), 0.75f);
    Reflection::SetInt32(m, d->FindFieldByName("si32"), -100);
    Reflection::SetInt64(m, d->FindFieldByName("si64"), -1000000000000LL);
    Reflection::SetUInt32(m, d->FindFieldByName("f32"), 0xDEADBEEF);
    Reflection::SetInt32(m, d->FindFieldByName("sf32"), -3);
    Reflection::SetString(m, d->FindFieldByName("by"), std::string(70000, 'z'));
    for (int i = 0; i < 40; ++i) Reflection::AddInt32(m, d->FindFieldByName("packed_i32"), i * 1000 - 7);
    Reflection::AddInt32(m, d->FindFieldByName("unpacked_i32"), -9);
    Message* in = Reflection::AddMessage(m, d->FindFieldByName("inners"));
    Reflection::SetInt32(in, in->GetDescriptor()->FindFieldByName("a"), 5);
    Reflection::AddString(in, in->GetDescriptor()->FindFieldByName("tags"), "t1");
    Reflection::SetString(m, d->FindFieldByName("name"), "oneof-name");
    const std::string wire = m->SerializeAsString();
    const std::vector<uint64_t> table = scan_fields(wire);
    Message* back = d->prototype->New();
    ASSERT_TRUE(back->MergeFromFieldTable((const uint8_t*)wire.data(), wire.size(), table.data(),
                                          (int)table.size() / 2));
    EXPECT_EQ(back->SerializeAsString(), wire);
    EXPECT_EQ(Reflection::GetInt64(*back, d->FindFieldByName("si64")), -1000000000000LL);
    EXPECT_EQ(Reflection::GetFloat(*back, d->FindFieldByName("f")), 0.75f);
    EXPECT_EQ(Reflection::FieldSize(*back, d->FindFieldByName("packed_i32")), 40);
    // declines what the table cannot express: ranges past the data, unknown fields
    std::vector<uint64_t> bad = table;
    for (size_t i = 0; i < bad.size(); i += 2) {
        if ((bad[i] & 7) == 2) bad[i + 1] = ((uint64_t)wire.size() << 32) | 1;
    }
    Message* b2 = d->prototype->New();
    EXPECT_FALSE(b2->MergeFromFieldTable((const uint8_t*)wire.data(), wire.size(), bad.data(), (int)bad.size() / 2));
    const uint64_t unknown[2] = {(99u << 3) | 0, 1};
    Message* b3 = d->prototype->New();
    EXPECT_FALSE(b3->MergeFromFieldTable((const uint8_t*)wire.data(), wire.size(), unknown, 1));
    delete m;
    delete back;
    delete b2;
    delete b3;
}
