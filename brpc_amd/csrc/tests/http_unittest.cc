// HTTP protocol + json2pb + builtin pages (spirit of the reference's
// test/brpc_http_rpc_protocol_unittest.cpp, brpc_http_message_unittest.cpp,
// test/brpc_builtin_service_unittest.cpp, json2pb unittests).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cmath>
#include <cstring>
#include <cerrno>
#include <thread>

#include "base/flags.h"

#include "base/time.h"
#include "fiber/fiber.h"
#include "http/http_header.h"
#include "http/hpack.h"
#include "http/http_message.h"
#include "json/json.h"
#include "json/json2pb.h"
#include "mrpc/proto/echo.pb.h"
#include "mrpc/proto/test_services.pb.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/progressive.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

class HttpTestImpl : public test::HttpTest {
public:
    void Push(RpcController* c, const test::Empty*, test::Empty*, Closure* done) override {
        Controller* cntl = static_cast<Controller*>(c);
        auto pa = cntl->CreateProgressiveAttachment();
        done->Run();  // header goes out now; the body follows
        std::thread([pa] {
            for (int i = 0; i < 5; ++i) {
                pa->Write("part" + std::to_string(i) + ";");
                usleep(2000);
            }
        }).detach();
    }
    void Raw(RpcController* c, const test::Empty*, test::Empty*, Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = static_cast<Controller*>(c);
        cntl->http_response().set_content_type("application/octet-stream");
        cntl->http_response().SetHeader("x-echo-method", HttpMethod2Str(cntl->http_request().method()));
        cntl->response_attachment().append(cntl->request_attachment());
        const std::string* q = cntl->http_request().uri().GetQuery("q");
        if (q) cntl->response_attachment().append("|q=" + *q);
    }
    void Rich(RpcController*, const test::Rich* req, test::Rich* res, Closure* done) override {
        ClosureGuard g(done);
        *res = *req;
        res->set_i32(req->i32() + 1);
    }
};

struct HttpServer {
    Server server;
    EchoServiceImpl echo;
    HttpTestImpl t;
    int port = 0;
    HttpServer() {
        server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        server.AddService(&t, SERVER_DOESNT_OWN_SERVICE, "/v1/raw/* => Raw");
        ServerOptions o;
        if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
    }
    std::string addr() const { return "127.0.0.1:" + std::to_string(port); }
};

}  // namespace

TEST(Json2pb, roundtrip) {
    test::Rich r;
    r.set_i32(-5);
    r.set_i64(1LL << 40);
    r.set_u64(~0ULL);
    r.set_d(2.5);
    r.set_flag(true);
    r.set_s("he\"llo\n");
    r.set_raw(std::string("\x00\x01\xff", 3));
    r.set_color(test::BLUE);
    r.mutable_inner()->set_x(7);
    r.mutable_inner()->add_tags("a");
    r.add_inners()->set_x(1);
    r.add_inners()->set_x(2);
    r.add_nums(3);
    r.add_nums(4);
    {
        test::Rich_CountsEntry* e = r.add_counts();
        e->set_key("k");
        e->set_value(9);
    }
    r.set_must("m");
    std::string json, err;
    ASSERT_TRUE(json2pb::ProtoMessageToJson(r, &json, json2pb::Pb2JsonOptions(), &err));
    EXPECT_TRUE(json.find("\"color\":\"BLUE\"") != std::string::npos);
    EXPECT_TRUE(json.find("\"raw\":\"AAH/\"") != std::string::npos);
    test::Rich back;
    ASSERT_TRUE(json2pb::JsonToProtoMessage(json, &back, json2pb::Json2PbOptions(), &err));
    EXPECT_EQ(back.i64(), 1LL << 40);
    EXPECT_EQ(back.u64(), ~0ULL);
    EXPECT_EQ(back.raw(), std::string("\x00\x01\xff", 3));
    EXPECT_EQ(back.color(), test::BLUE);
    EXPECT_EQ(back.inners_size(), 2);
    EXPECT_EQ(back.inners(1).x(), 2);
    ASSERT_EQ(back.counts_size(), 1);
    EXPECT_EQ(back.counts(0).key(), "k");
    EXPECT_EQ(back.counts(0).value(), 9);
    EXPECT_EQ(back.s(), "he\"llo\n");
    // missing required field / bad type
    test::Rich bad;
    EXPECT_FALSE(json2pb::JsonToProtoMessage("{\"i32\": 1}", &bad, json2pb::Json2PbOptions(), &err));
    // a wrong kind in an optional field is reported but not fatal (reference semantics)
    test::Rich soft;
    EXPECT_TRUE(json2pb::JsonToProtoMessage("{\"must\":\"x\",\"i32\":\"abc\"}", &soft, json2pb::Json2PbOptions(), &err));
    EXPECT_TRUE(err.find("SHOULD be INT32") != std::string::npos);
    EXPECT_FALSE(soft.has_i32());
    json2pb::Json2PbOptions strict;
    strict.allow_unknown_fields = false;
    EXPECT_FALSE(json2pb::JsonToProtoMessage("{\"must\":\"x\",\"nope\":1}", &bad, strict, &err));
}

TEST(Json2pb, scalar_coercions) {
    // 64-bit numbers quoted as strings (how int64 travels through
    // javascript), enums by number, NaN / Infinity, nulls skipped
    const std::string in =
        "{\"must\":\"m\",\"i64\":\"1099511627776\",\"u64\":\"18446744073709551615\",\"i32\":-7,"
        "\"color\":2,\"flag\":true,\"d\":\"-Infinity\",\"s\":null,\"nums\":[1,2,3]}";
    test::Rich r;
    std::string err;
    ASSERT_TRUE(json2pb::JsonToProtoMessage(in, &r, json2pb::Json2PbOptions(), &err));
    EXPECT_EQ(r.i64(), 1099511627776LL);
    EXPECT_EQ(r.u64(), 18446744073709551615ULL);
    EXPECT_EQ(r.i32(), -7);
    EXPECT_EQ((int)r.color(), 2);
    EXPECT_TRUE(r.flag());
    EXPECT_TRUE(std::isinf(r.d()) && r.d() < 0);
    EXPECT_FALSE(r.has_s());
    ASSERT_EQ(r.nums_size(), 3);
    EXPECT_EQ(r.nums(1), 2);
    // bytes: base64 by default, raw text when asked
    test::Rich b1, b2;
    ASSERT_TRUE(json2pb::JsonToProtoMessage("{\"must\":\"m\",\"raw\":\"AAH/\"}", &b1, json2pb::Json2PbOptions(), &err));
    EXPECT_EQ(b1.raw(), std::string("\x00\x01\xff", 3));
    json2pb::Json2PbOptions keep;
    keep.base64_to_bytes = false;
    ASSERT_TRUE(json2pb::JsonToProtoMessage("{\"must\":\"m\",\"raw\":\"AAH/\"}", &b2, keep, &err));
    EXPECT_EQ(b2.raw(), "AAH/");
}

TEST(Json2pb, pb2json_options) {
    test::Rich r;
    r.set_must("m");
    r.set_color(test::BLUE);
    r.set_raw(std::string("\x01\x02", 2));
    std::string out, err;
    json2pb::Pb2JsonOptions o;
    o.enum_option_as_string = false;
    ASSERT_TRUE(json2pb::ProtoMessageToJson(r, &out, o, &err));
    EXPECT_TRUE(out.find("\"color\":2") != std::string::npos);
    EXPECT_TRUE(out.find("\"nums\"") == std::string::npos);  // empty repeated omitted
    o.jsonify_empty_array = true;
    o.bytes_to_base64 = false;
    ASSERT_TRUE(json2pb::ProtoMessageToJson(r, &out, o, &err));
    EXPECT_TRUE(out.find("\"nums\":[]") != std::string::npos);
    EXPECT_TRUE(out.find("\"raw\":\"\\u0001\\u0002\"") != std::string::npos);
    json2pb::Pb2JsonOptions all;
    all.always_print_primitive_fields = true;
    ASSERT_TRUE(json2pb::ProtoMessageToJson(r, &out, all, &err));
    EXPECT_TRUE(out.find("\"i32\":0") != std::string::npos);
    EXPECT_TRUE(out.find("\"flag\":false") != std::string::npos);
    json2pb::Pb2JsonOptions pretty;
    pretty.pretty_json = true;
    ASSERT_TRUE(json2pb::ProtoMessageToJson(r, &out, pretty, &err));
    EXPECT_TRUE(out.find('\n') != std::string::npos);
    test::Rich back;
    ASSERT_TRUE(json2pb::JsonToProtoMessage(out, &back, json2pb::Json2PbOptions(), &err));
    EXPECT_EQ(back.SerializeAsString(), r.SerializeAsString());
}

TEST(Json2pb, type_errors_name_the_field) {
    test::Rich r;
    std::string err;
    EXPECT_FALSE(json2pb::JsonToProtoMessage("[1,2]", &r, json2pb::Json2PbOptions(), &err));
    EXPECT_TRUE(err.find("json object") != std::string::npos);
    EXPECT_FALSE(json2pb::JsonToProtoMessage("{\"must\":\"m\",\"nums\":5}", &r, json2pb::Json2PbOptions(), &err));
    EXPECT_TRUE(err.find("nums") != std::string::npos);
    EXPECT_FALSE(json2pb::JsonToProtoMessage("{\"must\":\"m\",\"counts\":[1]}", &r, json2pb::Json2PbOptions(), &err));
    EXPECT_TRUE(err.find("counts") != std::string::npos);
    // optional fields of the wrong kind: reported, skipped, not fatal
    EXPECT_TRUE(json2pb::JsonToProtoMessage("{\"must\":\"m\",\"color\":\"PURPLE\"}", &r, json2pb::Json2PbOptions(), &err));
    EXPECT_TRUE(err.find("field `mrpc.test.Rich.color' which SHOULD be enum") != std::string::npos);
    EXPECT_TRUE(json2pb::JsonToProtoMessage("{\"must\":\"m\",\"inner\":{\"x\":\"y\"}}", &r, json2pb::Json2PbOptions(), &err));
    EXPECT_TRUE(err.find("SHOULD be INT32") != std::string::npos);
    EXPECT_TRUE(json2pb::JsonToProtoMessage("{\"must\":\"m\",\"s\":7}", &r, json2pb::Json2PbOptions(), &err));
    EXPECT_TRUE(err.find("Invalid value `7'") != std::string::npos);
    // ... but fatal in required and repeated fields
    EXPECT_FALSE(json2pb::JsonToProtoMessage("{\"must\":7}", &r, json2pb::Json2PbOptions(), &err));
    EXPECT_FALSE(json2pb::JsonToProtoMessage("{\"must\":\"m\",\"nums\":[1,\"2\"]}", &r, json2pb::Json2PbOptions(), &err));
    EXPECT_FALSE(json2pb::JsonToProtoMessage("{\"must\":", &r, json2pb::Json2PbOptions(), &err));
    EXPECT_FALSE(err.empty());
}

TEST(Json2pb, large_document_round_trip) {
    test::Rich r;
    r.set_must(std::string(100000, 'q') + "\"\\\n\t end");
    for (int i = 0; i < 3000; ++i) {
        test::Inner* in = r.add_inners();
        in->set_x(i * 7 - 1000);
        in->add_tags("t" + std::to_string(i));
        r.add_nums(i);
    }
    std::string out, err;
    ASSERT_TRUE(json2pb::ProtoMessageToJson(r, &out, json2pb::Pb2JsonOptions(), &err));
    test::Rich back;
    ASSERT_TRUE(json2pb::JsonToProtoMessage(out, &back, json2pb::Json2PbOptions(), &err));
    EXPECT_EQ(back.SerializeAsString(), r.SerializeAsString());
}

// pb2json number-array offload (the device prints large repeated integer
// fields, gpu/json_offload.cc): a host stand-in with the same contract
// gives output identical to the DOM path; pretty output, enums printed as
// names and short fields stay on the DOM path.
namespace {
int g_fake_array_calls = 0;
bool fake_array_offload(const void* values, size_t n, uint32_t kind, std::string* text) {
    ++g_fake_array_calls;
    text->clear();
    for (size_t i = 0; i < n; ++i) {
        if (i) text->push_back(',');
        if (kind == 0) text->append(std::to_string(static_cast<const int32_t*>(values)[i]));
        else if (kind == 3) text->append(std::to_string(static_cast<const int64_t*>(values)[i]));
        else return false;
    }
    return true;
}
}  // namespace

TEST(Json2pb, pb2json_array_offload_matches_dom_output) {
    test::Rich r;
    r.set_must("m");
    for (int i = 0; i < 5000; ++i) r.add_nums(i * 977 - 2000000);
    example::EchoResponse e;
    e.set_message("x");
    for (int i = 0; i < 5000; ++i) e.add_ids(((int64_t)i << 40) * ((i & 1) ? -1 : 1));
    std::string want_r, want_e, got_r, got_e, pretty_want, pretty_got, err;
    json2pb::Pb2JsonOptions opt;
    ASSERT_TRUE(json2pb::ProtoMessageToJson(r, &want_r, opt, &err));
    ASSERT_TRUE(json2pb::ProtoMessageToJson(e, &want_e, opt, &err));
    json2pb::Pb2JsonOptions popt;
    popt.pretty_json = true;
    ASSERT_TRUE(json2pb::ProtoMessageToJson(r, &pretty_want, popt, &err));
    json2pb::SetPb2JsonArrayOffload(fake_array_offload, 4096);
    g_fake_array_calls = 0;
    ASSERT_TRUE(json2pb::ProtoMessageToJson(r, &got_r, opt, &err));
    ASSERT_TRUE(json2pb::ProtoMessageToJson(e, &got_e, opt, &err));
    EXPECT_EQ(g_fake_array_calls, 2);
    ASSERT_TRUE(json2pb::ProtoMessageToJson(r, &pretty_got, popt, &err));
    EXPECT_EQ(g_fake_array_calls, 2);  // pretty output stays on the DOM path
    test::Rich small;
    small.set_must("m");
    for (int i = 0; i < 100; ++i) small.add_nums(i);
    std::string s1;
    ASSERT_TRUE(json2pb::ProtoMessageToJson(small, &s1, opt, &err));
    EXPECT_EQ(g_fake_array_calls, 2);  // below min_elems
    json2pb::SetPb2JsonArrayOffload(nullptr, 0);
    EXPECT_EQ(got_r, want_r);
    EXPECT_EQ(got_e, want_e);
    EXPECT_EQ(pretty_got, pretty_want);
    // and the output parses back to the same message
    test::Rich back;
    ASSERT_TRUE(json2pb::JsonToProtoMessage(got_r, &back, json2pb::Json2PbOptions(), &err));
    EXPECT_EQ(back.SerializeAsString(), r.SerializeAsString());
}

// json2pb integer arrays parsed in bulk (the device parser's contract,
// json::SetIntArrayOffload): with a structural index, arrays of plain
// integers go to the offload in one call and into the message without a
// Value per element; arrays with anything else (a float, a string, an
// out-of-range value for the field) take the element-wise path.
namespace {
int g_fake_int_calls = 0;
bool fake_int_array(const char* base, const uint32_t* seps, size_t nseps, std::vector<int64_t>* out) {
    ++g_fake_int_calls;
    out->clear();
    for (size_t i = 0; i + 1 < nseps; ++i) {
        std::string e(base + seps[i] + 1, seps[i + 1] - seps[i] - 1);
        char* end = nullptr;
        errno = 0;
        const long long x = strtoll(e.c_str(), &end, 10);
        while (end && (*end == ' ' || *end == '\n')) ++end;
        if (errno || !end || *end) return false;
        out->push_back(x);
    }
    return true;
}
std::vector<uint32_t> host_index(const std::string& t) {
    std::vector<uint32_t> idx;
    bool in_str = false;
    for (size_t i = 0; i < t.size(); ++i) {
        const char c = t[i];
        if (in_str) {
            if (c == '\\') ++i;
            else if (c == '"') { in_str = false; idx.push_back((uint32_t)i); }
            continue;
        }
        if (c == '"') { in_str = true; idx.push_back((uint32_t)i); }
        else if (strchr("{}[]:,", c)) idx.push_back((uint32_t)i);
    }
    return idx;
}
}  // namespace

TEST(Json2pb, bulk_int_arrays_with_index) {
    example::EchoRequest want;
    want.set_message("m");
    std::string text = "{\"message\":\"m\",\"ids\":[";
    for (int i = 0; i < 6000; ++i) {
        const int64_t x = ((int64_t)i * 7919) << (i % 40);
        want.add_ids(i % 3 ? x : -x);
        if (i) text += (i % 50 == 0) ? ", " : ",";
        text += std::to_string(i % 3 ? x : -x);
    }
    text += "]}";
    const std::vector<uint32_t> idx = host_index(text);
    json::SetIntArrayOffload(fake_int_array, 4096);
    g_fake_int_calls = 0;
    json::Value v;
    std::string err;
    ASSERT_TRUE(json::ParseWithIndex(text.data(), text.size(), idx.data(), idx.size(), &v, &err));
    EXPECT_EQ(g_fake_int_calls, 1);
    const json::Value* ids = v.find("ids");
    ASSERT_TRUE(ids != nullptr && ids->packed_ints() != nullptr);
    EXPECT_EQ(ids->size(), (size_t)6000);
    example::EchoRequest got;
    ASSERT_TRUE(json2pb::JsonValueToProtoMessage(v, &got, json2pb::Json2PbOptions(), &err));
    EXPECT_EQ(got.SerializeAsString(), want.SerializeAsString());
    // the packed array prints like the element-wise one
    json::Value plain;
    ASSERT_TRUE(json::Parse(text, &plain, &err));
    EXPECT_EQ(v.ToString(), plain.ToString());
    EXPECT_EQ(ids->array().size(), (size_t)6000);  // materialized on demand
    // a float inside: the offload declines, the array parses element-wise
    std::string t2 = text;
    t2.insert(t2.find("[") + 1, "1.5,");
    const std::vector<uint32_t> idx2 = host_index(t2);
    json::Value v2;
    ASSERT_TRUE(json::ParseWithIndex(t2.data(), t2.size(), idx2.data(), idx2.size(), &v2, &err));
    EXPECT_TRUE(v2.find("ids")->packed_ints() == nullptr);
    EXPECT_EQ(v2.find("ids")->size(), (size_t)6001);
    // int32 field out of range: the element-wise rules report it
    test::Rich r;
    std::string t3 = "{\"must\":\"x\",\"nums\":[";
    for (int i = 0; i < 5000; ++i) t3 += std::to_string(i) + ",";
    t3 += "4294967296]}";
    const std::vector<uint32_t> idx3 = host_index(t3);
    json::Value v3;
    ASSERT_TRUE(json::ParseWithIndex(t3.data(), t3.size(), idx3.data(), idx3.size(), &v3, &err));
    EXPECT_TRUE(v3.find("nums")->packed_ints() != nullptr);
    std::string err3;
    EXPECT_FALSE(json2pb::JsonValueToProtoMessage(v3, &r, json2pb::Json2PbOptions(), &err3));
    EXPECT_TRUE(err3.find("nums") != std::string::npos);
    json::SetIntArrayOffload(nullptr, 0);
}

TEST(HttpParser, chunked_and_pipelined) {
    Buf b;
    b.append("POST /a/b?x=1&y=two HTTP/1.1\r\nHost: h\r\nTransfer-Encoding: chunked\r\nContent-Type: text/plain\r\n\r\n"
             "5\r\nhello\r\n6\r\n world\r\n0\r\n\r\n"
             "GET /c HTTP/1.0\r\nContent-Length: 3\r\n\r\nabc");
    HttpParser p(1 << 20);
    std::string err;
    ASSERT_EQ((int)p.Consume(&b, false, &err), (int)HttpParser::DONE);
    std::unique_ptr<HttpMessage> m(p.release());
    EXPECT_EQ(m->header.method(), HTTP_METHOD_POST);
    EXPECT_EQ(m->header.uri().path(), "/a/b");
    EXPECT_EQ(*m->header.uri().GetQuery("y"), "two");
    EXPECT_EQ(m->header.content_type(), "text/plain");
    EXPECT_EQ(m->body.to_string(), "hello world");
    EXPECT_TRUE(m->keep_alive);
    ASSERT_EQ((int)p.Consume(&b, false, &err), (int)HttpParser::DONE);
    m.reset(p.release());
    EXPECT_EQ(m->body.to_string(), "abc");
    EXPECT_FALSE(m->keep_alive);  // HTTP/1.0 default
    EXPECT_TRUE(b.empty());
    // byte-by-byte feeding
    const std::string resp = "HTTP/1.1 404 Not Found\r\nContent-Length: 4\r\nX-A: 1\r\n\r\nnope";
    HttpParser p2(1 << 20);
    Buf in;
    HttpParser::Result r = HttpParser::NEED_MORE;
    for (char ch : resp) {
        in.push_back(ch);
        r = p2.Consume(&in, false, &err);
        if (r != HttpParser::NEED_MORE) break;
    }
    ASSERT_EQ((int)r, (int)HttpParser::DONE);
    m.reset(p2.release());
    EXPECT_TRUE(m->is_response);
    EXPECT_EQ(m->header.status_code(), 404);
    EXPECT_EQ(*m->header.GetHeader("x-a"), "1");
    EXPECT_EQ(m->body.to_string(), "nope");
    // garbage
    Buf g;
    g.append("GET / HTTP/1.1\r\nbad header line\r\n\r\n");
    HttpParser p3(1 << 20);
    EXPECT_EQ((int)p3.Consume(&g, false, &err), (int)HttpParser::FAILED);
}

TEST(Http, pb_over_json_and_proto) {
    HttpServer s;
    ASSERT_GT(s.port, 0);
    Channel ch;
    ChannelOptions opt;
    opt.protocol = "http";
    opt.timeout_ms = 3000;
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    for (int i = 0; i < 20; ++i) {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("json " + std::to_string(i));
        stub.Echo(&cntl, &req, &res, nullptr);
        ASSERT_FALSE(cntl.Failed());
        EXPECT_EQ(res.message(), "json " + std::to_string(i));
        EXPECT_EQ(cntl.http_response().status_code(), 200);
    }
    Controller cntl;
    cntl.http_request().set_content_type("application/proto");
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("proto");
    stub.Echo(&cntl, &req, &res, nullptr);
    ASSERT_FALSE(cntl.Failed());
    EXPECT_EQ(res.message(), "proto");
    EXPECT_EQ(cntl.http_response().content_type(), "application/proto");
    // rich json round trip through a server
    test::HttpTest_Stub t(&ch);
    test::Rich rq, rs;
    rq.set_i32(41);
    rq.set_must("yes");
    rq.set_color(test::GREEN);
    {
        test::Rich_CountsEntry* e = rq.add_counts();
        e->set_key("a");
        e->set_value(1);
    }
    Controller c2;
    t.Rich(&c2, &rq, &rs, nullptr);
    ASSERT_FALSE(c2.Failed());
    EXPECT_EQ(rs.i32(), 42);
    EXPECT_EQ(rs.color(), test::GREEN);
    ASSERT_EQ(rs.counts_size(), 1);
    EXPECT_EQ(rs.counts(0).value(), 1);
}

TEST(Http, plain_calls_builtin_restful_errors) {
    HttpServer s;
    Channel ch;
    ChannelOptions opt;
    opt.protocol = "http";
    opt.timeout_ms = 3000;
    ASSERT_EQ(ch.Init(("http://" + s.addr()).c_str(), &opt), 0);
    {
        Controller cntl;
        cntl.http_request().uri().set_path("/health");
        ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        ASSERT_FALSE(cntl.Failed());
        EXPECT_EQ(cntl.response_attachment().to_string(), "OK\n");
    }
    {
        Controller cntl;
        cntl.http_request().uri().SetHttpURL("/v1/raw/anything?q=zz");
        cntl.http_request().set_method(HTTP_METHOD_PUT);
        cntl.request_attachment().append("body!");
        ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        ASSERT_FALSE(cntl.Failed());
        EXPECT_EQ(cntl.response_attachment().to_string(), "body!|q=zz");
        EXPECT_EQ(*cntl.http_response().GetHeader("x-echo-method"), "PUT");
    }
    {
        Controller cntl;
        cntl.http_request().uri().set_path("/vars/fiber_count");
        ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        ASSERT_FALSE(cntl.Failed());
        EXPECT_GT(atoi(cntl.response_attachment().to_string().c_str()), 0);
    }
    {
        Controller cntl;
        cntl.http_request().uri().set_path("/no/such/method");
        ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        ASSERT_TRUE(cntl.Failed());
        EXPECT_EQ(cntl.ErrorCode(), ENOMETHOD);
        EXPECT_EQ(cntl.http_response().status_code(), 404);
    }
    {
        Controller cntl;  // HEAD: no body even with Content-Length
        cntl.http_request().uri().set_path("/status");
        cntl.http_request().set_method(HTTP_METHOD_HEAD);
        ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        ASSERT_FALSE(cntl.Failed());
        EXPECT_TRUE(cntl.response_attachment().empty());
    }
    {
        Controller cntl;
        cntl.http_request().uri().set_path("/flags/max_body_size");
        cntl.http_request().uri().SetQuery("setvalue", "12345678");
        ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        ASSERT_FALSE(cntl.Failed());
        std::string v;
        GetFlag("max_body_size", &v);
        EXPECT_EQ(v, "12345678");
        SetFlag("max_body_size", "67108864");
    }
}

namespace {
struct CollectReader : public ProgressiveReader {
    std::string data;
    std::atomic<int> ended{0};
    Status st;
    Status OnReadOnePart(const void* d, size_t n) override {
        data.append((const char*)d, n);
        return Status();
    }
    void OnEndOfMessage(const Status& s) override {
        st = s;
        ended.store(1);
    }
};
}  // namespace

TEST(Http, progressive_attachment_and_reader) {
    HttpServer s;
    Channel ch;
    ChannelOptions opt;
    opt.protocol = "http";
    opt.timeout_ms = 3000;
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    // whole body
    {
        Controller cntl;
        cntl.http_request().uri().set_path("/HttpTest/Push");
        ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        ASSERT_FALSE(cntl.Failed());
        EXPECT_EQ(cntl.response_attachment().to_string(), "part0;part1;part2;part3;part4;");
    }
    // progressively
    {
        Controller cntl;
        cntl.http_request().uri().set_path("/HttpTest/Push");
        cntl.response_will_be_read_progressively();
        ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        ASSERT_FALSE(cntl.Failed());
        CollectReader r;
        cntl.ReadProgressiveAttachmentBy(&r);
        for (int i = 0; i < 300 && !r.ended.load(); ++i) usleep(10000);
        EXPECT_EQ(r.ended.load(), 1);
        EXPECT_TRUE(r.st.ok());
        EXPECT_EQ(r.data, "part0;part1;part2;part3;part4;");
    }
}

TEST(Hpack, roundtrip_and_huffman) {
    HPackEncoder enc;
    HPackDecoder dec;
    std::vector<HPackHeader> hs = {{":method", "POST"},
                                   {":path", "/example.EchoService/Echo"},
                                   {"content-type", "application/grpc"},
                                   {"custom-key", "custom-value"},
                                   {"authorization", "secret"},
                                   {"x-bin", std::string("\x00\xff\x80 z", 5)}};
    for (int round = 0; round < 3; ++round) {  // later rounds hit the dynamic table
        Buf block;
        for (auto& h : hs) enc.Encode(&block, h, h.name == "authorization" ? HPackIndexPolicy::NEVER_INDEXED
                                                                              : HPackIndexPolicy::INCREMENTAL);
        std::vector<HPackHeader> out;
        ASSERT_TRUE(dec.Decode(block.to_string(), &out));
        ASSERT_EQ(out.size(), hs.size());
        for (size_t i = 0; i < hs.size(); ++i) {
            EXPECT_EQ(out[i].name, hs[i].name);
            EXPECT_EQ(out[i].value, hs[i].value);
        }
    }
    std::string h;
    hpack::HuffmanEncode(&h, "www.example.com");
    std::string hex;
    for (unsigned char c : h) {
        char b[3];
        snprintf(b, 3, "%02x", c);
        hex += b;
    }
    EXPECT_EQ(hex, "f1e3c2e5f23a6ba0ab90f4ff");  // RFC 7541 C.4.1
    std::string back;
    ASSERT_TRUE(hpack::HuffmanDecode((const uint8_t*)h.data(), h.size(), &back));
    EXPECT_EQ(back, "www.example.com");
    for (int c = 0; c < 256; ++c) {
        std::string s(3, (char)c), e, d;
        hpack::HuffmanEncode(&e, s);
        ASSERT_TRUE(hpack::HuffmanDecode((const uint8_t*)e.data(), e.size(), &d));
        ASSERT_EQ(d, s);
    }
}

TEST(H2, json_and_grpc) {
    HttpServer s;
    ASSERT_GT(s.port, 0);
    for (const char* proto : {"h2", "h2:grpc"}) {
        Channel ch;
        ChannelOptions opt;
        opt.protocol = proto;
        opt.timeout_ms = 3000;
        ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
        example::EchoService_Stub stub(&ch);
        // concurrent calls multiplexed on one connection
        std::vector<std::thread> ths;
        std::atomic<int> ok{0};
        for (int t = 0; t < 4; ++t) {
            ths.emplace_back([&, t] {
                for (int i = 0; i < 50; ++i) {
                    Controller cntl;
                    example::EchoRequest req;
                    example::EchoResponse res;
                    req.set_message(std::string(proto) + " " + std::to_string(t * 1000 + i) +
                                    std::string(i == 7 ? 100000 : 0, 'z'));
                    stub.Echo(&cntl, &req, &res, nullptr);
                    if (!cntl.Failed() && res.message() == req.message()) ok.fetch_add(1);
                    else fprintf(stderr, "%s failed (i=%d, %zu bytes): %s\n", proto, i, req.message().size(),
                                 cntl.ErrorText().c_str());
                }
            });
        }
        for (auto& th : ths) th.join();
        EXPECT_EQ(ok.load(), 200);
        // server error maps through grpc-status / http status
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("x");
        req.set_server_fail(true);
        stub.Echo(&cntl, &req, &res, nullptr);
        EXPECT_TRUE(cntl.Failed());
    }
    // plain h2 GET of a builtin page
    Channel ch;
    ChannelOptions opt;
    opt.protocol = "h2";
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    Controller cntl;
    cntl.http_request().uri().set_path("/health");
    ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    ASSERT_FALSE(cntl.Failed());
    EXPECT_EQ(cntl.response_attachment().to_string(), "OK\n");
}

// Attachments over gRPC (policy/h2_protocol.cc kSettingsMrpcDevice): the
// reference refuses them (http_rpc_protocol.cpp:511); between brpc_amd peers
// that announced the private SETTINGS parameter they travel in-band (host
// bytes after the message, sized by the mrpc-meta-bin header) or lent (device
// blocks, GPU tests). Without the announcement nothing of it is on the wire.
DECLARE_bool(h2_mrpc_extensions);

TEST(H2, grpc_attachment_needs_an_mrpc_peer) {
    HttpServer s;
    ASSERT_GT(s.port, 0);
    Channel ch;
    ChannelOptions opt;
    opt.protocol = "h2:grpc";
    opt.timeout_ms = 3000;
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("with attachment");
    cntl.request_attachment().append("tail bytes");
    stub.Echo(&cntl, &req, &res, nullptr);
    ASSERT_TRUE(cntl.Failed());
    EXPECT_EQ(cntl.ErrorCode(), EREQUEST);
    EXPECT_NE(cntl.ErrorText().find("request_attachment must be empty"), std::string::npos);
    // the same channel still serves plain gRPC calls
    Controller c2;
    example::EchoResponse r2;
    stub.Echo(&c2, &req, &r2, nullptr);
    ASSERT_TRUE_M(!c2.Failed(), c2.ErrorText());
    EXPECT_EQ(r2.message(), "with attachment");
}

TEST(H2, grpc_attachments_between_mrpc_peers) {
    FLAGS_h2_mrpc_extensions = true;
    {
        HttpServer s;
        ASSERT_GT(s.port, 0);
        Channel ch;
        ChannelOptions opt;
        opt.protocol = "h2:grpc";
        opt.timeout_ms = 3000;
        ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
        example::EchoService_Stub stub(&ch);
        for (int i = 0; i < 40; ++i) {
            Controller cntl;
            example::EchoRequest req;
            example::EchoResponse res;
            req.set_message("m" + std::to_string(i));
            // 0, small and multi-frame attachments (> the 16 KiB frame size)
            const std::string att = i % 4 == 0 ? "" : std::string((size_t)(i % 4 == 3 ? 100000 : 37 * i), (char)('a' + i % 26));
            cntl.request_attachment().append(att);
            if (i % 5 == 1) cntl.set_request_compress_type(COMPRESS_TYPE_GZIP);  // the message compressed, not the attachment
            stub.Echo(&cntl, &req, &res, nullptr);
            ASSERT_TRUE_M(!cntl.Failed(), std::to_string(i) + ": " + cntl.ErrorText());
            EXPECT_EQ(res.message(), req.message());
            EXPECT_TRUE_M(cntl.response_attachment().to_string() == att, std::to_string(i));
        }
    }
    FLAGS_h2_mrpc_extensions = false;
}

TEST(H2, mrpc_settings_parameter_only_when_announced) {
    // a raw client reads the server's SETTINGS: 4 parameters by default
    // (grpcio peers see the frames they always saw), 5 with the extensions
    for (bool on : {false, true}) {
        FLAGS_h2_mrpc_extensions = on;
        HttpServer s;
        ASSERT_GT(s.port, 0);
        const int fd = socket(AF_INET, SOCK_STREAM, 0);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_port = htons((uint16_t)s.port);
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        ASSERT_EQ(connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)), 0);
        const std::string hello = std::string("PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n", 24) + std::string("\0\0\0\x04\0\0\0\0\0", 9);
        ASSERT_EQ(write(fd, hello.data(), hello.size()), (ssize_t)hello.size());
        std::string in;
        bool found = false;
        uint32_t settings_len = 0;
        for (int tries = 0; tries < 100 && !found; ++tries) {
            pollfd p{fd, POLLIN, 0};
            if (poll(&p, 1, 100) <= 0) continue;
            char buf[4096];
            const ssize_t n = read(fd, buf, sizeof(buf));
            if (n <= 0) break;
            in.append(buf, (size_t)n);
            for (size_t off = 0; off + 9 <= in.size();) {
                const uint32_t len = ((uint32_t)(uint8_t)in[off] << 16) | ((uint32_t)(uint8_t)in[off + 1] << 8) |
                                     (uint8_t)in[off + 2];
                if (off + 9 + len > in.size()) break;
                if (in[off + 3] == 4 && (in[off + 4] & 1) == 0) {
                    settings_len = len;
                    found = true;
                    bool has = false;
                    for (uint32_t k = 0; k + 6 <= len; k += 6) {
                        const uint16_t id = (uint16_t)(((uint8_t)in[off + 9 + k] << 8) | (uint8_t)in[off + 10 + k]);
                        has |= id == 0xF0A5;
                    }
                    EXPECT_EQ(has, on);
                }
                off += 9 + len;
            }
        }
        close(fd);
        ASSERT_TRUE(found);
        EXPECT_EQ(settings_len, on ? 30u : 24u);
    }
    FLAGS_h2_mrpc_extensions = false;
}
