// Legacy protocol family over loopback (spirit of the reference's
// test/brpc_hulu_pbrpc_protocol_unittest.cpp, brpc_sofa_pbrpc_protocol_unittest.cpp,
// brpc_nova_pbrpc_protocol_unittest.cpp, brpc_public_pbrpc_protocol_unittest.cpp,
// brpc_esp_protocol_unittest.cpp, brpc_mongo_protocol_unittest.cpp and the
// mcpack2pb tests): every client protocol is exercised against a server
// speaking it, including attachments, compression, errors and pipelining
// of nshead-framed calls on one connection.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <thread>
#include <vector>

#include "base/endpoint.h"
#include "base/time.h"
#include "fiber/fiber.h"
#include "mcpack/mcpack.h"
#include "mrpc/proto/echo.pb.h"
#include "mrpc/proto/mongo.pb.h"
#include "mrpc/proto/test_services.pb.h"
#include "rpc/channel.h"
#include "rpc/errno.h"
#include "rpc/esp.h"
#include "rpc/mongo.h"
#include "rpc/nshead.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

struct LegacyServer {
    Server server;
    EchoServiceImpl echo;
    int port = 0;
    explicit LegacyServer(NsheadService* ns = nullptr, MongoServiceAdaptor* mongo = nullptr, Service* extra = nullptr) {
        server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        if (extra) server.AddService(extra, SERVER_DOESNT_OWN_SERVICE);
        ServerOptions o;
        o.has_builtin_services = false;
        o.nshead_service = ns;
        o.mongo_service_adaptor = mongo;
        if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
    }
    std::string addr() const { return "127.0.0.1:" + std::to_string(port); }
};

void EchoOver(const std::string& addr, const std::string& protocol, CompressType ct, bool with_attachment,
              int n = 20) {
    Channel ch;
    ChannelOptions opt;
    opt.protocol = protocol;
    opt.timeout_ms = 3000;
    ASSERT_EQ(ch.Init(addr.c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    for (int i = 0; i < n; ++i) {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message(protocol + " #" + std::to_string(i) + std::string(i * 50, 'z'));
        cntl.set_request_compress_type(ct);
        if (with_attachment) cntl.request_attachment().append("att-" + std::to_string(i));
        stub.Echo(&cntl, &req, &res, nullptr);
        if (cntl.Failed()) fprintf(stderr, "%s call %d: %s\n", protocol.c_str(), i, cntl.ErrorText().c_str());
        ASSERT_FALSE(cntl.Failed());
        EXPECT_EQ(res.message(), req.message());
        if (with_attachment) EXPECT_EQ(cntl.response_attachment().to_string(), "att-" + std::to_string(i));
    }
}

}  // namespace

TEST(Legacy, hulu_echo_attachment_and_compression) {
    LegacyServer s;
    ASSERT_GT(s.port, 0);
    EchoOver(s.addr(), "hulu_pbrpc", COMPRESS_TYPE_NONE, true);
    EchoOver(s.addr(), "hulu_pbrpc", COMPRESS_TYPE_SNAPPY, true);
    EchoOver(s.addr(), "hulu_pbrpc", COMPRESS_TYPE_GZIP, false);
    EchoOver(s.addr(), "hulu_pbrpc", COMPRESS_TYPE_ZLIB, true);
}

TEST(Legacy, sofa_echo_and_compression) {
    LegacyServer s;
    EchoOver(s.addr(), "sofa_pbrpc", COMPRESS_TYPE_NONE, false);
    EchoOver(s.addr(), "sofa_pbrpc", COMPRESS_TYPE_SNAPPY, false);
    EchoOver(s.addr(), "sofa_pbrpc", COMPRESS_TYPE_GZIP, false);
}

TEST(Legacy, sofa_rejects_attachment_and_unknown_method) {
    LegacyServer s;
    Channel ch;
    ChannelOptions opt;
    opt.protocol = "sofa_pbrpc";
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("x");
    cntl.request_attachment().append("nope");
    stub.Echo(&cntl, &req, &res, nullptr);
    EXPECT_TRUE(cntl.Failed());
    EXPECT_EQ(cntl.ErrorCode(), (int)EREQUEST);
}

TEST(Legacy, hulu_unknown_service_reports_error) {
    // A server without EchoService: the hulu error meta carries ENOSERVICE.
    Server server;
    ServerOptions o;
    o.has_builtin_services = false;
    ASSERT_EQ(server.Start("127.0.0.1:0", &o), 0);
    Channel ch;
    ChannelOptions opt;
    opt.protocol = "hulu_pbrpc";
    opt.max_retry = 0;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("x");
    stub.Echo(&cntl, &req, &res, nullptr);
    EXPECT_TRUE(cntl.Failed());
    EXPECT_EQ(cntl.ErrorCode(), (int)ENOSERVICE);
}

TEST(Legacy, nova_pbrpc_via_adaptor) {
    NovaServiceAdaptor nova;
    LegacyServer s(&nova);
    EchoOver(s.addr(), "nova_pbrpc", COMPRESS_TYPE_NONE, false);
    EchoOver(s.addr(), "nova_pbrpc", COMPRESS_TYPE_SNAPPY, false);
}

TEST(Legacy, public_pbrpc_via_adaptor) {
    PublicPbrpcServiceAdaptor pub;
    LegacyServer s(&pub);
    EchoOver(s.addr(), "public_pbrpc", COMPRESS_TYPE_NONE, false);
    EchoOver(s.addr(), "public_pbrpc", COMPRESS_TYPE_SNAPPY, false);
}

TEST(Legacy, nshead_mcpack_via_adaptor) {
    NsheadMcpackAdaptor mc("example.EchoService.Echo");
    LegacyServer s(&mc);
    EchoOver(s.addr(), "nshead_mcpack", COMPRESS_TYPE_NONE, false);
}

namespace {
// Raw nshead service: echoes the body reversed, tags the head.
class ReverseNshead : public NsheadService {
public:
    void ProcessNsheadRequest(const Server&, Controller*, const NsheadMessage& req, NsheadMessage* res,
                              NsheadClosure* done) override {
        std::string s = req.body.to_string();
        std::reverse(s.begin(), s.end());
        res->body.append(s);
        res->head.reserved = 77;
        done->Run();
    }
};
}  // namespace

TEST(Legacy, raw_nshead_pipelined_on_single_connection) {
    ReverseNshead svc;
    LegacyServer s(&svc);
    Channel ch;
    ChannelOptions opt;
    opt.protocol = "nshead";
    opt.timeout_ms = 3000;
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    const int N = 64;
    std::vector<std::unique_ptr<Controller>> cntls(N);
    std::vector<NsheadMessage> reqs(N), ress(N);
    std::atomic<int> done_n{0};
    for (int i = 0; i < N; ++i) {
        cntls[i].reset(new Controller);
        reqs[i].head.log_id = (uint32_t)i;
        reqs[i].body.append("payload-" + std::to_string(i));
        ch.CallMethod(nullptr, cntls[i].get(), &reqs[i], &ress[i], NewCallback([&done_n] { done_n.fetch_add(1); }));
    }
    for (int i = 0; i < N; ++i) cntls[i]->Join();
    // Join() returns once the call id is gone; an async done may still be
    // running (the reference destroys the id before done->Run as well).
    for (int spin = 0; spin < 2000 && done_n.load() != N; ++spin) usleep(1000);
    EXPECT_EQ(done_n.load(), N);
    for (int i = 0; i < N; ++i) {
        if (cntls[i]->Failed()) fprintf(stderr, "nshead call %d: %s\n", i, cntls[i]->ErrorText().c_str());
        ASSERT_FALSE(cntls[i]->Failed());
        std::string want = "payload-" + std::to_string(i);
        std::reverse(want.begin(), want.end());
        EXPECT_EQ(ress[i].body.to_string(), want);
        EXPECT_EQ(ress[i].head.log_id, (uint32_t)i);
        EXPECT_EQ(ress[i].head.reserved, 77u);
        EXPECT_EQ(ress[i].head.magic_num, NSHEAD_MAGICNUM);
    }
}

namespace {
// A ubrpc server built on NsheadService: decodes
// {content:[{id, method, params:{req:{...}}}]} and answers
// {content:[{id, result_params:{res:{...}}}]} (or error for method "Fail").
class FakeUbrpcServer : public NsheadService {
public:
    explicit FakeUbrpcServer(mcpack::Format f) : _fmt(f) {}
    void ProcessNsheadRequest(const Server&, Controller*, const NsheadMessage& req, NsheadMessage* res,
                              NsheadClosure* done) override {
        const std::string raw = req.body.to_string();
        std::string name;
        mcpack::Value top;
        std::vector<mcpack::Item> items, content, fields, params;
        int64_t id = -1;
        example::EchoRequest er;
        bool fail = false;
        if (mcpack::DecodeField(raw.data(), raw.size(), &name, &top) && mcpack::ListItems(top, &items)) {
            for (auto& it : items) {
                if (it.name != "content" || !mcpack::ListItems(it.value, &content) || content.empty()) continue;
                mcpack::ListItems(content[0].value, &fields);
                for (auto& f : fields) {
                    if (f.name == "id") f.value.to_int64(&id);
                    std::string m;
                    if (f.name == "method" && f.value.to_string(&m)) fail = (m != "Echo");
                    if (f.name == "params" && mcpack::ListItems(f.value, &params)) {
                        for (auto& p : params) {
                            if (p.name == "req") mcpack::ParseFromObject(p.value, &er);
                        }
                    }
                }
            }
        }
        std::string out;
        mcpack::Serializer sr(&out);
        sr.begin_object();
        sr.begin_array("content", mcpack::FIELD_OBJECT, _fmt);
        sr.begin_object();
        sr.add_int64("id", id);
        if (fail || er.message() == "fail") {
            sr.begin_object("error");
            sr.add_int32("code", 4321);
            sr.add_string("message", "asked to fail");
            sr.end_object();
        } else {
            sr.add_int64("result", 7);
            sr.begin_object("result_params");
            sr.begin_object("res");
            example::EchoResponse eres;
            eres.set_message(er.message());
            mcpack::SerializeFields(eres, _fmt, &sr);
            sr.end_object();
            sr.end_object();
        }
        sr.end_object();
        sr.end_array();
        sr.end_object();
        res->body.append(out);
        done->Run();
    }

private:
    mcpack::Format _fmt;
};
}  // namespace

TEST(Legacy, ubrpc_compack_and_mcpack2) {
    for (int k = 0; k < 2; ++k) {
        const mcpack::Format fmt = k ? mcpack::FORMAT_MCPACK_V2 : mcpack::FORMAT_COMPACK;
        FakeUbrpcServer svc(fmt);
        LegacyServer s(&svc);
        Channel ch;
        ChannelOptions opt;
        opt.protocol = k ? "ubrpc_mcpack2" : "ubrpc_compack";
        opt.timeout_ms = 3000;
        opt.max_retry = 0;
        ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
        example::EchoService_Stub stub(&ch);
        for (int i = 0; i < 10; ++i) {
            Controller cntl;
            example::EchoRequest req;
            example::EchoResponse res;
            req.set_message("ub-" + std::to_string(i));
            stub.Echo(&cntl, &req, &res, nullptr);
            ASSERT_FALSE(cntl.Failed());
            EXPECT_EQ(res.message(), req.message());
            EXPECT_EQ(cntl.idl_result(), 7);
        }
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("fail");
        stub.Echo(&cntl, &req, &res, nullptr);
        EXPECT_TRUE(cntl.Failed());
        EXPECT_EQ(cntl.ErrorCode(), 4321);
    }
}

namespace {
// Minimal blocking ESP peer: answers each request with the body uppercased.
struct EspPeer {
    std::atomic<bool> bad_preamble{false};
    int lfd = -1;
    int port = 0;
    std::thread th;
    EspPeer() {
        lfd = socket(AF_INET, SOCK_STREAM, 0);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        bind(lfd, (sockaddr*)&a, sizeof(a));
        listen(lfd, 4);
        socklen_t len = sizeof(a);
        getsockname(lfd, (sockaddr*)&a, &len);
        port = ntohs(a.sin_port);
        th = std::thread([this] {
            const int fd = accept(lfd, nullptr, nullptr);
            if (fd < 0) return;
            // the connection's preamble (EspAuthenticator): magic + port
            char pre[8];
            if (!read_full(fd, pre, sizeof(pre)) || memcmp(pre, "\0ESP\x01\x02", 6) != 0) {
                bad_preamble = true;
                close(fd);
                return;
            }
            for (;;) {
                EspHead h;
                if (!read_full(fd, &h, sizeof(h))) break;
                std::string body(h.body_len, '\0');
                if (!read_full(fd, &body[0], body.size())) break;
                for (char& c : body) c = (char)toupper(c);
                h.msg = 0;
                std::swap(h.from, h.to);
                if (write(fd, &h, sizeof(h)) != (ssize_t)sizeof(h)) break;
                if (write(fd, body.data(), body.size()) != (ssize_t)body.size()) break;
            }
            close(fd);
        });
    }
    static bool read_full(int fd, void* p, size_t n) {
        char* c = (char*)p;
        while (n) {
            const ssize_t r = read(fd, c, n);
            if (r <= 0) return false;
            c += r;
            n -= (size_t)r;
        }
        return true;
    }
    ~EspPeer() {
        shutdown(lfd, SHUT_RDWR);
        close(lfd);
        th.join();
    }
};
}  // namespace

TEST(Legacy, esp_client_pipelined) {
    EspPeer peer;
    Channel ch;
    ChannelOptions opt;
    opt.protocol = "esp";
    opt.timeout_ms = 3000;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(peer.port)).c_str(), &opt), 0);
    const int N = 16;
    std::vector<std::unique_ptr<Controller>> cntls(N);
    std::vector<EspMessage> reqs(N), ress(N);
    for (int i = 0; i < N; ++i) {
        cntls[i].reset(new Controller);
        reqs[i].head.msg_id = (uint64_t)i;
        reqs[i].head.to.port = 8000;
        reqs[i].body.append("esp body " + std::to_string(i));
        ch.CallMethod(nullptr, cntls[i].get(), &reqs[i], &ress[i], NewCallback([] {}));
    }
    for (int i = 0; i < N; ++i) {
        cntls[i]->Join();
        ASSERT_FALSE(cntls[i]->Failed());
        EXPECT_EQ(ress[i].body.to_string(), "ESP BODY " + std::to_string(i));
        EXPECT_EQ(ress[i].head.msg_id, (uint64_t)i);
        EXPECT_EQ(ress[i].head.from.port, 8000);
    }
    EXPECT_FALSE(peer.bad_preamble.load());
}

namespace {
class CountingMongoContext : public MongoContext {
public:
    int nreq = 0;
};
class TestMongoAdaptor : public MongoServiceAdaptor {
public:
    void SerializeError(int response_to, Buf* out) const override {
        mongo_head_t h{(int32_t)sizeof(mongo_head_t), 0, response_to, policy::OPREPLY};
        out->append(&h, sizeof(h));
    }
    MongoContext* CreateSocketContext() const override { return new CountingMongoContext; }
};
class TestMongoService : public policy::MongoService {
public:
    void default_method(RpcController* c, const policy::MongoRequest* req, policy::MongoResponse* res,
                        Closure* done) override {
        ClosureGuard g(done);
        Controller* cntl = static_cast<Controller*>(c);
        CountingMongoContext* ctx = static_cast<CountingMongoContext*>(cntl->mongo_session_data());
        const int n = ctx ? ++ctx->nreq : -1;
        res->mutable_header()->set_message_length(0);
        res->mutable_header()->set_request_id(1000 + n);
        res->mutable_header()->set_op_code(policy::OPREPLY);
        res->set_response_flags(0);
        res->set_cursor_id(0);
        res->set_starting_from(0);
        res->set_number_returned(n);
        res->set_message("reply:" + req->message());
    }
};
}  // namespace

TEST(Legacy, mongo_server_adaptor) {
    TestMongoAdaptor adaptor;
    TestMongoService svc;
    LegacyServer s(nullptr, &adaptor, &svc);
    ASSERT_GT(s.port, 0);
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)s.port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    ASSERT_EQ(connect(fd, (sockaddr*)&a, sizeof(a)), 0);
    for (int i = 1; i <= 3; ++i) {
        const std::string body = "query-" + std::to_string(i);
        mongo_head_t h{(int32_t)(sizeof(mongo_head_t) + body.size()), 40 + i, 0, policy::DB_QUERY};
        ASSERT_EQ(write(fd, &h, sizeof(h)), (ssize_t)sizeof(h));
        ASSERT_EQ(write(fd, body.data(), body.size()), (ssize_t)body.size());
        mongo_head_t rh;
        ASSERT_TRUE(EspPeer::read_full(fd, &rh, sizeof(rh)));
        EXPECT_EQ(rh.response_to, 40 + i);
        EXPECT_EQ(rh.op_code, (int32_t)policy::OPREPLY);
        std::string rest(rh.message_length - sizeof(rh), '\0');
        ASSERT_TRUE(EspPeer::read_full(fd, &rest[0], rest.size()));
        int32_t nret;
        memcpy(&nret, rest.data() + 16, 4);
        EXPECT_EQ(nret, i);  // per-connection context counted the requests
        EXPECT_EQ(rest.substr(20), "reply:" + body);
    }
    close(fd);
}

TEST(Mcpack, roundtrip_both_formats) {
    for (int k = 0; k < 2; ++k) {
        const mcpack::Format fmt = k ? mcpack::FORMAT_MCPACK_V2 : mcpack::FORMAT_COMPACK;
        test::Rich r;
        r.set_i32(-5);
        r.set_i64(-1234567890123LL);
        r.set_u64(18000000000000000000ULL);
        r.set_d(3.25);
        r.set_flag(true);
        r.set_s(std::string(300, 's'));  // long string head
        r.set_raw(std::string("\0\1\2", 3));
        r.set_color(test::BLUE);
        r.mutable_inner()->set_x(9);
        r.mutable_inner()->add_tags("a");
        r.mutable_inner()->add_tags("bb");
        for (int i = 0; i < 3; ++i) r.add_inners()->set_x(i);
        for (int i = 0; i < 5; ++i) r.add_nums(i * i);
        r.set_must("m");
        std::string out;
        ASSERT_TRUE(mcpack::SerializeToString(r, fmt, &out));
        test::Rich back;
        ASSERT_TRUE(mcpack::ParseFromArray(out.data(), out.size(), &back));
        EXPECT_EQ(back.i32(), -5);
        EXPECT_EQ(back.i64(), -1234567890123LL);
        EXPECT_EQ(back.u64(), 18000000000000000000ULL);
        EXPECT_EQ(back.d(), 3.25);
        EXPECT_TRUE(back.flag());
        EXPECT_EQ(back.s(), r.s());
        EXPECT_EQ(back.raw(), r.raw());
        EXPECT_EQ((int)back.color(), (int)test::BLUE);
        EXPECT_EQ(back.inner().x(), 9);
        EXPECT_EQ(back.inner().tags_size(), 2);
        EXPECT_EQ(back.inners_size(), 3);
        EXPECT_EQ(back.inners(2).x(), 2);
        ASSERT_EQ(back.nums_size(), 5);
        EXPECT_EQ(back.nums(4), 16);
        EXPECT_EQ(back.must(), "m");
        // compack stores repeated primitives as an isomorphic array
        std::string name;
        mcpack::Value top;
        std::vector<mcpack::Item> items;
        ASSERT_TRUE(mcpack::DecodeField(out.data(), out.size(), &name, &top) > 0);
        ASSERT_TRUE(mcpack::ListItems(top, &items));
        for (auto& it : items) {
            if (it.name == "nums") EXPECT_EQ((int)it.value.type(), (int)(k ? mcpack::FIELD_ARRAY : mcpack::FIELD_ISOARRAY));
        }
    }
}

TEST(Mcpack, object_isoarray_and_lenient_numbers) {
    // {inners: object_isoarray {x:[1,2,3]}, i32: int8(7), d: int32(2)}
    std::string out;
    mcpack::Serializer sr(&out);
    sr.begin_object();
    sr.add_int8("i32", 7);
    sr.add_int32("d", 2);
    sr.add_string("must", "q");
    sr.add_null("s");
    sr.end_object();
    ASSERT_TRUE(sr.good());
    // Splice an OBJECTISOARRAY field by hand: long head(0x40), name, count, one array column.
    std::string col;
    mcpack::Serializer csr(&col);
    csr.begin_object();
    csr.begin_array("x", mcpack::FIELD_INT32, mcpack::FORMAT_COMPACK);
    for (int i = 1; i <= 3; ++i) csr.add_int32("", i);
    csr.end_array();
    csr.end_object();
    // col = [long head of anonymous object][count=1][x isoarray]; rename type to 0x40 and name it "inners".
    std::string field;
    field.push_back((char)mcpack::FIELD_OBJECTISOARRAY);
    field.push_back((char)7);
    const uint32_t vsize = (uint32_t)(col.size() - 6);
    field.append((const char*)&vsize, 4);
    field.append("inners", 7);
    field.append(col.substr(6));
    // append as a 5th item of the top object
    std::string top = out;
    uint32_t cnt;
    memcpy(&cnt, &top[6], 4);
    ++cnt;
    memcpy(&top[6], &cnt, 4);
    top += field;
    const uint32_t tsize = (uint32_t)(top.size() - 6);
    memcpy(&top[2], &tsize, 4);
    test::Rich r;
    ASSERT_TRUE(mcpack::ParseFromArray(top.data(), top.size(), &r));
    EXPECT_EQ(r.i32(), 7);
    EXPECT_EQ(r.d(), 2.0);
    EXPECT_FALSE(r.has_s());
    ASSERT_EQ(r.inners_size(), 3);
    EXPECT_EQ(r.inners(1).x(), 2);
}

// ---------------------------------------------------------------- thrift
#include "thrift/thrift.h"

namespace {
// add(1: i32 a, 2: i32 b) -> i32 ; echo(1: string s) -> string ; boom() -> exception
class CalcThrift : public ThriftService {
public:
    void ProcessThriftFramedRequest(Controller* cntl, ThriftFramedMessage* req, ThriftFramedMessage* res,
                                    Closure* done) override {
        ClosureGuard g(done);
        if (req->method_name == "add") {
            const thrift::Value* a = req->body.find(1);
            const thrift::Value* b = req->body.find(2);
            res->body.field(0) = thrift::Value::I32((int32_t)((a ? a->as_int() : 0) + (b ? b->as_int() : 0)));
        } else if (req->method_name == "echo") {
            const thrift::Value* s = req->body.find(1);
            res->body.field(0) = s ? *s : thrift::Value::String("");
        } else {
            cntl->SetFailed(ENOMETHOD, "no method %s", req->method_name.c_str());
        }
    }
};
}  // namespace

TEST(Thrift, binary_protocol_wire_format) {
    // CALL "ping" seqid=7 {1: i32 5}: bytes fixed by the TBinaryProtocol spec.
    thrift::MessageHeader h;
    h.name = "ping";
    h.type = thrift::T_CALL;
    h.seqid = 7;
    thrift::Value args = thrift::Value::Struct();
    args.field(1) = thrift::Value::I32(5);
    std::string out;
    thrift::WriteMessage(&out, h, args);
    const unsigned char want[] = {0x80, 0x01, 0x00, 0x01, 0, 0, 0, 4, 'p', 'i', 'n', 'g', 0, 0, 0, 7,
                                  0x08, 0x00, 0x01, 0, 0, 0, 5, 0x00};
    ASSERT_EQ(out.size(), sizeof(want));
    EXPECT_EQ(memcmp(out.data(), want, sizeof(want)), 0);
    // nested containers round trip
    thrift::Value v = thrift::Value::Struct();
    thrift::Value l = thrift::Value::List(thrift::T_STRING);
    l.elems().push_back(thrift::Value::String("a"));
    l.elems().push_back(thrift::Value::String("bc"));
    thrift::Value mp = thrift::Value::Map(thrift::T_I64, thrift::T_DOUBLE);
    mp.pairs().emplace_back(thrift::Value::I64(-3), thrift::Value::Double(2.5));
    v.field(1) = l;
    v.field(2) = mp;
    v.field(3) = thrift::Value::Bool(true);
    v.field(-4) = thrift::Value::I16(-9);
    std::string enc;
    thrift::WriteValue(&enc, v);
    thrift::Value back;
    ASSERT_EQ(thrift::ReadValue(enc.data(), enc.size(), thrift::T_STRUCT, &back), enc.size());
    EXPECT_TRUE(back == v);
    EXPECT_EQ(thrift::ReadValue(enc.data(), enc.size() - 1, thrift::T_STRUCT, &back), (size_t)0);
}

TEST(Thrift, framed_client_server_pipelined) {
    CalcThrift calc;
    Server server;
    ServerOptions o;
    o.has_builtin_services = false;
    o.thrift_service = &calc;
    ASSERT_EQ(server.Start("127.0.0.1:0", &o), 0);
    Channel ch;
    ChannelOptions opt;
    opt.protocol = "thrift";
    opt.timeout_ms = 3000;
    opt.max_retry = 0;
    ASSERT_EQ(ch.Init(("127.0.0.1:" + std::to_string(server.listen_port())).c_str(), &opt), 0);
    const int N = 32;
    std::vector<std::unique_ptr<Controller>> cntls(N);
    std::vector<ThriftFramedMessage> reqs(N), ress(N);
    for (int i = 0; i < N; ++i) {
        cntls[i].reset(new Controller);
        reqs[i].method_name = "add";
        reqs[i].body.field(1) = thrift::Value::I32(i);
        reqs[i].body.field(2) = thrift::Value::I32(1000);
        ch.CallMethod(nullptr, cntls[i].get(), &reqs[i], &ress[i], NewCallback([] {}));
    }
    for (int i = 0; i < N; ++i) {
        cntls[i]->Join();
        if (cntls[i]->Failed()) fprintf(stderr, "thrift %d: %s\n", i, cntls[i]->ErrorText().c_str());
        ASSERT_FALSE(cntls[i]->Failed());
        ASSERT_TRUE(ress[i].success() != nullptr);
        EXPECT_EQ(ress[i].success()->as_int(), 1000 + i);
    }
    Controller c2;
    ThriftFramedMessage r2, s2;
    r2.method_name = "echo";
    r2.body.field(1) = thrift::Value::String(std::string(100000, 'e'));
    ch.CallMethod(nullptr, &c2, &r2, &s2, nullptr);
    ASSERT_FALSE(c2.Failed());
    EXPECT_EQ(s2.success()->as_string().size(), 100000u);
    Controller c3;
    ThriftFramedMessage r3, s3;
    r3.method_name = "nope";
    ch.CallMethod(nullptr, &c3, &r3, &s3, nullptr);
    EXPECT_TRUE(c3.Failed());
    EXPECT_TRUE(c3.ErrorText().find("no method nope") != std::string::npos);
}

// Generated per-message codecs (mrpc_protoc --mcpack_out, the role of the
// reference's protoc-gen-mcpack) against the descriptor walk: same bytes
// both ways, and each path parses the other's output.
namespace {
test::Rich MakeRich() {
    test::Rich r;
    r.set_i32(-5);
    r.set_i64(-1234567890123LL);
    r.set_u64(18000000000000000000ULL);
    r.set_d(3.25);
    r.set_flag(true);
    r.set_s(std::string(300, 's'));
    r.set_raw(std::string("\0\1\2", 3));
    r.set_color(test::BLUE);
    r.mutable_inner()->set_x(9);
    r.mutable_inner()->add_tags("a");
    r.mutable_inner()->add_tags("bb");
    for (int i = 0; i < 3; ++i) r.add_inners()->set_x(i);
    for (int i = 0; i < 5; ++i) r.add_nums(i * i);
    r.set_must("m");
    return r;
}
test::IdlTyped MakeIdl() {
    test::IdlTyped t;
    t.set_small(-7);
    t.set_big(4000000000ULL);
    t.set_blob(std::string("\0bin", 4));
    t.add_fs(1.5f);
    t.add_fs(-2.25f);
    t.set_b(true);
    t.add_colors(test::GREEN);
    t.add_colors(test::BLUE);
    t.add_inners()->set_x(11);
    t.set_ratio(41.9);
    return t;
}
}  // namespace

TEST(Mcpack, generated_codec_matches_reflection) {
    ASSERT_TRUE(mcpack::FindMessageHandler(test::Rich::descriptor()) != nullptr);
    ASSERT_TRUE(mcpack::FindMessageHandler(test::IdlTyped::descriptor()) != nullptr);
    ASSERT_TRUE(mcpack::FindMessageHandler(example::EchoRequest::descriptor()) != nullptr);
    const test::Rich r = MakeRich();
    const test::IdlTyped t = MakeIdl();
    for (int k = 0; k < 2; ++k) {
        const mcpack::Format fmt = k ? mcpack::FORMAT_MCPACK_V2 : mcpack::FORMAT_COMPACK;
        std::string gen_r, ref_r, gen_t, ref_t;
        ASSERT_TRUE(mcpack::SerializeToString(r, fmt, &gen_r));
        ASSERT_TRUE(mcpack::SerializeToString(t, fmt, &gen_t));
        mcpack::SetGeneratedHandlersEnabled(false);
        ASSERT_TRUE(mcpack::SerializeToString(r, fmt, &ref_r));
        ASSERT_TRUE(mcpack::SerializeToString(t, fmt, &ref_t));
        // reflective parse of the generated bytes
        test::Rich r_ref;
        test::IdlTyped t_ref;
        ASSERT_TRUE(mcpack::ParseFromArray(gen_r.data(), gen_r.size(), &r_ref));
        ASSERT_TRUE(mcpack::ParseFromArray(gen_t.data(), gen_t.size(), &t_ref));
        mcpack::SetGeneratedHandlersEnabled(true);
        EXPECT_TRUE(gen_r == ref_r);
        EXPECT_TRUE(gen_t == ref_t);
        // generated parse of the reflective bytes
        test::Rich r_gen;
        test::IdlTyped t_gen;
        ASSERT_TRUE(mcpack::ParseFromArray(ref_r.data(), ref_r.size(), &r_gen));
        ASSERT_TRUE(mcpack::ParseFromArray(ref_t.data(), ref_t.size(), &t_gen));
        EXPECT_EQ(r_gen.SerializeAsString(), r.SerializeAsString());
        EXPECT_EQ(r_ref.SerializeAsString(), r.SerializeAsString());
        EXPECT_EQ(t_gen.SerializeAsString(), t_ref.SerializeAsString());
        // idl_type conversions: int8 wire for `small`, uint32 for `big`
        // (truncated), double for floats, int32 for the double `ratio`
        EXPECT_EQ(t_gen.small(), -7);
        EXPECT_EQ(t_gen.big(), (uint64_t)(uint32_t)4000000000ULL);
        EXPECT_EQ(t_gen.blob(), std::string("\0bin", 4));
        ASSERT_EQ(t_gen.fs_size(), 2);
        EXPECT_EQ(t_gen.fs(1), -2.25f);
        EXPECT_EQ(t_gen.colors(1), test::BLUE);
        ASSERT_EQ(t_gen.inners_size(), 1);
        EXPECT_EQ(t_gen.inners(0).x(), 11);
        EXPECT_EQ(t_gen.ratio(), 41.0);
        // idl_name renames the wire field
        std::string name;
        mcpack::Value top;
        std::vector<mcpack::Item> items;
        ASSERT_TRUE(mcpack::DecodeField(gen_t.data(), gen_t.size(), &name, &top) > 0);
        ASSERT_TRUE(mcpack::ListItems(top, &items));
        bool saw_big = false, saw_rows = false;
        for (auto& it : items) {
            if (it.name == "BigOne") saw_big = it.value.type() == mcpack::FIELD_UINT32;
            if (it.name == "rows") saw_rows = true;
            if (it.name == "small") EXPECT_EQ((int)it.value.type(), (int)mcpack::FIELD_INT8);
        }
        EXPECT_TRUE(saw_big && saw_rows);
    }
}

TEST(Mcpack, generated_codec_is_faster) {
    const test::Rich r = MakeRich();
    std::string out;
    auto run = [&](bool gen) {
        mcpack::SetGeneratedHandlersEnabled(gen);
        const int64_t t0 = monotonic_us();
        for (int i = 0; i < 20000; ++i) {
            mcpack::SerializeToString(r, mcpack::FORMAT_MCPACK_V2, &out);
            test::Rich back;
            mcpack::ParseFromArray(out.data(), out.size(), &back);
        }
        return monotonic_us() - t0;
    };
    run(true);
    const int64_t ref = run(false), gen = run(true);
    mcpack::SetGeneratedHandlersEnabled(true);
    printf("  mcpack serialize+parse x20000: reflection %lld us, generated %lld us (%.2fx)\n", (long long)ref,
           (long long)gen, (double)ref / std::max<int64_t>(1, gen));
    EXPECT_GT(ref, 0);
}
