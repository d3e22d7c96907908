// HTTP/1.1 and h2 protocol behaviour at the RPC level, in the spirit of the
// reference's test/brpc_http_rpc_protocol_unittest.cpp: server-side parsing
// of raw (pipelined, chunked, malformed, HTTP/1.0, Connection: close)
// requests written straight to a socket, client-side handling of scripted
// responses from a fake server (chunked, broken chunks, EOF-delimited,
// error statuses, progressive reads after the controller is gone, a socket
// that breaks mid-body), and h2 flow control / GOAWAY / error mapping.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "base/flags.h"
#include "base/time.h"
#include "http/http_header.h"
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

class PushImpl : public test::HttpTest {
public:
    void Push(RpcController* c, const test::Empty*, test::Empty*, Closure* done) override {
        Controller* cntl = static_cast<Controller*>(c);
        auto pa = cntl->CreateProgressiveAttachment();
        done->Run();
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
        for (const char* h : {"x-custom", "x-other"}) {
            if (const std::string* v = cntl->http_request().GetHeader(h)) cntl->http_response().SetHeader(h, *v);
        }
        cntl->http_response().SetHeader("x-path", cntl->http_request().uri().path());
        cntl->http_response().SetHeader("x-unresolved", cntl->http_request().unresolved_path());
        cntl->response_attachment().append(cntl->request_attachment());
        if (const std::string* code = cntl->http_request().uri().GetQuery("status")) {
            cntl->http_response().set_status_code(atoi(code->c_str()));
        }
    }
    void Rich(RpcController*, const test::Rich* req, test::Rich* res, Closure* done) override {
        ClosureGuard g(done);
        *res = *req;
        res->set_i32(req->i32() + 1);
    }
};

struct Srv {
    Server server;
    EchoServiceImpl echo;
    PushImpl t;
    int port = 0;
    explicit Srv(const ServerOptions* opt = nullptr) {
        server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        server.AddService(&t, SERVER_DOESNT_OWN_SERVICE, "/v1/raw/* => Raw");
        ServerOptions o;
        if (opt) o = *opt;
        if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
    }
    std::string addr() const { return "127.0.0.1:" + std::to_string(port); }
};

int connect_to(int port) {
    const int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (connect(fd, (sockaddr*)&a, sizeof(a)) != 0) {
        close(fd);
        return -1;
    }
    return fd;
}

void write_all(int fd, const std::string& s) {
    size_t off = 0;
    while (off < s.size()) {
        const ssize_t n = write(fd, s.data() + off, s.size() - off);
        if (n <= 0) return;
        off += (size_t)n;
    }
}

// Reads until `pred(buffer)` holds, EOF, or the timeout. Returns the bytes;
// *eof tells whether the peer closed.
std::string read_until(int fd, const std::function<bool(const std::string&)>& pred, int timeout_ms,
                       bool* eof = nullptr) {
    std::string got;
    const int64_t deadline = monotonic_us() + (int64_t)timeout_ms * 1000;
    if (eof) *eof = false;
    while (!pred(got)) {
        const int64_t left = (deadline - monotonic_us()) / 1000;
        if (left <= 0) break;
        pollfd p{fd, POLLIN, 0};
        if (poll(&p, 1, (int)left) <= 0) continue;
        char buf[65536];
        const ssize_t n = read(fd, buf, sizeof(buf));
        if (n <= 0) {
            if (eof) *eof = true;
            break;
        }
        got.append(buf, (size_t)n);
    }
    return got;
}

size_t count(const std::string& s, const std::string& needle) {
    size_t n = 0;
    for (size_t p = s.find(needle); p != std::string::npos; p = s.find(needle, p + 1)) ++n;
    return n;
}

// A one-connection fake HTTP server: reads one request head, then runs the
// script with the connected fd (write what you want, close or not).
struct FakeServer {
    int lfd = -1, port = 0;
    std::thread th;
    std::atomic<int> requests{0};
    explicit FakeServer(std::function<void(int fd)> script, int conns = 1) {
        lfd = socket(AF_INET, SOCK_STREAM, 0);
        int one = 1;
        setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        bind(lfd, (sockaddr*)&a, sizeof(a));
        socklen_t len = sizeof(a);
        getsockname(lfd, (sockaddr*)&a, &len);
        port = ntohs(a.sin_port);
        listen(lfd, 8);
        th = std::thread([this, script, conns] {
            for (int c = 0; c < conns; ++c) {
                pollfd p{lfd, POLLIN, 0};
                if (poll(&p, 1, 5000) <= 0) return;
                const int fd = accept(lfd, nullptr, nullptr);
                if (fd < 0) return;
                read_until(fd, [](const std::string& s) { return s.find("\r\n\r\n") != std::string::npos; }, 3000);
                requests.fetch_add(1);
                script(fd);
                close(fd);
            }
        });
    }
    ~FakeServer() {
        if (th.joinable()) th.join();
        close(lfd);
    }
    std::string addr() const { return "127.0.0.1:" + std::to_string(port); }
};

Channel* http_channel(const std::string& addr, int timeout_ms = 2000, const char* proto = "http") {
    Channel* ch = new Channel;
    ChannelOptions opt;
    opt.protocol = proto;
    opt.timeout_ms = timeout_ms;
    opt.max_retry = 0;
    if (ch->Init(addr.c_str(), &opt) != 0) {
        delete ch;
        return nullptr;
    }
    return ch;
}

struct CollectReader : public ProgressiveReader {
    std::string data;
    std::atomic<int> ended{0};
    std::atomic<int> parts{0};
    Status st;
    int stop_after = -1;  // OnReadOnePart fails after this many parts
    Status OnReadOnePart(const void* d, size_t n) override {
        data.append((const char*)d, n);
        if (stop_after >= 0 && parts.fetch_add(1) + 1 >= stop_after) return Status(ECANCELED, "enough");
        if (stop_after < 0) parts.fetch_add(1);
        return Status();
    }
    void OnEndOfMessage(const Status& s) override {
        st = s;
        ended.store(1);
    }
    bool wait(int ms) {
        for (int i = 0; i < ms / 5 && !ended.load(); ++i) usleep(5000);
        return ended.load() == 1;
    }
};

const char* kEchoJson = "{\"message\":\"hi\"}";

std::string post(const std::string& path, const std::string& body, const std::string& extra = "",
                 const char* version = "HTTP/1.1") {
    return "POST " + path + " " + version + "\r\nHost: t\r\nContent-Type: application/json\r\nContent-Length: " +
           std::to_string(body.size()) + "\r\n" + extra + "\r\n" + body;
}

}  // namespace

// ------------------------------------------------------------- addresses

TEST(HttpProtocol, channel_accepts_every_address_form) {
    Srv s;
    ASSERT_GT(s.port, 0);
    for (const std::string& a : {"http://" + s.addr(), s.addr(), "http://" + s.addr() + "/ignored/path",
                                 "localhost:" + std::to_string(s.port)}) {
        std::unique_ptr<Channel> ch(http_channel(a));
        ASSERT_TRUE(ch != nullptr);
        Controller cntl;
        cntl.http_request().uri().set_path("/health");
        ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        EXPECT_FALSE(cntl.Failed());
        EXPECT_EQ(cntl.response_attachment().to_string(), "OK\n");
    }
    Channel bad;
    ChannelOptions opt;
    opt.protocol = "http";
    EXPECT_NE(bad.Init("http://", &opt), 0);
}

// ------------------------------------------------------------- server side

TEST(HttpProtocol, pipelined_requests_are_answered_in_order) {
    Srv s;
    const int fd = connect_to(s.port);
    ASSERT_GE(fd, 0);
    std::string reqs;
    for (int i = 0; i < 3; ++i) {
        // the first is the slowest: answered in request order anyway
        reqs += post("/EchoService/Echo", "{\"message\":\"m" + std::to_string(i) + "\",\"sleep_us\":" +
                                              std::to_string((2 - i) * 30000) + "}");
    }
    write_all(fd, reqs);
    const std::string got =
        read_until(fd, [](const std::string& s) { return count(s, "HTTP/1.1 200") == 3 && s.find("\"m2\"") != std::string::npos; },
                   3000);
    close(fd);
    EXPECT_EQ(count(got, "HTTP/1.1 200"), 3u);
    const size_t a = got.find("\"m0\""), b = got.find("\"m1\""), c = got.find("\"m2\"");
    ASSERT_TRUE(a != std::string::npos && b != std::string::npos && c != std::string::npos);
    EXPECT_TRUE(a < b && b < c);
}

TEST(HttpProtocol, chunked_upload_is_reassembled) {
    Srv s;
    const int fd = connect_to(s.port);
    ASSERT_GE(fd, 0);
    const std::string body = "{\"message\":\"chunky body\"}";
    std::string req = "POST /EchoService/Echo HTTP/1.1\r\nHost: t\r\nContent-Type: application/json\r\n"
                      "Transfer-Encoding: chunked\r\n\r\n";
    for (size_t off = 0; off < body.size(); off += 7) {
        const std::string piece = body.substr(off, 7);
        char hex[16];
        snprintf(hex, sizeof(hex), "%zx", piece.size());
        req += std::string(hex) + "\r\n" + piece + "\r\n";
    }
    req += "0\r\n\r\n";
    // the chunks arrive in separate writes
    for (size_t off = 0; off < req.size(); off += 11) {
        write_all(fd, req.substr(off, 11));
        usleep(200);
    }
    const std::string got =
        read_until(fd, [](const std::string& s) { return s.find("chunky body") != std::string::npos; }, 3000);
    close(fd);
    EXPECT_TRUE(got.find("HTTP/1.1 200") != std::string::npos);
    EXPECT_TRUE(got.find("chunky body") != std::string::npos);
}

TEST(HttpProtocol, garbage_start_line_closes_the_connection) {
    Srv s;
    const int fd = connect_to(s.port);
    ASSERT_GE(fd, 0);
    write_all(fd, "GET /health HTTP/1.1\r\nHost: t\r\nContent-Length: zz\r\n\r\n");
    bool eof = false;
    const std::string got = read_until(fd, [](const std::string&) { return false; }, 2000, &eof);
    close(fd);
    EXPECT_TRUE(eof);
    EXPECT_TRUE(got.find("HTTP/1.1 200") == std::string::npos);
    // the server keeps serving others
    std::unique_ptr<Channel> ch(http_channel(s.addr()));
    Controller cntl;
    cntl.http_request().uri().set_path("/health");
    ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    EXPECT_FALSE(cntl.Failed());
}

TEST(HttpProtocol, get_without_body_to_a_pb_method_with_required_fields_is_rejected) {
    Srv s;
    const int fd = connect_to(s.port);
    ASSERT_GE(fd, 0);
    write_all(fd, "GET /EchoService/Echo HTTP/1.1\r\nHost: t\r\n\r\n");
    const std::string got =
        read_until(fd, [](const std::string& s) { return s.find("\r\n\r\n") != std::string::npos &&
                                                         s.find("required") != std::string::npos; },
                   2000);
    close(fd);
    EXPECT_TRUE(got.find("HTTP/1.1 400") != std::string::npos);
    EXPECT_TRUE(got.find("Missing required fields") != std::string::npos);
}

TEST(HttpProtocol, malformed_json_body_is_a_400_unknown_fields_are_not) {
    Srv s;
    std::unique_ptr<Channel> ch(http_channel(s.addr()));
    {
        Controller cntl;
        cntl.http_request().uri().set_path("/EchoService/Echo");
        cntl.http_request().set_method(HTTP_METHOD_POST);
        cntl.http_request().set_content_type("application/json");
        cntl.request_attachment().append("{\"message\": ");
        ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        ASSERT_TRUE(cntl.Failed());
        EXPECT_EQ(cntl.http_response().status_code(), 400);
        EXPECT_EQ(cntl.ErrorCode(), EREQUEST);
    }
    {
        Controller cntl;
        cntl.http_request().uri().set_path("/EchoService/Echo");
        cntl.http_request().set_method(HTTP_METHOD_POST);
        cntl.request_attachment().append("{\"message\":\"ok\",\"not_a_field\":[1,2]}");
        ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        EXPECT_FALSE(cntl.Failed());
        EXPECT_TRUE(cntl.response_attachment().to_string().find("\"ok\"") != std::string::npos);
    }
}

TEST(HttpProtocol, wrong_method_path_is_a_404_with_enomethod) {
    Srv s;
    std::unique_ptr<Channel> ch(http_channel(s.addr()));
    for (const char* path : {"/EchoService/NoSuchMethod", "/NoSuchService/Echo", "/a/b/c/d"}) {
        Controller cntl;
        cntl.http_request().uri().set_path(path);
        ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        ASSERT_TRUE(cntl.Failed());
        EXPECT_EQ(cntl.http_response().status_code(), 404);
        EXPECT_EQ(cntl.ErrorCode(), ENOMETHOD);
    }
}

TEST(HttpProtocol, proto_and_spring_protobuf_content_types) {
    Srv s;
    for (const char* ct : {"application/proto", "application/x-protobuf"}) {
        example::EchoRequest req;
        req.set_message(std::string("binary ") + ct);
        std::string bytes;
        ASSERT_TRUE(req.SerializeToString(&bytes));
        const int fd = connect_to(s.port);
        ASSERT_GE(fd, 0);
        write_all(fd, "POST /EchoService/Echo HTTP/1.1\r\nHost: t\r\nContent-Type: " + std::string(ct) +
                          "\r\nContent-Length: " + std::to_string(bytes.size()) + "\r\n\r\n" + bytes);
        const std::string got = read_until(
            fd, [&](const std::string& s) { return s.find(req.message()) != std::string::npos; }, 2000);
        close(fd);
        EXPECT_TRUE(got.find("HTTP/1.1 200") != std::string::npos);
        EXPECT_TRUE(got.find("Content-Type: application/proto") != std::string::npos ||
                    got.find("content-type: application/proto") != std::string::npos);
        const size_t body = got.find("\r\n\r\n");
        ASSERT_TRUE(body != std::string::npos);
        example::EchoResponse res;
        EXPECT_TRUE(res.ParseFromString(got.substr(body + 4)));
        EXPECT_EQ(res.message(), req.message());
    }
    // the client side: a proto content type makes the channel send pb bytes
    std::unique_ptr<Channel> ch(http_channel(s.addr()));
    example::EchoService_Stub stub(ch.get());
    Controller cntl;
    cntl.http_request().set_content_type("application/proto");
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("via stub");
    stub.Echo(&cntl, &req, &res, nullptr);
    ASSERT_FALSE(cntl.Failed());
    EXPECT_EQ(res.message(), "via stub");
}

TEST(HttpProtocol, service_errors_map_to_http_statuses_and_back) {
    Srv s;
    std::unique_ptr<Channel> ch(http_channel(s.addr()));
    example::EchoService_Stub stub(ch.get());
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("fail please");
    req.set_server_fail(true);
    stub.Echo(&cntl, &req, &res, nullptr);
    ASSERT_TRUE(cntl.Failed());
    EXPECT_GE(cntl.http_response().status_code(), 400);
    // the server's error code rides x-mrpc-error-code back to the client
    EXPECT_NE(cntl.ErrorCode(), EHTTP);
    EXPECT_TRUE(cntl.http_response().GetHeader("x-mrpc-error-code") != nullptr);
    // a plain status set by the handler is an EHTTP failure on the client
    Controller c2;
    c2.http_request().uri().SetHttpURL("/v1/raw/x?status=418");
    ch->CallMethod(nullptr, &c2, nullptr, nullptr, nullptr);
    ASSERT_TRUE(c2.Failed());
    EXPECT_EQ(c2.ErrorCode(), EHTTP);
    EXPECT_EQ(c2.http_response().status_code(), 418);
}

TEST(HttpProtocol, http10_and_connection_close_end_the_connection) {
    Srv s;
    for (const std::string& req : {post("/EchoService/Echo", kEchoJson, "", "HTTP/1.0"),
                                   post("/EchoService/Echo", kEchoJson, "Connection: close\r\n")}) {
        const int fd = connect_to(s.port);
        ASSERT_GE(fd, 0);
        write_all(fd, req);
        bool eof = false;
        const std::string got = read_until(fd, [](const std::string&) { return false; }, 2000, &eof);
        close(fd);
        EXPECT_TRUE(eof);
        EXPECT_TRUE(got.find(" 200 ") != std::string::npos);
        EXPECT_TRUE(got.find("\"hi\"") != std::string::npos);
    }
    // keep-alive (default in 1.1): two requests on one connection
    const int fd = connect_to(s.port);
    write_all(fd, post("/EchoService/Echo", kEchoJson));
    std::string got = read_until(fd, [](const std::string& s) { return s.find("\"hi\"") != std::string::npos; }, 2000);
    write_all(fd, post("/EchoService/Echo", kEchoJson));
    got += read_until(fd, [](const std::string& s) { return s.find("\"hi\"") != std::string::npos; }, 2000);
    close(fd);
    EXPECT_EQ(count(got, "HTTP/1.1 200"), 2u);
}

TEST(HttpProtocol, head_request_gets_headers_only) {
    Srv s;
    const int fd = connect_to(s.port);
    write_all(fd, "HEAD /health HTTP/1.1\r\nHost: t\r\n\r\nGET /health HTTP/1.1\r\nHost: t\r\n\r\n");
    const std::string got =
        read_until(fd, [](const std::string& s) { return count(s, "HTTP/1.1 200") == 2 && s.find("OK\n") != std::string::npos; },
                   2000);
    close(fd);
    EXPECT_EQ(count(got, "HTTP/1.1 200"), 2u);
    EXPECT_EQ(count(got, "OK\n"), 1u);  // only the GET has a body
}

TEST(HttpProtocol, headers_path_and_query_reach_the_handler) {
    Srv s;
    std::unique_ptr<Channel> ch(http_channel(s.addr()));
    Controller cntl;
    cntl.http_request().uri().SetHttpURL("/v1/raw/a%20b/c?x=1&y=two");
    cntl.http_request().SetHeader("X-Custom", "v1");
    cntl.http_request().SetHeader("x-other", "v2");
    cntl.http_request().set_method(HTTP_METHOD_POST);
    cntl.request_attachment().append("payload");
    ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    ASSERT_FALSE(cntl.Failed());
    EXPECT_EQ(cntl.response_attachment().to_string(), "payload");
    ASSERT_TRUE(cntl.http_response().GetHeader("x-custom") != nullptr);
    EXPECT_EQ(*cntl.http_response().GetHeader("x-custom"), "v1");
    EXPECT_EQ(*cntl.http_response().GetHeader("X-OTHER"), "v2");
    EXPECT_TRUE(cntl.http_response().GetHeader("x-unresolved")->find("c") != std::string::npos);
}

TEST(HttpProtocol, body_over_max_body_size_is_refused) {
    std::string prev;
    GetFlag("max_body_size", &prev);
    Srv s;
    SetFlag("max_body_size", "1000");
    const int fd = connect_to(s.port);
    write_all(fd, "POST /v1/raw/x HTTP/1.1\r\nHost: t\r\nContent-Length: 5000\r\n\r\n" + std::string(5000, 'b'));
    bool eof = false;
    const std::string got = read_until(fd, [](const std::string&) { return false; }, 2000, &eof);
    close(fd);
    SetFlag("max_body_size", prev);
    EXPECT_TRUE(eof);
    EXPECT_TRUE(got.find(" 200 ") == std::string::npos);
}

TEST(HttpProtocol, stopping_server_answers_elogoff_then_refuses) {
    Srv s;
    std::unique_ptr<Channel> ch(http_channel(s.addr()));
    example::EchoService_Stub stub(ch.get());
    // a slow call in flight while the server stops
    std::atomic<int> code{-1};
    std::thread slow([&] {
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("slow");
        req.set_sleep_us(300000);
        stub.Echo(&cntl, &req, &res, nullptr);
        code = cntl.ErrorCode();
    });
    usleep(100000);
    const int64_t t0 = monotonic_us();
    s.server.Stop(0);
    slow.join();
    // the call in flight ends promptly: answered, or failed with the
    // connection the stop closed (Stop(0) waits for nobody), never hung
    EXPECT_TRUE(code.load() == 0 || code.load() == EEOF || code.load() == ELOGOFF || code.load() == EFAILEDSOCKET);
    EXPECT_LT(monotonic_us() - t0, 1000000);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("late");
    stub.Echo(&cntl, &req, &res, nullptr);
    EXPECT_TRUE(cntl.Failed());
    s.server.Join();
}

TEST(HttpProtocol, authenticator_rejects_missing_credentials) {
    struct Auth : public Authenticator {
        int GenerateCredential(std::string* out) const override {
            *out = "Bearer good";
            return 0;
        }
        int VerifyCredential(const std::string& cred, const EndPoint&, AuthContext*) const override {
            return cred == "Bearer good" ? 0 : -1;
        }
    } auth;
    ServerOptions o;
    o.auth = &auth;
    Srv s(&o);
    ASSERT_GT(s.port, 0);
    // no credential: the connection is refused
    const int fd = connect_to(s.port);
    write_all(fd, post("/EchoService/Echo", kEchoJson));
    bool eof = false;
    const std::string got = read_until(fd, [](const std::string&) { return false; }, 1500, &eof);
    close(fd);
    EXPECT_TRUE(got.find(" 200 ") == std::string::npos);
    // with the channel's authenticator it works
    Channel ch;
    ChannelOptions opt;
    opt.protocol = "http";
    opt.auth = &auth;
    opt.timeout_ms = 2000;
    ASSERT_EQ(ch.Init(s.addr().c_str(), &opt), 0);
    example::EchoService_Stub stub(&ch);
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("authorized");
    stub.Echo(&cntl, &req, &res, nullptr);
    EXPECT_FALSE(cntl.Failed());
    EXPECT_EQ(res.message(), "authorized");
}

// ------------------------------------------------------------- client side

TEST(HttpProtocol, response_delimited_by_eof) {
    FakeServer f([](int fd) {
        write_all(fd, "HTTP/1.1 200 OK\r\nContent-Type: text/plain\r\nConnection: close\r\n\r\nbody until eof");
    });
    std::unique_ptr<Channel> ch(http_channel(f.addr()));
    Controller cntl;
    cntl.http_request().uri().set_path("/x");
    ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    ASSERT_FALSE(cntl.Failed());
    EXPECT_EQ(cntl.response_attachment().to_string(), "body until eof");
}

TEST(HttpProtocol, error_status_with_body_fails_the_call) {
    FakeServer f([](int fd) {
        write_all(fd, "HTTP/1.1 503 Service Unavailable\r\nContent-Length: 9\r\n\r\nbusy now!");
    });
    std::unique_ptr<Channel> ch(http_channel(f.addr()));
    Controller cntl;
    cntl.http_request().uri().set_path("/x");
    ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    ASSERT_TRUE(cntl.Failed());
    EXPECT_EQ(cntl.ErrorCode(), EHTTP);
    EXPECT_EQ(cntl.http_response().status_code(), 503);
    EXPECT_TRUE(cntl.ErrorText().find("busy now!") != std::string::npos);
}

TEST(HttpProtocol, chunked_response_read_normally) {
    FakeServer f([](int fd) {
        write_all(fd, "HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n");
        for (int i = 0; i < 10; ++i) {
            const std::string piece = "chunk" + std::to_string(i) + ";";
            char hex[16];
            snprintf(hex, sizeof(hex), "%zx\r\n", piece.size());
            write_all(fd, hex + piece + "\r\n");
            usleep(1000);
        }
        write_all(fd, "0\r\n\r\n");
        usleep(50000);
    });
    std::unique_ptr<Channel> ch(http_channel(f.addr()));
    Controller cntl;
    cntl.http_request().uri().set_path("/x");
    ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    ASSERT_FALSE(cntl.Failed());
    std::string want;
    for (int i = 0; i < 10; ++i) want += "chunk" + std::to_string(i) + ";";
    EXPECT_EQ(cntl.response_attachment().to_string(), want);
}

TEST(HttpProtocol, broken_chunk_fails_the_call) {
    FakeServer f([](int fd) {
        write_all(fd, "HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nhello\r\nZZZ\r\nnot hex\r\n");
        usleep(200000);
    });
    std::unique_ptr<Channel> ch(http_channel(f.addr(), 1000));
    Controller cntl;
    cntl.http_request().uri().set_path("/x");
    ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    EXPECT_TRUE(cntl.Failed());
}

TEST(HttpProtocol, long_body_read_progressively) {
    const int kParts = 200;
    FakeServer f([&](int fd) {
        write_all(fd, "HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n");
        for (int i = 0; i < kParts; ++i) {
            const std::string piece(1000, (char)('a' + i % 26));
            write_all(fd, "3e8\r\n" + piece + "\r\n");
        }
        write_all(fd, "0\r\n\r\n");
        usleep(50000);
    });
    std::unique_ptr<Channel> ch(http_channel(f.addr()));
    Controller cntl;
    cntl.http_request().uri().set_path("/x");
    cntl.response_will_be_read_progressively();
    ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    ASSERT_FALSE(cntl.Failed());
    CollectReader r;
    cntl.ReadProgressiveAttachmentBy(&r);
    ASSERT_TRUE(r.wait(5000));
    EXPECT_TRUE(r.st.ok());
    EXPECT_EQ(r.data.size(), (size_t)kParts * 1000);
    EXPECT_EQ(r.data[0], 'a');
    EXPECT_EQ(r.data[(kParts - 1) * 1000], (char)('a' + (kParts - 1) % 26));
}

TEST(HttpProtocol, short_body_read_progressively) {
    FakeServer f([](int fd) {
        write_all(fd, "HTTP/1.1 200 OK\r\nContent-Length: 11\r\n\r\nshort body!");
        usleep(50000);
    });
    std::unique_ptr<Channel> ch(http_channel(f.addr()));
    Controller cntl;
    cntl.http_request().uri().set_path("/x");
    cntl.response_will_be_read_progressively();
    ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    ASSERT_FALSE(cntl.Failed());
    CollectReader r;
    cntl.ReadProgressiveAttachmentBy(&r);
    ASSERT_TRUE(r.wait(3000));
    EXPECT_TRUE(r.st.ok());
    EXPECT_EQ(r.data, "short body!");
}

TEST(HttpProtocol, progressive_reading_outlives_the_controller) {
    std::atomic<bool> go{false};
    FakeServer f([&](int fd) {
        write_all(fd, "HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n5\r\nfirst\r\n");
        for (int i = 0; i < 200 && !go.load(); ++i) usleep(5000);
        write_all(fd, "6\r\nsecond\r\n0\r\n\r\n");
        usleep(50000);
    });
    std::unique_ptr<Channel> ch(http_channel(f.addr()));
    CollectReader r;
    {
        Controller cntl;
        cntl.http_request().uri().set_path("/x");
        cntl.response_will_be_read_progressively();
        ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        ASSERT_FALSE(cntl.Failed());
        cntl.ReadProgressiveAttachmentBy(&r);
    }  // the controller is gone; the rest of the body still reaches the reader
    go = true;
    ASSERT_TRUE(r.wait(3000));
    EXPECT_TRUE(r.st.ok());
    EXPECT_EQ(r.data, "firstsecond");
}

TEST(HttpProtocol, reader_that_stops_early_ends_the_body) {
    FakeServer f([](int fd) {
        write_all(fd, "HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n");
        for (int i = 0; i < 50; ++i) {
            if (write(fd, "4\r\npart\r\n", 9) <= 0) break;
            usleep(2000);
        }
        write(fd, "0\r\n\r\n", 5);
        usleep(50000);
    });
    std::unique_ptr<Channel> ch(http_channel(f.addr()));
    Controller cntl;
    cntl.http_request().uri().set_path("/x");
    cntl.response_will_be_read_progressively();
    ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    ASSERT_FALSE(cntl.Failed());
    CollectReader r;
    r.stop_after = 3;
    cntl.ReadProgressiveAttachmentBy(&r);
    ASSERT_TRUE(r.wait(3000));
    EXPECT_FALSE(r.st.ok());        // ended by the reader's own error
    EXPECT_LE(r.data.size(), 4u * 4);  // nothing delivered after the refusal
}

TEST(HttpProtocol, broken_socket_stops_progressive_reading) {
    FakeServer f([](int fd) {
        write_all(fd, "HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n4\r\nabcd\r\n");
        usleep(30000);
        // close mid-body: no terminating chunk
    });
    std::unique_ptr<Channel> ch(http_channel(f.addr()));
    Controller cntl;
    cntl.http_request().uri().set_path("/x");
    cntl.response_will_be_read_progressively();
    ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    ASSERT_FALSE(cntl.Failed());
    CollectReader r;
    cntl.ReadProgressiveAttachmentBy(&r);
    ASSERT_TRUE(r.wait(3000));
    EXPECT_FALSE(r.st.ok());
    EXPECT_EQ(r.data, "abcd");
}

TEST(HttpProtocol, progressive_response_never_read_is_harmless) {
    Srv s;
    std::unique_ptr<Channel> ch(http_channel(s.addr()));
    for (int i = 0; i < 3; ++i) {
        Controller cntl;
        cntl.http_request().uri().set_path("/HttpTest/Push");
        cntl.response_will_be_read_progressively();
        ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
        EXPECT_FALSE(cntl.Failed());
        if (cntl.Failed()) fprintf(stderr, "push %d: %s\n", i, cntl.ErrorText().c_str());
    }  // skipped: nobody reads the bodies
    Controller cntl;
    cntl.http_request().uri().set_path("/health");
    ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    EXPECT_FALSE(cntl.Failed());
}

TEST(HttpProtocol, progressive_attachment_over_http10_is_eof_delimited) {
    Srv s;
    const int fd = connect_to(s.port);
    write_all(fd, "GET /HttpTest/Push HTTP/1.0\r\nHost: t\r\n\r\n");
    bool eof = false;
    const std::string got = read_until(fd, [](const std::string&) { return false; }, 3000, &eof);
    close(fd);
    EXPECT_TRUE(eof);
    EXPECT_TRUE(got.find("Transfer-Encoding: chunked") == std::string::npos);
    EXPECT_TRUE(got.find("part0;part1;part2;part3;part4;") != std::string::npos);
    if (got.find("part4") == std::string::npos) fprintf(stderr, "http10 got: [%s]\n", got.c_str());
}

TEST(HttpProtocol, timeout_against_a_silent_server) {
    FakeServer f([](int) { usleep(400000); });
    std::unique_ptr<Channel> ch(http_channel(f.addr(), 100));
    Controller cntl;
    cntl.http_request().uri().set_path("/x");
    const int64_t t0 = monotonic_us();
    ch->CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    EXPECT_TRUE(cntl.Failed());
    EXPECT_EQ(cntl.ErrorCode(), ERPCTIMEDOUT);
    EXPECT_LT(monotonic_us() - t0, 350000);
}

// ------------------------------------------------------------- h2

TEST(HttpProtocol, h2_large_bodies_exceed_the_initial_window) {
    Srv s;
    std::unique_ptr<Channel> ch(http_channel(s.addr(), 5000, "h2"));
    ASSERT_TRUE(ch != nullptr);
    example::EchoService_Stub stub(ch.get());
    // 1 MiB each way: far beyond the 64 KiB initial stream window, so the
    // call completes only if WINDOW_UPDATEs flow both ways
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message(std::string(1 << 20, 'w'));
    stub.Echo(&cntl, &req, &res, nullptr);
    ASSERT_FALSE(cntl.Failed());
    EXPECT_EQ(res.message().size(), (size_t)1 << 20);
}

TEST(HttpProtocol, h2_many_streams_then_server_stop_sends_goaway) {
    Srv s;
    std::unique_ptr<Channel> ch(http_channel(s.addr(), 3000, "h2"));
    example::EchoService_Stub stub(ch.get());
    std::vector<std::thread> ths;
    std::atomic<int> ok{0};
    for (int t = 0; t < 8; ++t) {
        ths.emplace_back([&, t] {
            for (int i = 0; i < 25; ++i) {
                Controller cntl;
                example::EchoRequest req;
                example::EchoResponse res;
                req.set_message(std::to_string(t) + ":" + std::to_string(i));
                stub.Echo(&cntl, &req, &res, nullptr);
                if (!cntl.Failed() && res.message() == req.message()) ok.fetch_add(1);
            }
        });
    }
    for (auto& th : ths) th.join();
    EXPECT_EQ(ok.load(), 200);
    s.server.Stop(0);
    s.server.Join();
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("after stop");
    stub.Echo(&cntl, &req, &res, nullptr);
    EXPECT_TRUE(cntl.Failed());
}

TEST(HttpProtocol, h2_timeout_does_not_close_the_connection) {
    Srv s;
    std::unique_ptr<Channel> ch(http_channel(s.addr(), 3000, "h2"));
    example::EchoService_Stub stub(ch.get());
    {
        Controller cntl;
        cntl.set_timeout_ms(50);
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("slow");
        req.set_sleep_us(300000);
        stub.Echo(&cntl, &req, &res, nullptr);
        EXPECT_EQ(cntl.ErrorCode(), ERPCTIMEDOUT);
    }
    // the next call reuses the connection (the timed-out stream was reset,
    // not the socket) and succeeds
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("next");
    stub.Echo(&cntl, &req, &res, nullptr);
    EXPECT_FALSE(cntl.Failed());
    EXPECT_EQ(res.message(), "next");
}

TEST(HttpProtocol, grpc_status_carries_the_server_error) {
    Srv s;
    std::unique_ptr<Channel> ch(http_channel(s.addr(), 3000, "h2:grpc"));
    example::EchoService_Stub stub(ch.get());
    Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("x");
    req.set_server_fail(true);
    stub.Echo(&cntl, &req, &res, nullptr);
    ASSERT_TRUE(cntl.Failed());
    EXPECT_TRUE(cntl.ErrorText().size() > 0);
    Controller ok;
    req.set_server_fail(false);
    stub.Echo(&ok, &req, &res, nullptr);
    EXPECT_FALSE(ok.Failed());
}
