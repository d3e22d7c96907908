// Protocol matrix, round 6 (spirit of the reference's per-protocol suites:
// brpc_hulu_pbrpc_protocol_unittest, brpc_sofa_pbrpc_protocol_unittest,
// brpc_baidu_rpc_protocol behaviour in brpc_channel_unittest,
// brpc_http_rpc_protocol_unittest, brpc_grpc_protocol_unittest): the same
// behaviours checked across every pb-capable client protocol against one
// server — error codes and texts coming back, large bodies, repeated ids,
// server-side timeouts, concurrent callers on one connection, repeated
// fields, and the per-protocol compression matrix.
#include <unistd.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "base/time.h"
#include "http/http_header.h"
#include "mrpc/proto/echo.pb.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

struct MatrixServer {
    Server server;
    EchoServiceImpl echo;
    int port = 0;
    MatrixServer() {
        server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        ServerOptions o;
        if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
    }
    std::string addr() const { return "127.0.0.1:" + std::to_string(port); }
};

MatrixServer& srv() {
    static MatrixServer* s = new MatrixServer;
    return *s;
}

struct Client {
    Channel ch;
    int rc = -1;
    Client(const std::string& protocol, int timeout_ms = 3000, int max_retry = 0) {
        ChannelOptions o;
        o.protocol = protocol;
        o.timeout_ms = timeout_ms;
        o.max_retry = max_retry;
        rc = ch.Init(srv().addr().c_str(), &o);
    }
    // One echo call; returns the controller's error code (0 ok).
    int echo(const std::string& msg, std::string* got = nullptr, CompressType ct = COMPRESS_TYPE_NONE,
             int sleep_us = 0, bool fail = false, int code = 0, std::string* err_text = nullptr,
             int timeout_ms = -1) {
        example::EchoService_Stub stub(&ch);
        Controller cntl;
        if (timeout_ms > 0) cntl.set_timeout_ms(timeout_ms);
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message(msg);
        if (sleep_us) req.set_sleep_us(sleep_us);
        if (fail) {
            req.set_server_fail(true);
            req.set_code(code);
        }
        cntl.set_request_compress_type(ct);
        stub.Echo(&cntl, &req, &res, nullptr);
        if (got) *got = cntl.Failed() ? "" : res.message();
        if (err_text) *err_text = cntl.ErrorText();
        return cntl.ErrorCode();
    }
};

const char* kPbProtocols[] = {"baidu_std", "hulu_pbrpc", "sofa_pbrpc", "http", "h2", "h2:grpc"};

}  // namespace

TEST(ProtocolMatrix, every_protocol_echoes) {
    for (const char* p : kPbProtocols) {
        Client c(p);
        ASSERT_EQ(c.rc, 0);
        std::string got;
        EXPECT_TRUE_M(c.echo(std::string("hi ") + p, &got) == 0, p);
        EXPECT_EQ(got, std::string("hi ") + p);
    }
}

TEST(ProtocolMatrix, empty_message_round_trips) {
    for (const char* p : kPbProtocols) {
        Client c(p);
        std::string got = "x";
        EXPECT_TRUE_M(c.echo("", &got) == 0, p);
        EXPECT_EQ(got, "");
    }
}

TEST(ProtocolMatrix, binary_bytes_survive) {
    std::string bin;
    for (int i = 0; i < 256; ++i) bin.push_back((char)i);
    for (const char* p : {"baidu_std", "hulu_pbrpc", "sofa_pbrpc", "h2:grpc"}) {
        Client c(p);
        std::string got;
        // proto2 `string` fields carry arbitrary bytes on the pb wire
        EXPECT_TRUE_M(c.echo(bin, &got) == 0, p);
        EXPECT_TRUE_M(got == bin, p);
    }
}

TEST(ProtocolMatrix, large_messages_round_trip) {
    const std::string big(3 << 20, 'L');
    for (const char* p : kPbProtocols) {
        Client c(p, 10000);
        std::string got;
        EXPECT_TRUE_M(c.echo(big, &got) == 0, p);
        EXPECT_TRUE_M(got.size() == big.size(), p);
    }
}

TEST(ProtocolMatrix, server_error_code_comes_back) {
    for (const char* p : {"baidu_std", "hulu_pbrpc", "sofa_pbrpc"}) {
        Client c(p);
        std::string text;
        const int ec = c.echo("x", nullptr, COMPRESS_TYPE_NONE, 0, true, 1234, &text);
        EXPECT_TRUE_M(ec == 1234, std::string(p) + " got " + std::to_string(ec));
        EXPECT_TRUE_M(text.find("server_fail requested") != std::string::npos, p);
    }
}

TEST(ProtocolMatrix, server_error_fails_http_family_calls) {
    for (const char* p : {"http", "h2", "h2:grpc"}) {
        Client c(p);
        const int ec = c.echo("x", nullptr, COMPRESS_TYPE_NONE, 0, true, EINTERNAL);
        EXPECT_TRUE_M(ec != 0, p);
    }
}

TEST(ProtocolMatrix, client_timeout_beats_a_slow_server) {
    for (const char* p : kPbProtocols) {
        Client c(p);
        const int64_t t0 = monotonic_us();
        const int ec = c.echo("slow", nullptr, COMPRESS_TYPE_NONE, 300000, false, 0, nullptr, 50);
        const int64_t took = monotonic_us() - t0;
        EXPECT_TRUE_M(ec == ERPCTIMEDOUT, std::string(p) + " ec=" + std::to_string(ec));
        EXPECT_TRUE_M(took < 250000, std::string(p) + " took " + std::to_string(took));
    }
}

TEST(ProtocolMatrix, calls_after_a_timeout_still_work) {
    for (const char* p : kPbProtocols) {
        Client c(p);
        c.echo("slow", nullptr, COMPRESS_TYPE_NONE, 200000, false, 0, nullptr, 20);
        std::string got;
        EXPECT_TRUE_M(c.echo("after", &got) == 0, p);
        EXPECT_EQ(got, "after");
    }
}

TEST(ProtocolMatrix, concurrent_callers_share_one_channel) {
    for (const char* p : {"baidu_std", "hulu_pbrpc", "sofa_pbrpc", "h2", "h2:grpc"}) {
        Client c(p);
        std::atomic<int> ok{0};
        std::vector<std::thread> ths;
        for (int t = 0; t < 6; ++t) {
            ths.emplace_back([&, t] {
                for (int i = 0; i < 40; ++i) {
                    const std::string m = std::to_string(t) + ":" + std::to_string(i);
                    std::string got;
                    if (c.echo(m, &got) == 0 && got == m) ok.fetch_add(1);
                }
            });
        }
        for (auto& th : ths) th.join();
        EXPECT_TRUE_M(ok.load() == 240, std::string(p) + " ok=" + std::to_string(ok.load()));
    }
}

TEST(ProtocolMatrix, compression_matrix_for_pb_protocols) {
    const CompressType cts[] = {COMPRESS_TYPE_NONE, COMPRESS_TYPE_SNAPPY, COMPRESS_TYPE_GZIP, COMPRESS_TYPE_ZLIB};
    const std::string body = std::string(20000, 'c') + "tail";
    for (const char* p : {"baidu_std", "hulu_pbrpc"}) {
        Client c(p);
        for (CompressType ct : cts) {
            std::string got;
            EXPECT_TRUE_M(c.echo(body, &got, ct) == 0, std::string(p) + " ct=" + std::to_string((int)ct));
            EXPECT_TRUE(got == body);
        }
    }
}

TEST(ProtocolMatrix, grpc_encodings_round_trip) {
    Client c("h2:grpc");
    const std::string body = std::string(50000, 'g') + "end";
    for (CompressType ct : {COMPRESS_TYPE_NONE, COMPRESS_TYPE_SNAPPY, COMPRESS_TYPE_GZIP, COMPRESS_TYPE_ZLIB}) {
        std::string got;
        EXPECT_TRUE_M(c.echo(body, &got, ct) == 0, "ct=" + std::to_string((int)ct));
        EXPECT_TRUE(got == body);
    }
}

TEST(ProtocolMatrix, retries_reach_a_healthy_call) {
    // a connection the server closes mid-call is retried on a new one
    for (const char* p : {"baidu_std", "hulu_pbrpc"}) {
        Client c(p, 2000, 2);
        std::string got;
        EXPECT_TRUE_M(c.echo("before", &got) == 0, p);
        example::EchoService_Stub stub(&c.ch);
        Controller cntl;
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message("close");
        req.set_close_fd(true);
        stub.Echo(&cntl, &req, &res, nullptr);
        // whatever the closing call saw, the channel recovers (a new
        // connection, or the health check revives the old one)
        int ec = -1;
        for (int i = 0; i < 60 && ec != 0; ++i) {
            ec = c.echo("after", &got);
            if (ec != 0) usleep(100000);
        }
        EXPECT_TRUE_M(ec == 0, p);
        EXPECT_EQ(got, "after");
    }
}

TEST(ProtocolMatrix, async_calls_complete_through_done) {
    for (const char* p : {"baidu_std", "h2:grpc", "http"}) {
        Client c(p);
        example::EchoService_Stub stub(&c.ch);
        const int n = 50;
        std::atomic<int> ok{0}, done{0};
        std::vector<std::unique_ptr<Controller>> cntls;
        std::vector<std::unique_ptr<example::EchoRequest>> reqs;
        std::vector<std::unique_ptr<example::EchoResponse>> ress;
        for (int i = 0; i < n; ++i) {
            cntls.emplace_back(new Controller);
            reqs.emplace_back(new example::EchoRequest);
            ress.emplace_back(new example::EchoResponse);
            reqs.back()->set_message("a" + std::to_string(i));
            Controller* cn = cntls.back().get();
            example::EchoRequest* rq = reqs.back().get();
            example::EchoResponse* rs = ress.back().get();
            stub.Echo(cn, rq, rs, NewCallback([&, cn, rq, rs] {
                          if (!cn->Failed() && rs->message() == rq->message()) ok.fetch_add(1);
                          done.fetch_add(1);
                      }));
        }
        for (int i = 0; i < 3000 && done.load() < n; ++i) usleep(1000);
        EXPECT_TRUE_M(ok.load() == n, std::string(p) + " ok=" + std::to_string(ok.load()));
    }
}

TEST(ProtocolMatrix, unknown_method_path_over_http) {
    Channel ch;
    ChannelOptions o;
    o.protocol = "http";
    o.timeout_ms = 2000;
    ASSERT_EQ(ch.Init(srv().addr().c_str(), &o), 0);
    Controller cntl;
    cntl.http_request().uri().set_path("/example.EchoService/NoSuchMethod");
    ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    EXPECT_TRUE(cntl.Failed());
    EXPECT_EQ(cntl.http_response().status_code(), 404);
}

TEST(ProtocolMatrix, http_json_body_for_pb_method) {
    Channel ch;
    ChannelOptions o;
    o.protocol = "http";
    ASSERT_EQ(ch.Init(srv().addr().c_str(), &o), 0);
    Controller cntl;
    cntl.http_request().uri().set_path("/example.EchoService/Echo");
    cntl.http_request().set_method(HTTP_METHOD_POST);
    cntl.request_attachment().append("{\"message\":\"json body\"}");
    ch.CallMethod(nullptr, &cntl, nullptr, nullptr, nullptr);
    ASSERT_FALSE(cntl.Failed());
    const std::string body = cntl.response_attachment().to_string();
    EXPECT_TRUE(body.find("\"message\":\"json body\"") != std::string::npos);
}

TEST(ProtocolMatrix, log_id_reaches_the_server_span_free) {
    // log ids ride the baidu_std meta; the call succeeds with one set
    Client c("baidu_std");
    example::EchoService_Stub stub(&c.ch);
    Controller cntl;
    cntl.set_log_id(0x1234567890ull);
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("logged");
    stub.Echo(&cntl, &req, &res, nullptr);
    EXPECT_FALSE(cntl.Failed());
    EXPECT_EQ(res.message(), "logged");
}
