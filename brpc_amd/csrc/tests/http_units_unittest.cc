// HTTP building blocks, one behaviour per case (spirit of the reference's
// test/brpc_uri_unittest.cpp, brpc_http_parser_unittest.cpp,
// brpc_http_message_unittest.cpp, brpc_hpack_unittest.cpp).
#include <memory>
#include <string>
#include <vector>

#include "base/buf.h"
#include "http/hpack.h"
#include "http/http_header.h"
#include "http/http_message.h"
#include "tests/test.h"

using namespace mrpc;

namespace {
HttpParser::Result Feed(HttpParser* p, const std::string& s, std::unique_ptr<HttpMessage>* out, std::string* err,
                        bool eof = false) {
    Buf b;
    b.append(s);
    HttpParser::Result r = p->Consume(&b, eof, err);
    if (r == HttpParser::DONE) out->reset(p->release());
    return r;
}
}  // namespace

TEST(UriUnit, full_url_components) {
    URI u;
    ASSERT_EQ(u.SetHttpURL("http://example.com:8080/a/b%20c?x=1&y=&z=3#frag"), 0);
    EXPECT_EQ(u.scheme(), "http");
    EXPECT_EQ(u.host(), "example.com");
    EXPECT_EQ(u.port(), 8080);
    EXPECT_EQ(u.fragment(), "frag");
    ASSERT_TRUE(u.GetQuery("x") != nullptr);
    EXPECT_EQ(*u.GetQuery("x"), "1");
    ASSERT_TRUE(u.GetQuery("y") != nullptr);
    EXPECT_EQ(*u.GetQuery("y"), "");
    EXPECT_TRUE(u.GetQuery("w") == nullptr);
    EXPECT_EQ(u.queries().size(), 3u);
}

TEST(UriUnit, path_only_and_default_port) {
    URI u;
    ASSERT_EQ(u.SetHttpURL("/status?verbose"), 0);
    EXPECT_EQ(u.path(), "/status");
    EXPECT_TRUE(u.host().empty());
    EXPECT_EQ(u.port(), -1);
    EXPECT_TRUE(u.GetQuery("verbose") != nullptr);
    URI v;
    ASSERT_EQ(v.SetHttpURL("https://h/"), 0);
    EXPECT_EQ(v.scheme(), "https");
    EXPECT_EQ(v.path(), "/");
}

TEST(UriUnit, set_remove_query_and_serialize) {
    URI u;
    ASSERT_EQ(u.SetHttpURL("/p?a=1"), 0);
    u.SetQuery("b", "x y");
    u.RemoveQuery("a");
    const std::string q = u.query_string();
    EXPECT_TRUE(q.find("b=") != std::string::npos);
    EXPECT_TRUE(q.find("a=") == std::string::npos);
    URI back;
    ASSERT_EQ(back.SetHttpURL(u.to_string()), 0);
    ASSERT_TRUE(back.GetQuery("b") != nullptr);
    EXPECT_EQ(*back.GetQuery("b"), "x y");
}

TEST(HttpHeaderUnit, case_insensitive_names_and_append) {
    HttpHeader h;
    h.SetHeader("X-Trace-Id", "abc");
    ASSERT_TRUE(h.GetHeader("x-trace-id") != nullptr);
    EXPECT_EQ(*h.GetHeader("X-TRACE-ID"), "abc");
    h.AppendHeader("Accept", "text/html");
    h.AppendHeader("accept", "application/json");
    ASSERT_TRUE(h.GetHeader("Accept") != nullptr);
    EXPECT_TRUE(h.GetHeader("Accept")->find("text/html") != std::string::npos);
    EXPECT_TRUE(h.GetHeader("Accept")->find("application/json") != std::string::npos);
    h.RemoveHeader("ACCEPT");
    EXPECT_TRUE(h.GetHeader("accept") == nullptr);
}

TEST(HttpHeaderUnit, methods_statuses_and_error_mapping) {
    HttpMethod m;
    EXPECT_TRUE(Str2HttpMethod("PATCH", &m));
    EXPECT_EQ(m, HTTP_METHOD_PATCH);
    EXPECT_EQ(std::string(HttpMethod2Str(HTTP_METHOD_OPTIONS)), "OPTIONS");
    EXPECT_FALSE(Str2HttpMethod("FETCH", &m));
    EXPECT_EQ(std::string(HttpReasonPhrase(404)), "Not Found");
    EXPECT_EQ(std::string(HttpReasonPhrase(503)), "Service Unavailable");
    EXPECT_EQ(ErrorCodeToStatusCode(0), 200);
    EXPECT_NE(ErrorCodeToStatusCode(1002), 200);  // ENOMETHOD is an error status
}

TEST(HttpParserUnit, content_length_body_split_across_reads) {
    HttpParser p(1 << 20);
    std::string err;
    Buf b;
    b.append("PUT /x HTTP/1.1\r\nContent-Length: 10\r\n\r\n01234");
    EXPECT_EQ((int)p.Consume(&b, false, &err), (int)HttpParser::NEED_MORE);
    b.append("56789");
    ASSERT_EQ((int)p.Consume(&b, false, &err), (int)HttpParser::DONE);
    std::unique_ptr<HttpMessage> m(p.release());
    EXPECT_EQ(m->header.method(), HTTP_METHOD_PUT);
    EXPECT_EQ(m->body.to_string(), "0123456789");
}

TEST(HttpParserUnit, rejects_body_over_limit) {
    HttpParser p(100);
    std::string err;
    std::unique_ptr<HttpMessage> m;
    EXPECT_EQ((int)Feed(&p, "POST / HTTP/1.1\r\nContent-Length: 1000\r\n\r\n", &m, &err), (int)HttpParser::FAILED);
    EXPECT_FALSE(err.empty());
    HttpParser q(100);  // chunked bodies count too
    std::string big(200, 'a');
    char hex[16];
    snprintf(hex, sizeof(hex), "%zx", big.size());
    err.clear();
    EXPECT_EQ((int)Feed(&q, "POST / HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n" + std::string(hex) + "\r\n" + big +
                                "\r\n0\r\n\r\n",
                        &m, &err),
              (int)HttpParser::FAILED);
}

TEST(HttpParserUnit, malformed_start_lines_fail) {
    for (const char* bad : {"GARBAGE\r\n\r\n", "GET\r\n\r\n", "HTTP/1.1 abc OK\r\n\r\n",
                            "GET / HTTP/1.1\r\nContent-Length: -5\r\n\r\n",
                            "GET / HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\nzz\r\n"}) {
        HttpParser p(1 << 20);
        std::string err;
        std::unique_ptr<HttpMessage> m;
        const int r = (int)Feed(&p, bad, &m, &err);
        if (r != (int)HttpParser::FAILED) fprintf(stderr, "  not rejected: %s\n", bad);
        EXPECT_EQ(r, (int)HttpParser::FAILED);
    }
}

TEST(HttpParserUnit, response_without_length_reads_until_eof) {
    HttpParser p(1 << 20);
    std::string err;
    Buf b;
    b.append("HTTP/1.1 200 OK\r\nConnection: close\r\n\r\npart1");
    EXPECT_EQ((int)p.Consume(&b, false, &err), (int)HttpParser::NEED_MORE);
    b.append("part2");
    ASSERT_EQ((int)p.Consume(&b, true, &err), (int)HttpParser::DONE);
    std::unique_ptr<HttpMessage> m(p.release());
    EXPECT_EQ(m->header.status_code(), 200);
    EXPECT_EQ(m->body.to_string(), "part1part2");
    EXPECT_FALSE(m->keep_alive);
}

TEST(HttpParserUnit, chunk_extensions_and_trailers) {
    HttpParser p(1 << 20);
    std::string err;
    std::unique_ptr<HttpMessage> m;
    ASSERT_EQ((int)Feed(&p,
                        "POST /t HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n"
                        "3;name=value\r\nabc\r\n0\r\nX-Checksum: 42\r\n\r\n",
                        &m, &err),
              (int)HttpParser::DONE);
    EXPECT_EQ(m->body.to_string(), "abc");
}

TEST(HttpParserUnit, looks_like_http_sniffing) {
    EXPECT_EQ(HttpParser::LooksLikeHttp("GET / HTTP/1.1\r\n", 16), 1);
    EXPECT_EQ(HttpParser::LooksLikeHttp("HTTP/1.1 200 OK", 15), 1);
    EXPECT_EQ(HttpParser::LooksLikeHttp("PRPC", 4), 0);
    EXPECT_EQ(HttpParser::LooksLikeHttp("GE", 2), -1);
}

TEST(HttpParserUnit, serialize_heads_round_trip) {
    HttpHeader h;
    h.set_method(HTTP_METHOD_POST);
    h.uri().SetHttpURL("/svc/method?k=v");
    h.set_content_type("application/json");
    h.SetHeader("X-Custom", "1");
    Buf out;
    SerializeHttpRequestHead(&out, h, "host.example", 2, false);
    out.append("{}");
    HttpParser p(1 << 20);
    std::string err;
    ASSERT_EQ((int)p.Consume(&out, false, &err), (int)HttpParser::DONE);
    std::unique_ptr<HttpMessage> m(p.release());
    EXPECT_EQ(m->header.method(), HTTP_METHOD_POST);
    EXPECT_EQ(m->header.uri().path(), "/svc/method");
    EXPECT_EQ(*m->header.uri().GetQuery("k"), "v");
    EXPECT_EQ(m->header.content_type(), "application/json");
    EXPECT_EQ(*m->header.GetHeader("x-custom"), "1");
    EXPECT_EQ(m->body.to_string(), "{}");
    HttpHeader r;
    r.set_status_code(503);
    Buf rout;
    SerializeHttpResponseHead(&rout, r, 0, false, true);
    HttpParser rp(1 << 20);
    ASSERT_EQ((int)rp.Consume(&rout, false, &err), (int)HttpParser::DONE);
    m.reset(rp.release());
    EXPECT_EQ(m->header.status_code(), 503);
    EXPECT_TRUE(m->body.empty());
}

TEST(HpackUnit, integer_codec_rfc7541_examples) {
    std::string out;
    hpack::EncodeInteger(&out, 0, 5, 10);  // C.1.1
    ASSERT_EQ(out.size(), 1u);
    EXPECT_EQ((uint8_t)out[0], 10);
    out.clear();
    hpack::EncodeInteger(&out, 0, 5, 1337);  // C.1.2: 31, 154, 10
    ASSERT_EQ(out.size(), 3u);
    EXPECT_EQ((uint8_t)out[0], 31);
    EXPECT_EQ((uint8_t)out[1], 154);
    EXPECT_EQ((uint8_t)out[2], 10);
    uint64_t v = 0;
    EXPECT_EQ(hpack::DecodeInteger((const uint8_t*)out.data(), out.size(), 5, &v), 3u);
    EXPECT_EQ(v, 1337u);
    EXPECT_EQ(hpack::DecodeInteger((const uint8_t*)out.data(), 2, 5, &v), 0u);  // truncated
}

TEST(HpackUnit, huffman_rfc7541_vector) {
    // C.4.1: "www.example.com" -> f1e3 c2e5 f23a 6ba0 ab90 f4ff
    std::string enc;
    hpack::HuffmanEncode(&enc, "www.example.com");
    const unsigned char want[] = {0xf1, 0xe3, 0xc2, 0xe5, 0xf2, 0x3a, 0x6b, 0xa0, 0xab, 0x90, 0xf4, 0xff};
    ASSERT_EQ(enc.size(), sizeof(want));
    EXPECT_EQ(memcmp(enc.data(), want, sizeof(want)), 0);
    EXPECT_EQ(hpack::HuffmanEncodedLength("www.example.com"), sizeof(want));
    std::string dec;
    ASSERT_TRUE(hpack::HuffmanDecode(want, sizeof(want), &dec));
    EXPECT_EQ(dec, "www.example.com");
    const unsigned char bad[] = {0xff, 0xff, 0xff, 0xff};  // EOS inside the string
    EXPECT_FALSE(hpack::HuffmanDecode(bad, sizeof(bad), &dec));
}

TEST(HpackUnit, dynamic_table_eviction_and_size) {
    HPackTable t(100);
    t.Add("aaaa", "bbbb");  // 4+4+32 = 40
    t.Add("cccc", "dddd");  // 80
    EXPECT_EQ(t.size(), 80u);
    EXPECT_EQ(t.dynamic_count(), 2u);
    t.Add("eeee", "ffff");  // 120 > 100: the oldest goes
    EXPECT_EQ(t.dynamic_count(), 2u);
    EXPECT_EQ(t.Get(62)->name, "eeee");  // first dynamic index is the newest
    EXPECT_EQ(t.Get(63)->name, "cccc");
    size_t full = 0, name_only = 0;
    t.Find("cccc", "dddd", &full, &name_only);
    EXPECT_EQ(full, 63u);
    t.Find(":method", "GET", &full, &name_only);  // static table
    EXPECT_EQ(full, 2u);
    t.SetMaxSize(0);
    EXPECT_EQ(t.dynamic_count(), 0u);
    EXPECT_EQ(t.Get(62), nullptr);
}

TEST(HpackUnit, encoder_decoder_share_dynamic_state) {
    HPackEncoder enc;
    HPackDecoder dec;
    for (int round = 0; round < 3; ++round) {
        Buf block;
        enc.Encode(&block, {":method", "POST"});
        enc.Encode(&block, {":path", "/example.EchoService/Echo"});
        enc.Encode(&block, {"x-request-id", "req-" + std::to_string(round)});
        enc.Encode(&block, {"authorization", "secret"}, HPackIndexPolicy::NEVER_INDEXED);
        std::vector<HPackHeader> out;
        ASSERT_TRUE(dec.Decode(block.to_string(), &out));
        ASSERT_EQ(out.size(), 4u);
        EXPECT_EQ(out[1].value, "/example.EchoService/Echo");
        EXPECT_EQ(out[2].value, "req-" + std::to_string(round));
        EXPECT_EQ(out[3].value, "secret");
        if (round > 0) EXPECT_LT(block.size(), 40u);  // repeated headers are table references
    }
    std::vector<HPackHeader> out;
    EXPECT_FALSE(dec.Decode(std::string("\xff\xff\xff\xff\x0f", 5), &out));  // index far past the table
}

// RFC 7541 Appendix C.3 / C.4: three requests on one connection, without
// and with Huffman coding; the second and third reference entries the
// first ones added to the dynamic table (indices 62, 63).
namespace {
std::string unhex(const char* h) {
    std::string s;
    for (size_t i = 0; h[i] && h[i + 1]; i += 2) {
        if (h[i] == ' ') {
            --i;
            continue;
        }
        s.push_back((char)std::stoi(std::string(h + i, 2), nullptr, 16));
    }
    return s;
}
void expect_headers(const std::vector<HPackHeader>& got, const std::vector<std::pair<std::string, std::string>>& want) {
    ASSERT_EQ(got.size(), want.size());
    for (size_t i = 0; i < want.size(); ++i) {
        EXPECT_EQ(got[i].name, want[i].first);
        EXPECT_EQ(got[i].value, want[i].second);
    }
}
void run_rfc_requests(const char* r1, const char* r2, const char* r3) {
    HPackDecoder dec;
    std::vector<HPackHeader> out;
    ASSERT_TRUE(dec.Decode(unhex(r1), &out));
    expect_headers(out, {{":method", "GET"}, {":scheme", "http"}, {":path", "/"}, {":authority", "www.example.com"}});
    out.clear();
    ASSERT_TRUE(dec.Decode(unhex(r2), &out));
    expect_headers(out, {{":method", "GET"}, {":scheme", "http"}, {":path", "/"}, {":authority", "www.example.com"},
                         {"cache-control", "no-cache"}});
    out.clear();
    ASSERT_TRUE(dec.Decode(unhex(r3), &out));
    expect_headers(out, {{":method", "GET"}, {":scheme", "https"}, {":path", "/index.html"},
                         {":authority", "www.example.com"}, {"custom-key", "custom-value"}});
}
}  // namespace

TEST(HpackUnit, rfc7541_c3_requests_without_huffman) {
    run_rfc_requests("828684410f7777772e6578616d706c652e636f6d", "828684be58086e6f2d6361636865",
                     "828785bf400a637573746f6d2d6b65790c637573746f6d2d76616c7565");
}

TEST(HpackUnit, rfc7541_c4_requests_with_huffman) {
    run_rfc_requests("828684418cf1e3c2e5f23a6ba0ab90f4ff", "828684be5886a8eb10649cbf",
                     "828785bf408825a849e95ba97d7f8925a849e95bb8e8b4bf");
}

TEST(HpackUnit, encoder_output_decodes_in_rfc_order) {
    // our encoder on the C.3 header lists: whatever it chooses to index,
    // a fresh decoder reproduces the lists in order across the three blocks
    HPackEncoder enc;
    HPackDecoder dec;
    const std::vector<std::vector<std::pair<std::string, std::string>>> reqs = {
        {{":method", "GET"}, {":scheme", "http"}, {":path", "/"}, {":authority", "www.example.com"}},
        {{":method", "GET"}, {":scheme", "http"}, {":path", "/"}, {":authority", "www.example.com"},
         {"cache-control", "no-cache"}},
        {{":method", "GET"}, {":scheme", "https"}, {":path", "/index.html"}, {":authority", "www.example.com"},
         {"custom-key", "custom-value"}}};
    size_t prev = 0;
    for (size_t r = 0; r < reqs.size(); ++r) {
        Buf block;
        for (const auto& h : reqs[r]) enc.Encode(&block, {h.first, h.second});
        std::vector<HPackHeader> out;
        ASSERT_TRUE(dec.Decode(block.to_string(), &out));
        expect_headers(out, reqs[r]);
        if (r == 1) EXPECT_LT(block.size(), prev);  // the authority is a table reference now
        prev = block.size();
    }
}
