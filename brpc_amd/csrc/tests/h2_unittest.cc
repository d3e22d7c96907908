// HTTP/2 connection-level behaviour driven by a raw-frame client on a real
// server port (spirit of the reference's test/brpc_http_rpc_protocol_unittest
// h2 cases and test/brpc_h2_unsent_message_unittest.cpp): SETTINGS/PING
// acknowledgements, RFC 7540 flow-control and SETTINGS validation (GOAWAY
// with the right error code), CONTINUATION sequencing and RST_STREAM on
// stream-level window errors.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "http/hpack.h"
#include "base/buf.h"
#include "rpc/server.h"
#include "services/echo_service.h"
#include "tests/test.h"

using namespace mrpc;

namespace {

enum { DATA = 0, HEADERS = 1, RST_STREAM = 3, SETTINGS = 4, PING = 6, GOAWAY = 7, WINDOW_UPDATE = 8, CONTINUATION = 9 };

struct Frame {
    uint32_t len = 0;
    uint8_t type = 0, flags = 0;
    uint32_t sid = 0;
    std::string payload;
};

std::string frame(uint8_t type, uint8_t flags, uint32_t sid, const std::string& payload) {
    std::string f;
    const uint32_t n = (uint32_t)payload.size();
    f.push_back((char)(n >> 16));
    f.push_back((char)(n >> 8));
    f.push_back((char)n);
    f.push_back((char)type);
    f.push_back((char)flags);
    const uint32_t be = htonl(sid & 0x7FFFFFFF);
    f.append(reinterpret_cast<const char*>(&be), 4);
    return f + payload;
}

std::string u32(uint32_t v) {
    const uint32_t be = htonl(v);
    return std::string(reinterpret_cast<const char*>(&be), 4);
}

std::string setting(uint16_t id, uint32_t v) {
    std::string s;
    s.push_back((char)(id >> 8));
    s.push_back((char)id);
    return s + u32(v);
}

class RawH2 {
public:
    explicit RawH2(int port) {
        _fd = socket(AF_INET, SOCK_STREAM, 0);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_port = htons((uint16_t)port);
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        if (connect(_fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
            close(_fd);
            _fd = -1;
            return;
        }
        send_raw(std::string("PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n", 24) + frame(SETTINGS, 0, 0, ""));
    }
    ~RawH2() {
        if (_fd >= 0) close(_fd);
    }
    bool ok() const { return _fd >= 0; }
    void send_raw(const std::string& s) {
        size_t off = 0;
        while (off < s.size()) {
            const ssize_t n = write(_fd, s.data() + off, s.size() - off);
            if (n <= 0) return;
            off += (size_t)n;
        }
    }
    // Next frame, or false on EOF/timeout.
    bool read_frame(Frame* f, int timeout_ms = 3000) {
        while (_in.size() < 9 || _in.size() < 9 + frame_len()) {
            pollfd p{_fd, POLLIN, 0};
            if (poll(&p, 1, timeout_ms) <= 0) return false;
            char buf[16384];
            const ssize_t n = read(_fd, buf, sizeof(buf));
            if (n <= 0) return false;
            _in.append(buf, (size_t)n);
        }
        f->len = frame_len();
        f->type = (uint8_t)_in[3];
        f->flags = (uint8_t)_in[4];
        f->sid = ntohl(*reinterpret_cast<const uint32_t*>(_in.data() + 5)) & 0x7FFFFFFF;
        f->payload = _in.substr(9, f->len);
        _in.erase(0, 9 + f->len);
        return true;
    }
    // Skip frames until one of `type` arrives.
    bool expect(uint8_t type, Frame* f, int timeout_ms = 3000) {
        while (read_frame(f, timeout_ms)) {
            if (f->type == type) return true;
        }
        return false;
    }
    // True when the server closes the connection within the timeout.
    bool closed(int timeout_ms = 3000) {
        Frame f;
        while (read_frame(&f, timeout_ms)) {
        }
        pollfd p{_fd, POLLIN, 0};
        if (poll(&p, 1, timeout_ms) <= 0) return false;
        char c;
        return read(_fd, &c, 1) <= 0;
    }

private:
    uint32_t frame_len() const {
        return ((uint32_t)(uint8_t)_in[0] << 16) | ((uint32_t)(uint8_t)_in[1] << 8) | (uint8_t)_in[2];
    }
    int _fd = -1;
    std::string _in;
};

struct H2Server {
    Server server;
    EchoServiceImpl echo;
    int port = 0;
    H2Server() {
        server.AddService(&echo, SERVER_DOESNT_OWN_SERVICE);
        ServerOptions o;
        if (server.Start("127.0.0.1:0", &o) == 0) port = server.listen_port();
    }
};

H2Server& srv() {
    static H2Server* s = new H2Server;
    return *s;
}

uint32_t goaway_code(const Frame& f) {
    return f.payload.size() >= 8 ? ntohl(*reinterpret_cast<const uint32_t*>(f.payload.data() + 4)) : 0xFFFFFFFF;
}

// HEADERS block of a gRPC-less POST to the echo method (no END_STREAM).
std::string request_headers() {
    HPackEncoder enc;
    Buf block;
    std::vector<HPackHeader> hs = {{":method", "POST"},
                                   {":scheme", "http"},
                                   {":path", "/example.EchoService/Echo"},
                                   {":authority", "127.0.0.1"},
                                   {"content-type", "application/json"}};
    for (const auto& h : hs) enc.Encode(&block, h);
    return block.to_string();
}

}  // namespace

TEST(H2Frames, settings_and_ping_are_acknowledged) {
    ASSERT_GT(srv().port, 0);
    RawH2 c(srv().port);
    ASSERT_TRUE(c.ok());
    Frame f;
    ASSERT_TRUE(c.expect(SETTINGS, &f));  // the server's own SETTINGS
    c.send_raw(frame(PING, 0, 0, "12345678"));
    bool acked = false;
    while (c.read_frame(&f)) {
        if (f.type == PING) {
            EXPECT_EQ((int)f.flags & 1, 1);
            EXPECT_EQ(f.payload, std::string("12345678"));
            acked = true;
            break;
        }
    }
    EXPECT_TRUE(acked);
}

TEST(H2Frames, unknown_frame_type_is_ignored) {
    RawH2 c(srv().port);
    ASSERT_TRUE(c.ok());
    c.send_raw(frame(0xEE, 0, 0, "whatever"));
    c.send_raw(frame(PING, 0, 0, "abcdefgh"));
    Frame f;
    ASSERT_TRUE(c.expect(PING, &f));
    EXPECT_EQ(f.payload, std::string("abcdefgh"));
}

TEST(H2Frames, window_update_zero_increment_is_protocol_error) {
    RawH2 c(srv().port);
    ASSERT_TRUE(c.ok());
    c.send_raw(frame(WINDOW_UPDATE, 0, 0, u32(0)));
    Frame f;
    ASSERT_TRUE(c.expect(GOAWAY, &f));
    EXPECT_EQ(goaway_code(f), 1u);  // PROTOCOL_ERROR
}

TEST(H2Frames, connection_window_overflow_is_flow_control_error) {
    RawH2 c(srv().port);
    ASSERT_TRUE(c.ok());
    c.send_raw(frame(WINDOW_UPDATE, 0, 0, u32(0x7FFFFFFF)));
    Frame f;
    ASSERT_TRUE(c.expect(GOAWAY, &f));
    EXPECT_EQ(goaway_code(f), 3u);  // FLOW_CONTROL_ERROR
}

TEST(H2Frames, bad_initial_window_setting_is_flow_control_error) {
    RawH2 c(srv().port);
    ASSERT_TRUE(c.ok());
    c.send_raw(frame(SETTINGS, 0, 0, setting(4, 0x80000000u)));
    Frame f;
    ASSERT_TRUE(c.expect(GOAWAY, &f));
    EXPECT_EQ(goaway_code(f), 3u);
}

TEST(H2Frames, bad_max_frame_size_setting_is_protocol_error) {
    RawH2 c(srv().port);
    ASSERT_TRUE(c.ok());
    c.send_raw(frame(SETTINGS, 0, 0, setting(5, 100)));
    Frame f;
    ASSERT_TRUE(c.expect(GOAWAY, &f));
    EXPECT_EQ(goaway_code(f), 1u);
}

TEST(H2Frames, settings_with_bad_length_is_frame_size_error) {
    RawH2 c(srv().port);
    ASSERT_TRUE(c.ok());
    c.send_raw(frame(SETTINGS, 0, 0, "12345"));
    Frame f;
    ASSERT_TRUE(c.expect(GOAWAY, &f));
    EXPECT_EQ(goaway_code(f), 6u);  // FRAME_SIZE_ERROR
}

TEST(H2Frames, headers_must_be_followed_by_continuation) {
    RawH2 c(srv().port);
    ASSERT_TRUE(c.ok());
    const std::string block = request_headers();
    // HEADERS without END_HEADERS, then a PING instead of CONTINUATION
    c.send_raw(frame(HEADERS, 0, 1, block.substr(0, block.size() / 2)));
    c.send_raw(frame(PING, 0, 0, "xxxxxxxx"));
    Frame f;
    ASSERT_TRUE(c.expect(GOAWAY, &f));
    EXPECT_EQ(goaway_code(f), 1u);
}

TEST(H2Frames, split_header_block_with_continuation_is_served) {
    RawH2 c(srv().port);
    ASSERT_TRUE(c.ok());
    const std::string block = request_headers();
    c.send_raw(frame(HEADERS, 0, 1, block.substr(0, 5)));
    c.send_raw(frame(CONTINUATION, 4 /*END_HEADERS*/, 1, block.substr(5)));
    c.send_raw(frame(DATA, 1 /*END_STREAM*/, 1, "{\"message\":\"hi\"}"));
    Frame f;
    ASSERT_TRUE(c.expect(HEADERS, &f));
    EXPECT_EQ(f.sid, 1u);
    ASSERT_TRUE(c.expect(DATA, &f));
    EXPECT_TRUE(f.payload.find("\"hi\"") != std::string::npos);
}

TEST(H2Frames, stream_window_update_zero_resets_the_stream) {
    RawH2 c(srv().port);
    ASSERT_TRUE(c.ok());
    // open stream 1 (request not finished yet), then a 0 stream increment
    c.send_raw(frame(HEADERS, 4, 1, request_headers()));
    c.send_raw(frame(WINDOW_UPDATE, 0, 1, u32(0)));
    Frame f;
    ASSERT_TRUE(c.expect(RST_STREAM, &f));
    EXPECT_EQ(f.sid, 1u);
    EXPECT_EQ(ntohl(*reinterpret_cast<const uint32_t*>(f.payload.data())), 1u);
    // the connection itself survives
    c.send_raw(frame(PING, 0, 0, "stillup!"));
    ASSERT_TRUE(c.expect(PING, &f));
}
