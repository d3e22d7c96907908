// Incremental HTTP/1.x message parser over Buf (role of the reference's
// details/http_message.cpp + the joyent http_parser it embeds,
// src/brpc/details/http_parser.cpp). Written from the RFC 7230 grammar:
// start line, header fields, then a body delimited by Content-Length,
// chunked transfer coding, or connection close. State survives across
// reads so a body arriving in pieces is scanned once.
#pragma once

#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>

#include "base/buf.h"
#include "http/http_header.h"
#include "net/socket.h"
#include "rpc/protocol.h"

namespace mrpc {

class ProgressiveReader;

// Body sink of a response read progressively (client side): the parser
// feeds parts, the user attaches a reader whenever it likes; parts that
// arrive before the reader are buffered.
class ProgressiveSink {
public:
    void Feed(Buf&& part);
    void End(int error_code, const std::string& error_text);
    void SetReader(ProgressiveReader* r);
    bool ended() const;
    bool body_done() const;
    // Runs once the body left the connection (now, if it already did): a
    // pooled connection goes back to its pool only then.
    void SetOnBodyDone(std::function<void()> fn);

private:
    void Drain();
    void RunOnEndLocked();
    mutable std::mutex _mu;
    ProgressiveReader* _reader = nullptr;
    Buf _pending;
    bool _ended = false;          // no more parts for the reader (end of body, or it refused)
    bool _body_done = false;      // the parser reached the end of the body
    bool _end_delivered = false;
    bool _delivering = false;
    int _error_code = 0;
    std::string _error_text;
    std::function<void()> _on_body_done;
};

// In-order responses on one HTTP/1.x connection (RFC 7230 §6.3.2): the
// server runs pipelined requests concurrently, each response waits here for
// the ones before it. One per connection, shared by its requests.
struct HttpResponseOrder {
    std::mutex mu;
    uint64_t next_req = 0;   // the parser's counter (one parsing thread per socket)
    uint64_t next_resp = 0;  // under mu
    std::map<uint64_t, std::pair<Buf, bool>> ready;  // seq -> (packet, shutdown after), under mu
};

class HttpMessage : public InputMessageBase {
public:
    HttpHeader header;
    Buf body;
    bool is_response = false;
    bool keep_alive = true;
    PipelinedInfo pi;                           // client: the call this response answers
    uint32_t stream_id = 0;                     // h2: stream of this message
    std::shared_ptr<ProgressiveSink> progressive;  // client: body continues through the sink
    std::shared_ptr<HttpResponseOrder> order;      // server, HTTP/1.x: the connection's response order
    uint64_t order_seq = 0;
};

class HttpParser : public ParsingContext {
public:
    static const int kTag = 0x48545450;  // "HTTP"
    int protocol_tag() const override { return kTag; }
    enum Result { NEED_MORE = 0, DONE, FAILED };
    explicit HttpParser(int64_t max_body_size) : _max_body(max_body_size) {}
    ~HttpParser() override;
    // Consume bytes from `src`. DONE: a complete message is ready via
    // release(). With a progressive sink installed for the current message,
    // DONE is returned once the headers are complete and the body is
    // streamed into the sink by subsequent calls.
    Result Consume(Buf* src, bool read_eof, std::string* error);
    HttpMessage* release();
    // Set before the body of the current response is parsed.
    void set_progressive(std::shared_ptr<ProgressiveSink> sink) { _sink = std::move(sink); }
    bool headers_done() const { return _state != ST_HEADER; }
    HttpMessage* current() { return _msg; }
    // Called by the protocol right after headers are parsed (DONE for a
    // progressive response) so the body framing can account for HEAD.
    void set_no_body() { _no_body = true; }
    bool streaming_body() const { return _streaming; }
    // Runs after the start line + headers are parsed and before the body
    // framing is decided (the client protocol looks up the pending call
    // there: HEAD => no body, progressive => stream through a sink).
    void (*on_head)(HttpParser* p, HttpMessage* m, void* arg) = nullptr;
    void* on_head_arg = nullptr;
    // server side: numbers the requests of this connection
    std::shared_ptr<HttpResponseOrder> order;

    // Quick check used for protocol sniffing: returns 1 if `head` starts an
    // HTTP message, 0 if it cannot, -1 if more bytes are needed.
    static int LooksLikeHttp(const char* head, size_t n);

private:
    enum State {
        ST_HEADER = 0,
        ST_BODY_LENGTH,
        ST_CHUNK_SIZE,
        ST_CHUNK_DATA,
        ST_CHUNK_DATA_CRLF,
        ST_TRAILER,
        ST_BODY_EOF,
        ST_DONE,
    };
    bool parse_head(const std::string& head, std::string* error);
    bool body_bytes(Buf* src, size_t n);
    bool finish_headers(std::string* error);
    int cut_line(Buf* src, std::string* line, std::string* error);

    int64_t _max_body;
    State _state = ST_HEADER;
    size_t _scanned = 0;  // bytes of src already searched for the header end
    uint64_t _remaining = 0;
    uint64_t _body_total = 0;
    bool _no_body = false;
    bool _streaming = false;
    HttpMessage* _msg = nullptr;
    std::shared_ptr<ProgressiveSink> _sink;
};

// Serialize a request/response head (start line + headers + blank line).
void SerializeHttpRequestHead(Buf* out, const HttpHeader& h, const std::string& host, int64_t content_length,
                              bool chunked);
void SerializeHttpResponseHead(Buf* out, const HttpHeader& h, int64_t content_length, bool chunked, bool keep_alive);

}  // namespace mrpc
