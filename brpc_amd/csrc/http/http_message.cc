#include "http/http_message.h"

#include <cstring>

#include "base/logging.h"
#include "rpc/errno.h"
#include "rpc/progressive.h"

namespace mrpc {

// ---------------------------------------------------------------- sink
// Parts, the end and the reader arrive from different threads (the parser's
// and the user's); one of them at a time owns delivery (_delivering) and
// drains what is queued, so the reader sees its callbacks one at a time and
// in order: every part, then OnEndOfMessage exactly once.
void ProgressiveSink::Feed(Buf&& part) {
    {
        std::lock_guard<std::mutex> g(_mu);
        if (_ended) return;  // the reader refused earlier: the rest is dropped
        _pending.append(std::move(part));
        if (!_reader || _delivering) return;
        _delivering = true;
    }
    Drain();
}

void ProgressiveSink::End(int error_code, const std::string& error_text) {
    {
        std::lock_guard<std::mutex> g(_mu);
        if (_body_done) return;
        _body_done = true;
        if (!_ended) {
            _ended = true;
            _error_code = error_code;
            _error_text = error_text;
        }
        if (!_reader || _delivering) {
            if (!_reader) RunOnEndLocked();  // nobody reads: the connection is free now
            return;
        }
        _delivering = true;
    }
    Drain();
}

void ProgressiveSink::SetReader(ProgressiveReader* r) {
    {
        std::lock_guard<std::mutex> g(_mu);
        if (_reader) return;
        _reader = r;
        if (_delivering) return;
        _delivering = true;
    }
    Drain();
}

void ProgressiveSink::SetOnBodyDone(std::function<void()> fn) {
    std::function<void()> now;
    {
        std::lock_guard<std::mutex> g(_mu);
        if (_body_done) now = std::move(fn);
        else _on_body_done = std::move(fn);
    }
    if (now) now();
}

void ProgressiveSink::RunOnEndLocked() {
    if (!_on_body_done) return;
    std::function<void()> fn = std::move(_on_body_done);
    _on_body_done = nullptr;
    // run outside the lock by the caller's thread: defer through a fiber-safe
    // path is not needed (the callback only returns a socket to its pool)
    _mu.unlock();
    fn();
    _mu.lock();
}

void ProgressiveSink::Drain() {
    for (;;) {
        Buf batch;
        ProgressiveReader* r;
        bool deliver_end = false;
        Status end_st;
        {
            std::lock_guard<std::mutex> g(_mu);
            r = _reader;
            batch.swap(_pending);
            if (batch.empty()) {
                if (_ended && !_end_delivered) {
                    _end_delivered = true;
                    deliver_end = true;
                    end_st = _error_code ? Status(_error_code, _error_text) : Status();
                }
                _delivering = false;
                if (_body_done) RunOnEndLocked();
            }
        }
        if (batch.empty()) {
            if (deliver_end) r->OnEndOfMessage(end_st);
            return;
        }
        for (size_t i = 0; i < batch.backing_block_num(); ++i) {
            Status st = r->OnReadOnePart(batch.block_data(i), batch.block_len(i));
            if (!st.ok()) {
                // the reader refused: it gets no more parts, and its
                // OnEndOfMessage carries that error (the reference's
                // ProgressiveReader contract, failed_on_read_one_part); the
                // rest of the body is still parsed off the connection
                bool deliver;
                {
                    std::lock_guard<std::mutex> g(_mu);
                    _ended = true;
                    _pending.clear();
                    deliver = !_end_delivered;
                    _end_delivered = true;
                    _error_code = st.error_code();
                    _error_text = st.error_str();
                    _delivering = false;
                    if (_body_done) RunOnEndLocked();
                }
                if (deliver) r->OnEndOfMessage(st);
                return;
            }
        }
    }
}

bool ProgressiveSink::body_done() const {
    std::lock_guard<std::mutex> g(_mu);
    return _body_done;
}

bool ProgressiveSink::ended() const {
    std::lock_guard<std::mutex> g(_mu);
    return _ended;
}

// ---------------------------------------------------------------- parser
static const char* const kMethods[] = {"GET ", "POST ", "PUT ", "HEAD ", "DELETE ", "OPTIONS ", "PATCH ",
                                       "CONNECT ", "TRACE ", "HTTP/"};

int HttpParser::LooksLikeHttp(const char* head, size_t n) {
    bool prefix_of_some = false;
    for (const char* m : kMethods) {
        const size_t ml = strlen(m);
        if (n >= ml) {
            if (memcmp(head, m, ml) == 0) return 1;
        } else if (memcmp(head, m, n) == 0) {
            prefix_of_some = true;
        }
    }
    return prefix_of_some ? -1 : 0;
}

HttpParser::~HttpParser() {
    if (_sink) _sink->End(EEOF, "connection closed while reading the body");
    delete _msg;
}

HttpMessage* HttpParser::release() {
    HttpMessage* m = _msg;
    _msg = nullptr;
    return m;
}

static inline std::string trim_ws(const std::string& s) {
    size_t b = 0, e = s.size();
    while (b < e && (s[b] == ' ' || s[b] == '\t')) ++b;
    while (e > b && (s[e - 1] == ' ' || s[e - 1] == '\t' || s[e - 1] == '\r')) --e;
    return s.substr(b, e - b);
}

bool HttpParser::parse_head(const std::string& head, std::string* error) {
    size_t pos = 0;
    bool first = true;
    std::string last_name;
    while (pos < head.size()) {
        size_t eol = head.find('\n', pos);
        if (eol == std::string::npos) eol = head.size();
        std::string line = head.substr(pos, eol - pos);
        if (!line.empty() && line.back() == '\r') line.pop_back();
        pos = eol + 1;
        if (first) {
            first = false;
            if (line.compare(0, 5, "HTTP/") == 0) {
                // HTTP/1.1 200 OK
                _msg->is_response = true;
                // RFC 9112: status-code = 3DIGIT, followed by SP or end of line
                if (line.size() < 12 || line[6] != '.' || line[8] != ' ' || !isdigit((unsigned char)line[5]) ||
                    !isdigit((unsigned char)line[7]) || !isdigit((unsigned char)line[9]) ||
                    !isdigit((unsigned char)line[10]) || !isdigit((unsigned char)line[11]) ||
                    (line.size() > 12 && line[12] != ' ') || line[9] == '0') {
                    *error = "bad status line: " + line;
                    return false;
                }
                _msg->header.set_version(line[5] - '0', line[7] - '0');
                _msg->header.set_status_code(atoi(line.c_str() + 9));
            } else {
                const size_t sp1 = line.find(' ');
                const size_t sp2 = line.rfind(' ');
                if (sp1 == std::string::npos || sp2 == sp1 || line.compare(sp2 + 1, 5, "HTTP/") != 0 ||
                    line.size() < sp2 + 9) {
                    *error = "bad request line: " + line;
                    return false;
                }
                HttpMethod m;
                if (!Str2HttpMethod(line.substr(0, sp1), &m)) {
                    *error = "unknown method in: " + line;
                    return false;
                }
                _msg->header.set_method(m);
                _msg->header.set_version(line[sp2 + 6] - '0', line[sp2 + 8] - '0');
                if (_msg->header.uri().SetHttpURL(line.substr(sp1 + 1, sp2 - sp1 - 1)) != 0) {
                    *error = "bad uri in: " + line;
                    return false;
                }
            }
            continue;
        }
        if (line.empty()) continue;
        if ((line[0] == ' ' || line[0] == '\t') && !last_name.empty()) {  // obsolete folding
            const std::string* v = _msg->header.GetHeader(last_name);
            _msg->header.SetHeader(last_name, (v ? *v + " " : std::string()) + trim_ws(line));
            continue;
        }
        const size_t colon = line.find(':');
        if (colon == std::string::npos || colon == 0) {
            *error = "bad header line: " + line;
            return false;
        }
        const std::string name = trim_ws(line.substr(0, colon));
        const std::string value = trim_ws(line.substr(colon + 1));
        if (strcasecmp(name.c_str(), "content-type") == 0) {
            _msg->header.set_content_type(value);
        } else {
            _msg->header.AppendHeader(name, value);
        }
        last_name = name;
    }
    return true;
}

bool HttpParser::finish_headers(std::string* error) {
    HttpHeader& h = _msg->header;
    const std::string* conn = h.GetHeader("Connection");
    if (h.major_version() == 1 && h.minor_version() == 0) {
        _msg->keep_alive = conn && strcasecmp(conn->c_str(), "keep-alive") == 0;
    } else {
        _msg->keep_alive = !(conn && strcasecmp(conn->c_str(), "close") == 0);
    }
    const std::string* te = h.GetHeader("Transfer-Encoding");
    const std::string* cl = h.GetHeader("Content-Length");
    const int status = h.status_code();
    if (_no_body || (_msg->is_response && (status / 100 == 1 || status == 204 || status == 304))) {
        _state = ST_DONE;
    } else if (te && strcasestr(te->c_str(), "chunked")) {
        _state = ST_CHUNK_SIZE;
    } else if (cl) {
        char* end = nullptr;
        const long long n = strtoll(cl->c_str(), &end, 10);
        if (n < 0 || end == cl->c_str()) {
            *error = "bad Content-Length: " + *cl;
            return false;
        }
        if (_max_body > 0 && n > _max_body) {
            *error = "body of " + std::to_string(n) + " bytes exceeds max_body_size";
            return false;
        }
        _remaining = (uint64_t)n;
        _state = n ? ST_BODY_LENGTH : ST_DONE;
    } else if (_msg->is_response) {
        _state = ST_BODY_EOF;  // delimited by connection close
        _msg->keep_alive = false;
    } else {
        _state = ST_DONE;  // request without a body
    }
    return true;
}

bool HttpParser::body_bytes(Buf* src, size_t n) {
    _body_total += n;
    if (_max_body > 0 && (int64_t)_body_total > _max_body && !_sink) return false;
    if (_sink) {
        Buf part;
        src->cutn(&part, n);
        _sink->Feed(std::move(part));
    } else {
        src->cutn(&_msg->body, n);
    }
    return true;
}

// Returns 1 with a line, 0 when more data is needed, -1 on error.
int HttpParser::cut_line(Buf* src, std::string* line, std::string* error) {
    char buf[128];
    const size_t n = src->copy_to(buf, std::min(src->size(), sizeof(buf)));
    for (size_t i = 0; i < n; ++i) {
        if (buf[i] == '\n') {
            line->assign(buf, i);
            if (!line->empty() && line->back() == '\r') line->pop_back();
            src->pop_front(i + 1);
            return 1;
        }
    }
    if (n == sizeof(buf)) {
        *error = "chunk line too long";
        return -1;
    }
    return 0;
}

HttpParser::Result HttpParser::Consume(Buf* src, bool read_eof, std::string* error) {
    if (_state == ST_DONE && _msg == nullptr) {
        // previous message delivered: start over
        _state = ST_HEADER;
        _scanned = 0;
        _remaining = 0;
        _body_total = 0;
        _no_body = false;
        _streaming = false;
        _sink.reset();
    }
    for (;;) {
        switch (_state) {
        case ST_HEADER: {
            // search "\n\r\n" or "\n\n" from where we stopped last time
            const size_t n = src->size();
            if (n == 0) return NEED_MORE;
            const size_t kMaxHead = 64 * 1024;
            std::string head;
            const size_t look = std::min(n, kMaxHead + 4);
            src->copy_to(&head, look);
            size_t end = std::string::npos, skip = 0;
            for (size_t i = _scanned > 3 ? _scanned - 3 : 0; i < head.size(); ++i) {
                if (head[i] != '\n') continue;
                if (i + 1 < head.size() && head[i + 1] == '\n') {
                    end = i + 1;
                    skip = 1;
                    break;
                }
                if (i + 2 < head.size() && head[i + 1] == '\r' && head[i + 2] == '\n') {
                    end = i + 1;
                    skip = 2;
                    break;
                }
            }
            if (end == std::string::npos) {
                if (look > kMaxHead) {
                    *error = "http header too large";
                    return FAILED;
                }
                _scanned = head.size();
                if (read_eof) {
                    *error = "connection closed inside http header";
                    return FAILED;
                }
                return NEED_MORE;
            }
            head.resize(end);
            src->pop_front(end + skip);
            _msg = new HttpMessage;
            bool ok = parse_head(head, error);
            if (ok && on_head) on_head(this, _msg, on_head_arg);
            if (!ok || !finish_headers(error)) {
                delete _msg;
                _msg = nullptr;
                return FAILED;
            }
            if (_sink && _state != ST_DONE) {
                // progressive response: hand the headers over now, the body
                // keeps flowing through the sink
                _streaming = true;
                _msg->progressive = _sink;
                return DONE;
            }
            break;
        }
        case ST_BODY_LENGTH: {
            const size_t take = (size_t)std::min<uint64_t>(_remaining, src->size());
            if (take && !body_bytes(src, take)) {
                *error = "body exceeds max_body_size";
                return FAILED;
            }
            _remaining -= take;
            if (_remaining) {
                if (read_eof) {
                    *error = "connection closed inside http body";
                    return FAILED;
                }
                return NEED_MORE;
            }
            _state = ST_DONE;
            break;
        }
        case ST_CHUNK_SIZE: {
            std::string line;
            const int r = cut_line(src, &line, error);
            if (r < 0) return FAILED;
            if (r == 0) return NEED_MORE;
            char* end = nullptr;
            const unsigned long long n = strtoull(line.c_str(), &end, 16);
            if (end == line.c_str()) {
                *error = "bad chunk size line: " + line;
                return FAILED;
            }
            if (n == 0) {
                _state = ST_TRAILER;
            } else {
                _remaining = n;
                _state = ST_CHUNK_DATA;
            }
            break;
        }
        case ST_CHUNK_DATA: {
            const size_t take = (size_t)std::min<uint64_t>(_remaining, src->size());
            if (take && !body_bytes(src, take)) {
                *error = "body exceeds max_body_size";
                return FAILED;
            }
            _remaining -= take;
            if (_remaining) return NEED_MORE;
            _state = ST_CHUNK_DATA_CRLF;
            break;
        }
        case ST_CHUNK_DATA_CRLF: {
            std::string line;
            const int r = cut_line(src, &line, error);
            if (r < 0) return FAILED;
            if (r == 0) return NEED_MORE;
            if (!line.empty()) {
                *error = "missing CRLF after chunk data";
                return FAILED;
            }
            _state = ST_CHUNK_SIZE;
            break;
        }
        case ST_TRAILER: {
            std::string line;
            const int r = cut_line(src, &line, error);
            if (r < 0) return FAILED;
            if (r == 0) return NEED_MORE;
            if (line.empty()) _state = ST_DONE;
            break;
        }
        case ST_BODY_EOF: {
            if (!src->empty() && !body_bytes(src, src->size())) {
                *error = "body exceeds max_body_size";
                return FAILED;
            }
            if (!read_eof) return NEED_MORE;
            _state = ST_DONE;
            break;
        }
        case ST_DONE: {
            if (_streaming) {
                _sink->End(0, "");
                _sink.reset();
                _streaming = false;
                // the message itself was delivered at header time
                return NEED_MORE;
            }
            return DONE;
        }
        }
    }
}

// ---------------------------------------------------------------- serialize
static void append_headers(std::string* s, const HttpHeader& h) {
    for (auto& kv : h.headers()) {
        if (strcasecmp(kv.first.c_str(), "content-length") == 0 ||
            strcasecmp(kv.first.c_str(), "transfer-encoding") == 0) {
            continue;
        }
        s->append(kv.first).append(": ").append(kv.second).append("\r\n");
    }
    if (!h.content_type().empty()) s->append("Content-Type: ").append(h.content_type()).append("\r\n");
}

void SerializeHttpRequestHead(Buf* out, const HttpHeader& h, const std::string& host, int64_t content_length,
                              bool chunked) {
    std::string s;
    s.reserve(256);
    s.append(HttpMethod2Str(h.method())).append(" ");
    std::string path = h.uri().path().empty() ? "/" : h.uri().path();
    const std::string q = h.uri().query_string();
    if (!q.empty()) path += "?" + q;
    s.append(path).append(" HTTP/").append(std::to_string(h.major_version())).append(".")
        .append(std::to_string(h.minor_version())).append("\r\n");
    if (!h.GetHeader("Host") && !host.empty()) s.append("Host: ").append(host).append("\r\n");
    append_headers(&s, h);
    if (chunked) {
        s.append("Transfer-Encoding: chunked\r\n");
    } else if (content_length >= 0 &&
               (content_length > 0 || h.method() == HTTP_METHOD_POST || h.method() == HTTP_METHOD_PUT ||
                h.method() == HTTP_METHOD_PATCH)) {
        s.append("Content-Length: ").append(std::to_string(content_length)).append("\r\n");
    }
    if (!h.GetHeader("Accept")) s.append("Accept: */*\r\n");
    if (!h.GetHeader("User-Agent")) s.append("User-Agent: mrpc/1.0\r\n");
    s.append("\r\n");
    out->append(s);
}

void SerializeHttpResponseHead(Buf* out, const HttpHeader& h, int64_t content_length, bool chunked, bool keep_alive) {
    std::string s;
    s.reserve(256);
    s.append("HTTP/").append(std::to_string(h.major_version())).append(".").append(std::to_string(h.minor_version()));
    s.append(" ").append(std::to_string(h.status_code())).append(" ").append(h.reason_phrase()).append("\r\n");
    append_headers(&s, h);
    if (chunked) {
        s.append("Transfer-Encoding: chunked\r\n");
    } else if (content_length >= 0) {
        s.append("Content-Length: ").append(std::to_string(content_length)).append("\r\n");
    }
    if (!keep_alive && !h.GetHeader("Connection")) s.append("Connection: close\r\n");
    s.append("\r\n");
    out->append(s);
}

}  // namespace mrpc
