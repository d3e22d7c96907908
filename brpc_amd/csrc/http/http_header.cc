#include "http/http_header.h"

#include <strings.h>

#include <cstdlib>

#include "rpc/errno.h"

namespace mrpc {

const char* HttpMethod2Str(HttpMethod m) {
    switch (m) {
    case HTTP_METHOD_DELETE: return "DELETE";
    case HTTP_METHOD_GET: return "GET";
    case HTTP_METHOD_HEAD: return "HEAD";
    case HTTP_METHOD_POST: return "POST";
    case HTTP_METHOD_PUT: return "PUT";
    case HTTP_METHOD_CONNECT: return "CONNECT";
    case HTTP_METHOD_OPTIONS: return "OPTIONS";
    case HTTP_METHOD_TRACE: return "TRACE";
    case HTTP_METHOD_PATCH: return "PATCH";
    }
    return "UNKNOWN";
}

bool Str2HttpMethod(const std::string& s, HttpMethod* m) {
    static const HttpMethod all[] = {HTTP_METHOD_DELETE, HTTP_METHOD_GET, HTTP_METHOD_HEAD, HTTP_METHOD_POST,
                                     HTTP_METHOD_PUT, HTTP_METHOD_CONNECT, HTTP_METHOD_OPTIONS, HTTP_METHOD_TRACE,
                                     HTTP_METHOD_PATCH};
    for (HttpMethod x : all) {
        if (strcasecmp(s.c_str(), HttpMethod2Str(x)) == 0) {
            *m = x;
            return true;
        }
    }
    return false;
}

const char* HttpReasonPhrase(int s) {
    switch (s) {
    case 100: return "Continue";
    case 200: return "OK";
    case 201: return "Created";
    case 202: return "Accepted";
    case 204: return "No Content";
    case 206: return "Partial Content";
    case 301: return "Moved Permanently";
    case 302: return "Found";
    case 304: return "Not Modified";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 403: return "Forbidden";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 408: return "Request Timeout";
    case 413: return "Payload Too Large";
    case 429: return "Too Many Requests";
    case 500: return "Internal Server Error";
    case 501: return "Not Implemented";
    case 502: return "Bad Gateway";
    case 503: return "Service Unavailable";
    case 504: return "Gateway Timeout";
    default: return "Unknown";
    }
}

int ErrorCodeToStatusCode(int ec) {
    switch (ec) {
    case 0: return HTTP_STATUS_OK;
    case ENOSERVICE:
    case ENOMETHOD: return HTTP_STATUS_NOT_FOUND;
    case ERPCAUTH: return HTTP_STATUS_UNAUTHORIZED;
    case EREQUEST:
    case EINVAL: return HTTP_STATUS_BAD_REQUEST;
    case ELIMIT:
    case ELOGOFF: return HTTP_STATUS_SERVICE_UNAVAILABLE;
    case EPERM: return HTTP_STATUS_FORBIDDEN;
    case ERPCTIMEDOUT:
    case ETIMEDOUT: return HTTP_STATUS_GATEWAY_TIMEOUT;
    default: return HTTP_STATUS_INTERNAL_SERVER_ERROR;
    }
}

bool CaseIgnoredLess::operator()(const std::string& a, const std::string& b) const {
    return strcasecmp(a.c_str(), b.c_str()) < 0;
}

namespace {
bool bad_char(char c) { return (unsigned char)c <= 0x20 || c == 0x7f; }
// Where a space lands decides the message (the reference's wording).
int first_bad(const std::string& s, size_t from, size_t to) {
    for (size_t i = from; i < to; ++i) {
        if (bad_char(s[i])) return (int)i;
    }
    return -1;
}
}  // namespace

int URI::SetHttpURL(const std::string& url) {
    _scheme.clear();
    _user_info.clear();
    _host.clear();
    _path.clear();
    _fragment.clear();
    _status.clear();
    _port = -1;
    set_raw_query("");
    size_t b = 0, e = url.size();
    while (b < e && url[b] == ' ') ++b;
    while (e > b && url[e - 1] == ' ') --e;
    const std::string s = url.substr(b, e - b);
    // split off fragment, then query, then the authority/path part
    const size_t hash = s.find('#');
    const size_t qm = s.find('?');
    const size_t qend = hash == std::string::npos ? s.size() : hash;
    const size_t q = qm != std::string::npos && qm < qend ? qm : std::string::npos;
    const size_t head_end = q != std::string::npos ? q : qend;
    size_t pos = 0;
    const size_t scheme_end = s.find("://");
    if (scheme_end != std::string::npos && scheme_end < head_end && !s.empty() && s[0] != '/') {
        if (first_bad(s, 0, scheme_end) >= 0) {
            _status = "Invalid space in url";
            return -1;
        }
        _scheme = s.substr(0, scheme_end);
        pos = scheme_end + 3;
    }
    if (pos > 0 || (head_end > 0 && s[0] != '/')) {
        // authority: [user_info@]host[:port]
        size_t slash = s.find('/', pos);
        if (slash == std::string::npos || slash > head_end) slash = head_end;
        if (first_bad(s, pos, slash) >= 0) {
            _status = "Invalid space in url";
            return -1;
        }
        std::string auth = s.substr(pos, slash - pos);
        const size_t at = auth.rfind('@');
        if (at != std::string::npos) {
            _user_info = auth.substr(0, at);
            auth = auth.substr(at + 1);
        }
        std::string port_str;
        if (!auth.empty() && auth[0] == '[') {  // IPv6 literal
            const size_t close = auth.find(']');
            if (close == std::string::npos) {
                _status = "Unclosed IPv6 host";
                return -1;
            }
            _host = auth.substr(1, close - 1);
            if (close + 1 < auth.size()) {
                if (auth[close + 1] != ':') {
                    _status = "Invalid character after IPv6 host";
                    return -1;
                }
                port_str = auth.substr(close + 2);
            }
        } else {
            const size_t colon = auth.rfind(':');
            _host = colon == std::string::npos ? auth : auth.substr(0, colon);
            if (colon != std::string::npos) port_str = auth.substr(colon + 1);
        }
        if (!port_str.empty()) {
            long v = 0;
            for (char c : port_str) {
                if (c < '0' || c > '9' || (v = v * 10 + (c - '0')) > 65535) {
                    _status = "Invalid port";
                    return -1;
                }
            }
            _port = (int)v;
        }
        pos = slash;
    }
    if (first_bad(s, pos, head_end) >= 0) {
        _status = "Invalid space in path";
        return -1;
    }
    _path = s.substr(pos, head_end - pos);
    if (q != std::string::npos) {
        if (first_bad(s, q + 1, qend) >= 0) {
            _status = "Invalid space in query";
            return -1;
        }
        set_raw_query(s.substr(q + 1, qend - q - 1));
    }
    if (hash != std::string::npos) {
        if (first_bad(s, hash + 1, s.size()) >= 0) {
            _status = "Invalid space in fragment";
            return -1;
        }
        _fragment = s.substr(hash + 1);
    }
    return 0;
}

void URI::SetH2Path(const std::string& p) {
    _path.clear();
    _fragment.clear();
    set_raw_query("");
    const size_t hash = p.find('#');
    const size_t qend = hash == std::string::npos ? p.size() : hash;
    const size_t q = p.find('?');
    const size_t path_end = q != std::string::npos && q < qend ? q : qend;
    _path = p.substr(0, path_end);
    if (path_end < qend) set_raw_query(p.substr(path_end + 1, qend - path_end - 1));
    if (hash != std::string::npos) _fragment = p.substr(hash + 1);
}

void URI::GenerateH2Path(std::string* out) const {
    *out = _path;
    const std::string& q = query();
    if (!q.empty()) *out += "?" + q;
    if (!_fragment.empty()) *out += "#" + _fragment;
}

void URI::parse_query() const {
    if (_parsed) return;
    _parsed = true;
    _qv.clear();
    size_t i = 0;
    while (i <= _query.size()) {
        size_t amp = _query.find('&', i);
        if (amp == std::string::npos) amp = _query.size();
        if (amp > i) {
            const std::string kv = _query.substr(i, amp - i);
            const size_t eq = kv.find('=');
            const std::string k = url_decode(eq == std::string::npos ? kv : kv.substr(0, eq));
            if (!k.empty()) {
                std::string v = eq == std::string::npos ? std::string() : url_decode(kv.substr(eq + 1));
                bool dup = false;
                for (auto& x : _qv) {
                    if (x.first == k) {  // the last one wins
                        x.second = v;
                        dup = true;
                        break;
                    }
                }
                if (!dup) _qv.emplace_back(k, std::move(v));
            }
        }
        i = amp + 1;
    }
}

const std::string* URI::GetQuery(const std::string& key) const {
    parse_query();
    for (auto& x : _qv) {
        if (x.first == key) return &x.second;
    }
    return nullptr;
}

void URI::SetQuery(const std::string& key, const std::string& value) {
    parse_query();
    _dirty = true;
    for (auto& x : _qv) {
        if (x.first == key) {
            x.second = value;
            return;
        }
    }
    _qv.emplace_back(key, value);
}

size_t URI::RemoveQuery(const std::string& key) {
    parse_query();
    for (size_t i = 0; i < _qv.size(); ++i) {
        if (_qv[i].first == key) {
            _qv.erase(_qv.begin() + i);
            _dirty = true;
            return 1;
        }
    }
    return 0;
}

size_t URI::QueryCount() const {
    parse_query();
    return _qv.size();
}

const std::string& URI::query() const {
    if (_dirty) {
        _query.clear();
        for (auto& x : _qv) {
            if (!_query.empty()) _query += "&";
            _query += url_encode(x.first);
            if (!x.second.empty()) _query += "=" + url_encode(x.second);
        }
        _dirty = false;
    }
    return _query;
}

std::map<std::string, std::string> URI::queries() const {
    parse_query();
    return std::map<std::string, std::string>(_qv.begin(), _qv.end());
}

std::string URI::to_string() const {
    std::string out;
    if (!_scheme.empty()) out += _scheme + "://";
    if (!_host.empty()) {
        if (!_user_info.empty()) out += _user_info + "@";
        out += _host.find(':') != std::string::npos ? "[" + _host + "]" : _host;
        if (_port >= 0) out += ":" + std::to_string(_port);
    }
    out += _path.empty() ? "/" : _path;
    const std::string& q = query();
    if (!q.empty()) out += "?" + q;
    if (!_fragment.empty()) out += "#" + _fragment;
    return out;
}

const std::string* HttpHeader::GetHeader(const std::string& key) const {
    if (strcasecmp(key.c_str(), "content-type") == 0 && !_content_type.empty()) return &_content_type;
    auto it = _headers.find(key);
    return it == _headers.end() ? nullptr : &it->second;
}

void HttpHeader::SetHeader(const std::string& key, const std::string& value) {
    if (strcasecmp(key.c_str(), "content-type") == 0) {
        _content_type = value;
        return;
    }
    _headers[key] = value;
}

void HttpHeader::AppendHeader(const std::string& key, const std::string& value) {
    auto it = _headers.find(key);
    if (it == _headers.end()) _headers[key] = value;
    else it->second += "," + value;
}

void HttpHeader::RemoveHeader(const std::string& key) { _headers.erase(key); }

void HttpHeader::Clear() {
    _status = HTTP_STATUS_OK;
    _method = HTTP_METHOD_GET;
    _major = _minor = 1;
    _uri = URI();
    _content_type.clear();
    _unresolved_path.clear();
    _headers.clear();
}

}  // namespace mrpc
