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

int URI::SetHttpURL(const std::string& url) {
    _scheme.clear();
    _host.clear();
    _path.clear();
    _fragment.clear();
    _query.clear();
    _port = -1;
    std::string s = url;
    size_t hash = s.find('#');
    if (hash != std::string::npos) {
        _fragment = s.substr(hash + 1);
        s = s.substr(0, hash);
    }
    size_t scheme_end = s.find("://");
    size_t path_begin = 0;
    if (scheme_end != std::string::npos) {
        _scheme = s.substr(0, scheme_end);
        size_t host_begin = scheme_end + 3;
        path_begin = s.find_first_of("/?", host_begin);
        std::string hostport = s.substr(host_begin, path_begin == std::string::npos ? std::string::npos : path_begin - host_begin);
        size_t at = hostport.rfind('@');
        if (at != std::string::npos) hostport = hostport.substr(at + 1);
        size_t colon = hostport.rfind(':');
        if (colon != std::string::npos) {
            _host = hostport.substr(0, colon);
            _port = atoi(hostport.c_str() + colon + 1);
        } else {
            _host = hostport;
        }
        if (path_begin == std::string::npos) {
            _path = "/";
            return 0;
        }
    }
    std::string rest = s.substr(path_begin);
    size_t q = rest.find('?');
    _path = q == std::string::npos ? rest : rest.substr(0, q);
    if (_path.empty()) _path = "/";
    if (q != std::string::npos) {
        for (const std::string& kv : split_string(rest.substr(q + 1), '&')) {
            size_t eq = kv.find('=');
            if (eq == std::string::npos) _query[url_decode(kv)] = "";
            else _query[url_decode(kv.substr(0, eq))] = url_decode(kv.substr(eq + 1));
        }
    }
    return 0;
}

const std::string* URI::GetQuery(const std::string& key) const {
    auto it = _query.find(key);
    return it == _query.end() ? nullptr : &it->second;
}

std::string URI::query_string() const {
    std::string out;
    for (auto& kv : _query) {
        if (!out.empty()) out += "&";
        out += url_encode(kv.first);
        if (!kv.second.empty()) out += "=" + url_encode(kv.second);
    }
    return out;
}

std::string URI::to_string() const {
    std::string out;
    if (!_scheme.empty()) out += _scheme + "://" + _host + (_port >= 0 ? ":" + std::to_string(_port) : "");
    out += _path.empty() ? "/" : _path;
    std::string q = query_string();
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
