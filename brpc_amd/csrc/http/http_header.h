// HTTP header container + URI (role of src/brpc/http_header.h, uri.h,
// http_method.h, http_status_code.h).
#pragma once

#include <map>
#include <string>
#include <vector>

#include "base/util.h"

namespace mrpc {

enum HttpMethod {
    HTTP_METHOD_DELETE = 0,
    HTTP_METHOD_GET = 1,
    HTTP_METHOD_HEAD = 2,
    HTTP_METHOD_POST = 3,
    HTTP_METHOD_PUT = 4,
    HTTP_METHOD_CONNECT = 5,
    HTTP_METHOD_OPTIONS = 6,
    HTTP_METHOD_TRACE = 7,
    HTTP_METHOD_PATCH = 28,
};
const char* HttpMethod2Str(HttpMethod m);
bool Str2HttpMethod(const std::string& s, HttpMethod* m);

// status codes
enum {
    HTTP_STATUS_OK = 200,
    HTTP_STATUS_NO_CONTENT = 204,
    HTTP_STATUS_MOVE_PERMANENTLY = 301,
    HTTP_STATUS_FOUND = 302,
    HTTP_STATUS_NOT_MODIFIED = 304,
    HTTP_STATUS_BAD_REQUEST = 400,
    HTTP_STATUS_UNAUTHORIZED = 401,
    HTTP_STATUS_FORBIDDEN = 403,
    HTTP_STATUS_NOT_FOUND = 404,
    HTTP_STATUS_METHOD_NOT_ALLOWED = 405,
    HTTP_STATUS_REQUEST_TIMEOUT = 408,
    HTTP_STATUS_PAYLOAD_TOO_LARGE = 413,
    HTTP_STATUS_TOO_MANY_REQUESTS = 429,
    HTTP_STATUS_INTERNAL_SERVER_ERROR = 500,
    HTTP_STATUS_NOT_IMPLEMENTED = 501,
    HTTP_STATUS_BAD_GATEWAY = 502,
    HTTP_STATUS_SERVICE_UNAVAILABLE = 503,
    HTTP_STATUS_GATEWAY_TIMEOUT = 504,
};
const char* HttpReasonPhrase(int status);
// RPC error code <-> http status mapping
int ErrorCodeToStatusCode(int error_code);

struct CaseIgnoredLess {
    bool operator()(const std::string& a, const std::string& b) const;
};

// A request URL (role of src/brpc/uri.h). The query keeps its raw text:
// lookups parse it lazily (empty segments and empty keys are skipped, a key
// without '=' has an empty value, keys and values are percent-decoded), and
// query()/GenerateH2Path() give back the original text until SetQuery or
// RemoveQuery change it, after which the pairs are re-serialized in their
// original order (percent-encoded).
class URI {
public:
    URI() : _port(-1) {}
    // Parse "[scheme://][user_info@]host[:port][/path][?query][#fragment]"
    // or "/path[?query][#fragment]". Surrounding spaces are ignored; a space
    // or control character inside, a bad port or an unclosed IPv6 bracket
    // fail with -1 and status() names the problem. Without a scheme, text
    // that does not start with '/' is a host (and optional port, path...).
    int SetHttpURL(const std::string& url);
    // The h2 :path pseudo header: "/path[?query][#fragment]" (no host part).
    void SetH2Path(const std::string& path);
    void GenerateH2Path(std::string* out) const;
    std::string to_string() const;
    const std::string& status() const { return _status; }
    const std::string& scheme() const { return _scheme; }
    const std::string& host() const { return _host; }
    int port() const { return _port; }
    const std::string& user_info() const { return _user_info; }
    const std::string& path() const { return _path; }
    void set_path(const std::string& p) { _path = p; }
    const std::string& fragment() const { return _fragment; }
    void set_host(const std::string& h) { _host = h; }
    const std::string* GetQuery(const std::string& key) const;
    void SetQuery(const std::string& key, const std::string& value);
    // number of pairs removed (0 or 1)
    size_t RemoveQuery(const std::string& key);
    size_t QueryCount() const;
    // the raw query text (or its re-serialization after a change)
    const std::string& query() const;
    std::string query_string() const { return query(); }
    std::map<std::string, std::string> queries() const;

private:
    void parse_query() const;
    void set_raw_query(const std::string& q) {
        _query = q;
        _qv.clear();
        _parsed = false;
        _dirty = false;
    }
    std::string _scheme, _user_info, _host, _path, _fragment, _status;
    int _port;
    mutable std::string _query;
    mutable std::vector<std::pair<std::string, std::string>> _qv;
    mutable bool _parsed = false;
    mutable bool _dirty = false;
};

class HttpHeader {
public:
    HttpHeader() : _status(HTTP_STATUS_OK), _method(HTTP_METHOD_GET), _major(1), _minor(1) {}
    int status_code() const { return _status; }
    void set_status_code(int s) { _status = s; }
    const char* reason_phrase() const { return HttpReasonPhrase(_status); }
    HttpMethod method() const { return _method; }
    void set_method(HttpMethod m) { _method = m; }
    URI& uri() { return _uri; }
    const URI& uri() const { return _uri; }
    const std::string& content_type() const { return _content_type; }
    void set_content_type(const std::string& t) { _content_type = t; }
    const std::string* GetHeader(const std::string& key) const;
    void SetHeader(const std::string& key, const std::string& value);
    void AppendHeader(const std::string& key, const std::string& value);
    void RemoveHeader(const std::string& key);
    const std::map<std::string, std::string, CaseIgnoredLess>& headers() const { return _headers; }
    int major_version() const { return _major; }
    int minor_version() const { return _minor; }
    void set_version(int major, int minor) {
        _major = major;
        _minor = minor;
    }
    // path after the service/method prefix for restful/builtin services
    const std::string& unresolved_path() const { return _unresolved_path; }
    void set_unresolved_path(const std::string& p) { _unresolved_path = p; }
    void Clear();

private:
    int _status;
    HttpMethod _method;
    int _major, _minor;
    URI _uri;
    std::string _content_type;
    std::string _unresolved_path;
    std::map<std::string, std::string, CaseIgnoredLess> _headers;
};

}  // namespace mrpc
