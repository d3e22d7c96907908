// Minimal self-contained HTTP/1.1 GET used by control-plane code (naming
// services, health checks, parallel_http tool) that must not depend on a
// Channel. Fiber-aware: waits through fiber::fd_timedwait.
#pragma once

#include <map>
#include <string>

namespace mrpc {

struct HttpSimpleResponse {
    int status = 0;
    std::map<std::string, std::string> headers;
    std::string body;
};

// url: "http://host:port/path?q". Returns 0 on HTTP 2xx, -1 otherwise.
int HttpGet(const std::string& url, std::string* body, int timeout_ms);
int HttpFetch(const std::string& method, const std::string& url, const std::string& req_body,
              HttpSimpleResponse* resp, int timeout_ms);

}  // namespace mrpc
