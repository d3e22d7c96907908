// rpcz tracing spans (role of src/brpc/span.h/.cpp, builtin/rpcz_service).
// Client spans are created in Channel::CallMethod, server spans in protocol
// process functions; trace/span ids propagate through RpcMeta. Spans are
// kept in an in-memory, speed-limited store (the reference indexes into
// leveldb, which is not available here) and browsed at /rpcz.
// MI355X-native: annotations carry HIP event timestamps of device work
// (copies / kernels) executed on behalf of the call (gpu/stream_wait.h).
#pragma once

#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "base/endpoint.h"

namespace mrpc {

class Controller;
class SpanRecord;

class Span {
public:
    enum Type { SERVER = 0, CLIENT = 1 };
    static Span* CreateClientSpan(const std::string& full_method_name, int64_t base_real_us);
    static Span* CreateServerSpan(uint64_t trace_id, uint64_t span_id, uint64_t parent_span_id,
                                  const std::string& full_method_name, int64_t base_real_us);
    static void EndClientSpan(Span* s, const Controller* cntl);
    // Hand over to the store (or delete if rpcz is off).
    static void Submit(Span* s, int64_t end_us);
    // TRACEPRINTF target: the span bound to the current fiber.
    static Span* tls_parent();
    static void set_tls_parent(Span* s);

    void Annotate(const std::string& text);
    void AnnotateDevice(const std::string& what, float device_ms);
    std::string Describe() const;
    void ToRecord(SpanRecord* r) const;

    uint64_t trace_id = 0, span_id = 0, parent_span_id = 0, log_id = 0;
    Type type = CLIENT;
    EndPoint remote_side;
    std::string full_method_name;
    int protocol = 0;
    int error_code = 0;
    int64_t request_size = 0, response_size = 0;
    // server: received = request cut from the socket, parse, callback,
    // send (response), sent. client: start_send = call start, sent = request
    // handed to the socket, cut = response cut from the socket, parse =
    // response processing began, received = call ended.
    int64_t received_real_us = 0, start_parse_real_us = 0, start_callback_real_us = 0, start_send_real_us = 0,
            sent_real_us = 0, cut_real_us = 0;
    std::vector<std::pair<int64_t, std::string>> annotations;
    std::vector<Span*> client_spans;
    Span* local_parent = nullptr;
    ~Span();
};

bool IsRpczEnabled();
uint64_t NewTraceId();
// Recent spans (most recent first), optionally filtered by trace id.
std::vector<std::string> ListRecentSpans(size_t max, uint64_t trace_id = 0);

}  // namespace mrpc

#define TRACEPRINTF(fmt, ...)                                                          \
    do {                                                                               \
        ::mrpc::Span* _mrpc_span = ::mrpc::Span::tls_parent();                         \
        if (_mrpc_span) _mrpc_span->Annotate(::mrpc::string_printf(fmt, ##__VA_ARGS__)); \
    } while (0)
