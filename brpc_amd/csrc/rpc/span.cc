#include "rpc/span.h"

#include <deque>

#include "base/flags.h"
#include "base/time.h"
#include "base/util.h"
#include "fiber/fiber.h"
#include "fiber/internal.h"
#include "mrpc/proto/rpcz.pb.h"
#include "rpc/controller.h"
#include "rpc/span_db.h"

DEFINE_bool(enable_rpcz, false, "collect rpcz spans (browse at /rpcz)");
DEFINE_int32(rpcz_max_spans, 10000, "max spans kept in memory");
DEFINE_int32(rpcz_max_spans_per_second, 5000, "sampling speed limit of spans");
DEFINE_bool(rpcz_save_to_disk, true, "also append spans to the on-disk store (rpc/span_db.h)");
MRPC_VALIDATE_FLAG(enable_rpcz, ::mrpc::PassValidator);

namespace mrpc {

namespace {
struct Store {
    std::mutex mu;
    std::deque<Span*> spans;
    int64_t second = 0;
    int in_second = 0;
};
Store& store() {
    static Store* s = new Store;
    return *s;
}
thread_local Span* tls_span = nullptr;
}  // namespace

bool IsRpczEnabled() { return FLAGS_enable_rpcz; }

uint64_t NewTraceId() {
    uint64_t v;
    do {
        v = fast_rand();
    } while (v == 0);
    return v;
}

Span::~Span() {
    for (Span* c : client_spans) delete c;
}

Span* Span::CreateClientSpan(const std::string& name, int64_t base_real_us) {
    if (!FLAGS_enable_rpcz) return nullptr;
    Span* s = new Span;
    s->type = CLIENT;
    s->full_method_name = name;
    Span* parent = tls_parent();
    if (parent) {
        s->trace_id = parent->trace_id;
        s->parent_span_id = parent->span_id;
        s->local_parent = parent;
    } else {
        s->trace_id = NewTraceId();
    }
    s->span_id = NewTraceId();
    s->start_send_real_us = base_real_us;
    return s;
}

Span* Span::CreateServerSpan(uint64_t trace_id, uint64_t span_id, uint64_t parent_span_id, const std::string& name,
                             int64_t base_real_us) {
    if (!FLAGS_enable_rpcz) return nullptr;
    Span* s = new Span;
    s->type = SERVER;
    s->trace_id = trace_id ? trace_id : NewTraceId();
    s->span_id = span_id ? span_id : NewTraceId();
    s->parent_span_id = parent_span_id;
    s->full_method_name = name;
    s->received_real_us = base_real_us;
    return s;
}

void Span::EndClientSpan(Span* s, const Controller* cntl) {
    s->error_code = cntl->ErrorCode();
    s->remote_side = cntl->remote_side();
    s->received_real_us = realtime_us();
}

void Span::Submit(Span* s, int64_t) {
    if (!s) return;
    if (s->local_parent && s->type == CLIENT) {
        // attach to the server span that issued it (kept with the parent)
        s->local_parent->client_spans.push_back(s);
        return;
    }
    Store& st = store();
    std::lock_guard<std::mutex> g(st.mu);
    const int64_t sec = monotonic_us() / 1000000;
    if (sec != st.second) {
        st.second = sec;
        st.in_second = 0;
    }
    if (++st.in_second > FLAGS_rpcz_max_spans_per_second) {
        delete s;
        return;
    }
    if (FLAGS_rpcz_save_to_disk) {
        SpanRecord* r = new SpanRecord;
        s->ToRecord(r);
        span_db::Submit(r);
    }
    st.spans.push_front(s);
    while ((int)st.spans.size() > FLAGS_rpcz_max_spans) {
        delete st.spans.back();
        st.spans.pop_back();
    }
}

Span* Span::tls_parent() {
    fiber::TaskGroup* g = fiber::tls_group();
    if (g && !g->is_current_main_task()) return static_cast<Span*>(g->current_task()->span);
    return tls_span;
}

void Span::set_tls_parent(Span* s) {
    fiber::TaskGroup* g = fiber::tls_group();
    if (g && !g->is_current_main_task()) {
        g->current_task()->span = s;
        return;
    }
    tls_span = s;
}

void Span::Annotate(const std::string& text) { annotations.emplace_back(realtime_us(), text); }

void Span::AnnotateDevice(const std::string& what, float device_ms) {
    annotations.emplace_back(realtime_us(), string_printf("[gpu] %s %.3f ms", what.c_str(), device_ms));
}

void Span::ToRecord(SpanRecord* r) const {
    r->set_trace_id(trace_id);
    r->set_span_id(span_id);
    r->set_parent_span_id(parent_span_id);
    r->set_log_id(log_id);
    r->set_type(type);
    r->set_remote(remote_side.to_string());
    r->set_full_method_name(full_method_name);
    r->set_protocol(protocol);
    r->set_error_code(error_code);
    r->set_request_size(request_size);
    r->set_response_size(response_size);
    r->set_received_real_us(received_real_us);
    r->set_start_parse_real_us(start_parse_real_us);
    r->set_start_callback_real_us(start_callback_real_us);
    r->set_start_send_real_us(start_send_real_us);
    r->set_sent_real_us(sent_real_us);
    for (auto& a : annotations) {
        SpanAnnotation* x = r->add_annotations();
        x->set_realtime_us(a.first);
        x->set_text(a.second);
    }
    for (const Span* c : client_spans) c->ToRecord(r->add_client_spans());
}

std::string Span::Describe() const {
    std::string out = string_printf("%s trace=%016llx span=%016llx parent=%016llx %s %s err=%d req=%lld res=%lld",
                                    type == SERVER ? "S" : "C", (unsigned long long)trace_id,
                                    (unsigned long long)span_id, (unsigned long long)parent_span_id,
                                    full_method_name.c_str(), remote_side.to_string().c_str(), error_code,
                                    (long long)request_size, (long long)response_size);
    if (type == SERVER) {
        string_appendf(&out, " received=%lld parse=+%lld callback=+%lld send=+%lld sent=+%lld", (long long)received_real_us,
                       (long long)(start_parse_real_us - received_real_us),
                       (long long)(start_callback_real_us - received_real_us),
                       (long long)(start_send_real_us - received_real_us), (long long)(sent_real_us - received_real_us));
    } else {
        string_appendf(&out, " latency=%lldus start=%lld", (long long)(received_real_us - start_send_real_us),
                       (long long)start_send_real_us);
        if (sent_real_us) string_appendf(&out, " sent=+%lld", (long long)(sent_real_us - start_send_real_us));
        if (cut_real_us) string_appendf(&out, " cut=+%lld", (long long)(cut_real_us - start_send_real_us));
        if (start_parse_real_us) string_appendf(&out, " parse=+%lld", (long long)(start_parse_real_us - start_send_real_us));
    }
    for (auto& a : annotations) string_appendf(&out, "\n    %lld %s", (long long)a.first, a.second.c_str());
    for (const Span* c : client_spans) out += "\n  " + c->Describe();
    return out;
}

std::vector<std::string> ListRecentSpans(size_t max, uint64_t trace_id) {
    std::vector<std::string> out;
    Store& st = store();
    std::lock_guard<std::mutex> g(st.mu);
    for (Span* s : st.spans) {
        if (trace_id && s->trace_id != trace_id) continue;
        out.push_back(s->Describe());
        if (out.size() >= max) break;
    }
    return out;
}

}  // namespace mrpc
