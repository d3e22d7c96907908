#include "press/press.h"

#include <fstream>
#include <sstream>

#include "base/crc32c.h"
#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "base/util.h"
#include "fiber/fiber.h"
#include "json/json.h"
#include "json/json2pb.h"
#include "mrpc/proto/echo.pb.h"
#include "pb/dynamic.h"
#include "pb/parser.h"
#include "gpu/gpu.h"
#include "gpu/hbm_pool.h"
#include "rpc/channel.h"
#include "rpc/combo_channels.h"
#include "rpc/controller.h"
#include "rpc/errno.h"

DEFINE_int32(press_slow_trace_us, 0,
             "record start time and latency of calls at least this slow (0: off; SlowCalls() returns them)");

namespace mrpc {
namespace press {

namespace {
std::mutex g_slow_mu;
std::vector<std::pair<int64_t, int64_t>> g_slow;  // (monotonic start us, latency us)
}  // namespace

void RecordSlowCall(int64_t t0_us, int64_t lat_us) {
    std::lock_guard<std::mutex> g(g_slow_mu);
    if (g_slow.size() < 100000) g_slow.emplace_back(t0_us, lat_us);
}

std::vector<std::pair<int64_t, int64_t>> TakeSlowCalls() {
    std::lock_guard<std::mutex> g(g_slow_mu);
    std::vector<std::pair<int64_t, int64_t>> out;
    out.swap(g_slow);
    return out;
}

// Per-worker state. Each worker owns its histograms; the lock is only
// contended when the 1-second ticker swaps the interval histogram out.
struct PressSession::Worker {
    PressSession* s = nullptr;
    int index = 0;
    std::mutex mu;
    var::LatencyHistogram total, interval;
    int64_t sent = 0, ok = 0, err = 0, bytes = 0;
    int64_t i_sent = 0, i_ok = 0, i_err = 0, i_bytes = 0;
    int last_code = 0;
    std::string last_error;
    std::map<int, std::pair<int64_t, std::string>> codes;  // error histogram
    std::atomic<int64_t>* remaining = nullptr;  // closed loop with a budget
    std::atomic<bool>* stop = nullptr;          // run-until-stopped
    int64_t deadline_us = 0;                    // closed loop: stop issuing after this (0: none)
    int64_t pace_us = 0;                        // open loop interval per sender
    fiber::fiber_t tid = 0;

    void add(int64_t lat, bool okk, int code, const std::string& etext, int64_t nbytes) {
        std::lock_guard<std::mutex> g(mu);
        ++sent;
        ++i_sent;
        if (okk) {
            ++ok;
            ++i_ok;
            bytes += nbytes;
            i_bytes += nbytes;
            total.add(lat);
            interval.add(lat);
        } else {
            ++err;
            ++i_err;
            last_code = code;
            last_error = etext;
            auto& c = codes[code];
            ++c.first;
            c.second = etext;
        }
    }
};

std::string EchoBody(const std::string& kind, size_t size) {
    std::string out;
    if (kind == "const") {
        out.assign(size, 'x');
        return out;
    }
    uint64_t q = 0x2545F4914F6CDD1Dull;
    auto next = [&q] {
        q ^= q << 13;
        q ^= q >> 7;
        q ^= q << 17;
        return q;
    };
    if (kind == "random") {
        out.resize(size);
        for (size_t i = 0; i < size; i += 8) {
            const uint64_t r = next();
            memcpy(&out[i], &r, std::min<size_t>(8, size - i));
        }
        return out;
    }
    if (kind != "text") return out;
    // service-log records: a timestamp, a level, small vocabularies, hex
    // ids and decimal numbers — repeated structure, high-entropy fields
    static const char* kLevels[] = {"INFO", "INFO", "INFO", "WARN", "DEBUG", "ERROR"};
    static const char* kPaths[] = {"/api/v1/items", "/api/v1/users", "/api/v2/search", "/healthz", "/api/v1/orders",
                                   "/static/app.js", "/api/v2/cart", "/login"};
    static const char* kUsers[] = {"alice", "bob", "carol", "dave", "erin", "frank", "grace", "heidi", "ivan", "judy"};
    static const char* kAgents[] = {"curl/8.5.0", "Mozilla/5.0 (X11; Linux x86_64)", "python-requests/2.31",
                                    "grpc-go/1.62.0"};
    out.reserve(size + 256);
    uint64_t ts = 1792242500000000ull;
    char line[384];
    while (out.size() < size) {
        ts += next() % 5000;
        const uint64_t r = next(), id = next();
        const int n = snprintf(line, sizeof(line),
                               "{\"ts\":%llu,\"level\":\"%s\",\"rank\":%u,\"req\":\"%016llx\",\"user\":\"%s\","
                               "\"path\":\"%s/%u\",\"status\":%u,\"latency_us\":%u,\"bytes\":%u,\"agent\":\"%s\"}\n",
                               (unsigned long long)ts, kLevels[r % 6], (unsigned)((r >> 8) % 8),
                               (unsigned long long)id, kUsers[(r >> 12) % 10], kPaths[(r >> 16) % 8],
                               (unsigned)((r >> 20) % 100000), (r >> 40) % 10 ? 200u : 404u,
                               (unsigned)((r >> 24) % 20000), (unsigned)((id >> 7) % 1000000),
                               kAgents[(r >> 44) % 4]);
        out.append(line, (size_t)n);
    }
    out.resize(size);
    return out;
}

PressSession::PressSession() {}

PressSession::~PressSession() {
    _channels.clear();
    if (_device_attachment) gpu::HbmFree(_device_attachment, _attachment.size(), _opt.gpu_device);
}

static bool read_file(const std::string& path, std::string* out) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return false;
    std::stringstream ss;
    ss << in.rdbuf();
    *out = ss.str();
    return true;
}

// Splits a file of concatenated json objects ("{..}{..}" or "[{..},{..}]" or
// one per line) into values (tools/rpc_press/json_loader.cpp semantics).
static bool load_json_requests(const std::string& text, std::vector<json::Value>* out, std::string* error) {
    json::Value v;
    if (json::Parse(text, &v, nullptr)) {
        if (v.is_array()) {
            for (auto& e : v.array()) out->push_back(e);
        } else {
            out->push_back(v);
        }
        return true;
    }
    // concatenated objects: scan braces outside strings
    size_t depth = 0, start = std::string::npos;
    bool in_str = false, esc = false;
    for (size_t i = 0; i < text.size(); ++i) {
        const char c = text[i];
        if (in_str) {
            if (esc) esc = false;
            else if (c == '\\') esc = true;
            else if (c == '"') in_str = false;
            continue;
        }
        if (c == '"') {
            in_str = true;
        } else if (c == '{') {
            if (depth++ == 0) start = i;
        } else if (c == '}') {
            if (depth == 0) {
                *error = "unbalanced '}' in json input";
                return false;
            }
            if (--depth == 0) {
                json::Value one;
                std::string perr;
                if (!json::Parse(text.substr(start, i - start + 1), &one, &perr)) {
                    *error = "bad json request: " + perr;
                    return false;
                }
                out->push_back(std::move(one));
            }
        }
    }
    if (out->empty()) {
        *error = "no json request found";
        return false;
    }
    return true;
}

int PressSession::Init(const PressOptions& opt, std::string* error) {
    _opt = opt;
    if (_opt.concurrency <= 0) _opt.concurrency = _opt.qps > 0 ? std::max(1, std::min(64, (int)(_opt.qps / 2000) + 1)) : 50;
    if (_opt.num_channels <= 0) _opt.num_channels = 1;
    ChannelOptions copt;
    copt.protocol = _opt.protocol;
    copt.connection_type = _opt.connection_type;
    copt.use_rdma = _opt.use_rdma;
    copt.timeout_ms = _opt.timeout_ms;
    copt.connect_timeout_ms = _opt.connect_timeout_ms;
    copt.max_retry = _opt.max_retry;
    copt.use_device_transport = _opt.device_attachment;
    copt.gpu_device = _opt.gpu_device;
    std::vector<std::string> fan;
    for (const std::string& f : split_string(_opt.fanout_servers, ',')) {
        if (!f.empty()) fan.push_back(f);
    }
    for (int i = 0; i < _opt.num_channels && !fan.empty(); ++i) {
        ParallelChannelOptions po;
        po.timeout_ms = _opt.timeout_ms;
        po.gather_response_attachments = true;  // echoes come back in channel order
        std::unique_ptr<ParallelChannel> pc(new ParallelChannel);
        pc->Init(&po);
        std::shared_ptr<CallMapper> mapper;
        if (_opt.scatter) mapper = std::make_shared<ScatterAttachmentMapper>();
        copt.connection_group = _opt.num_channels > 1 ? "press" + std::to_string(i) : std::string();
        for (const std::string& f : fan) {
            std::unique_ptr<Channel> sub(new Channel);
            if (sub->Init(f.c_str(), &copt) != 0) {
                *error = "fail to init channel to " + f;
                return -1;
            }
            pc->AddChannel(sub.release(), OWNS_CHANNEL, mapper, nullptr);
        }
        _channels.push_back(std::move(pc));
    }
    _fanout = fan.empty() ? 1 : (int)fan.size();
    for (int i = 0; i < _opt.num_channels && fan.empty(); ++i) {
        std::unique_ptr<Channel> ch(new Channel);
        // distinct groups => distinct "single" connections per channel
        copt.connection_group = _opt.num_channels > 1 ? "press" + std::to_string(i) : std::string();
        int rc = _opt.lb_policy.empty() ? ch->Init(_opt.server.c_str(), &copt)
                                        : ch->Init(_opt.server.c_str(), _opt.lb_policy.c_str(), &copt);
        if (rc != 0) {
            *error = "fail to init channel to " + _opt.server;
            return -1;
        }
        _channels.push_back(std::move(ch));
    }
    if (!_opt.proto_file.empty()) {
        std::vector<std::string> paths;
        for (auto& p : split_string(_opt.include_paths, ';')) {
            if (!p.empty()) paths.push_back(p);
        }
        std::string dir = ".";
        std::string file = _opt.proto_file;
        const size_t slash = file.rfind('/');
        if (slash != std::string::npos) {
            dir = file.substr(0, slash);
            file = file.substr(slash + 1);
        }
        paths.insert(paths.begin(), dir);
        _importer.reset(new pb::Importer(paths));
        if (!_importer->Import(file, error)) return -1;
        _method = _importer->FindMethodByName(_opt.method);
        if (!_method) {
            // accept "Service.Method" / "pkg.Service/Method"
            std::string m = _opt.method;
            std::replace(m.begin(), m.end(), '/', '.');
            _method = _importer->FindMethodByName(m);
        }
        if (!_method) {
            *error = "no method named " + _opt.method + " in " + _opt.proto_file;
            return -1;
        }
        std::string text = _opt.input;
        if (!text.empty() && text[0] != '{' && text[0] != '[') {
            if (!read_file(_opt.input, &text)) {
                *error = "fail to read input file " + _opt.input;
                return -1;
            }
        }
        std::vector<json::Value> reqs;
        if (text.empty()) text = "{}";
        if (!load_json_requests(text, &reqs, error)) return -1;
        for (auto& v : reqs) {
            std::unique_ptr<pb::Message> m(_method->input_type->prototype->New());
            json2pb::Json2PbOptions jopt;
            if (!json2pb::JsonValueToProtoMessage(v, m.get(), jopt, error)) return -1;
            _requests.push_back(std::move(m));
        }
    } else {
        _echo_message = EchoBody(_opt.body, (size_t)std::max(0, _opt.request_size));
        if (_opt.request_size > 0 && _echo_message.empty()) {
            *error = "unknown body kind '" + _opt.body + "' (const, text or random)";
            return -1;
        }
        // ids of every varint length (1..10 bytes, a few negative)
        uint64_t q = 0xD1B54A32D192ED03ull;
        _ids.resize((size_t)std::max(0, _opt.packed_ids));
        for (int64_t& id : _ids) {
            q ^= q << 13;
            q ^= q >> 7;
            q ^= q << 17;
            id = (int64_t)(q >> (q % 57));
            if ((q & 0xff) == 0) id = -id;
        }
        if (_opt.attachment_size > 0) {
            if (!_opt.attachment_body.empty()) {
                _attachment = EchoBody(_opt.attachment_body, (size_t)_opt.attachment_size);
                if (_attachment.size() != (size_t)_opt.attachment_size) {
                    *error = "unknown attachment body kind '" + _opt.attachment_body + "' (const, text or random)";
                    return -1;
                }
            } else {
                _attachment.resize(_opt.attachment_size);
                uint64_t r = 0x9E3779B97F4A7C15ull;
                for (size_t i = 0; i < _attachment.size(); ++i) {
                    r ^= r << 13;
                    r ^= r >> 7;
                    r ^= r << 17;
                    _attachment[i] = (char)r;
                }
            }
            if (_opt.attachment_pb) {
                example::EchoRequest m;
                m.set_message(_attachment);
                _attachment.clear();
                m.SerializeToString(&_attachment);
            }
            char* blk = _attachment_buf.append_contiguous(_attachment.size());
            if (blk) memcpy(blk, _attachment.data(), _attachment.size());
            else _attachment_buf.append(_attachment);
            if (_opt.device_attachment) {
                if (gpu::Init(_opt.gpu_device, error) != 0) return -1;
                // arena memory: the xGMI transport lends it to the server
                // without a copy (gpu/xgmi.h)
                _device_attachment = gpu::HbmAlloc(_attachment.size(), _opt.gpu_device);
                if (!_device_attachment) {
                    *error = "fail to allocate the HBM attachment";
                    return -1;
                }
                if (gpu::CopyHostToDevice(_device_attachment, _attachment.data(), _attachment.size(),
                                          _opt.gpu_device) != 0) {
                    *error = "fail to upload the attachment to HBM";
                    return -1;
                }
            }
        }
    }
    return 0;
}

// One in-flight call; heap-allocated for the open-loop (async) path.
struct PressCall : public Closure {
    PressSession* s = nullptr;
    PressSession::Worker* w = nullptr;
    std::atomic<int64_t>* inflight = nullptr;
    Controller cntl;
    example::EchoRequest echo_req;
    example::EchoResponse echo_res;
    std::unique_ptr<pb::Message> res;
    int64_t t0 = 0;
    int64_t nbytes = 0;
    bool check = false;
    void Run() override;
};

void PressSession::issue(Worker* w, int64_t seq, PressCall* call, bool async) {
    ChannelBase* ch = _channels[w->index % _channels.size()].get();
    Controller& cntl = call->cntl;
    if (_opt.request_compress_type) cntl.set_request_compress_type((CompressType)_opt.request_compress_type);
    if (_opt.response_compress_type) cntl.set_response_compress_type((CompressType)_opt.response_compress_type);
    // with a load balancer the sequence number is the routing key
    // (consistent-hash balancers send a key to the server owning its shard)
    if (!_opt.lb_policy.empty()) cntl.set_request_code((uint64_t)seq * 0x9E3779B97F4A7C15ull);
    call->s = this;
    call->w = w;
    call->t0 = monotonic_us();
    Closure* done = async ? call : nullptr;
    if (_method) {
        const pb::Message& req = *_requests[seq % _requests.size()];
        call->res.reset(_method->output_type->prototype->New());
        ch->CallMethod(_method, &cntl, &req, call->res.get(), done);
        return;
    }
    call->echo_req.set_message(_echo_message);
    if (_opt.gpu_process) call->echo_req.set_gpu_process(true);
    if (_opt.cpu_process) call->echo_req.set_cpu_process(true);
    if (call->echo_req.ids_size() != (int)_ids.size()) *call->echo_req.mutable_ids() = _ids;
    if (_device_attachment) {
        gpu::AppendDevice(&cntl.request_attachment(), _device_attachment, _attachment.size(), _opt.gpu_device);
        if (_opt.device_compress) cntl.set_device_payload_compress_type((CompressType)_opt.device_compress);
        if (_opt.device_scan) cntl.set_device_payload_scan(true);
        if (_opt.verify_device_payload) cntl.set_verify_device_payload(true);
    } else if (!_attachment.empty()) {
        // one shared block, appended by reference like rpc_press's IOBuf
        // attachment (tools/rpc_press/rpc_press_impl.cpp): no per-call copy
        cntl.request_attachment().append(_attachment_buf);
    }
    call->nbytes = _opt.scatter ? 2 * (int64_t)(_echo_message.size() * _fanout + _attachment.size())
                                : 2 * (int64_t)(_echo_message.size() + _attachment.size()) * _fanout;
    call->nbytes += 2 * (int64_t)(_ids.size() * sizeof(int64_t));
    call->check = _opt.check_echo && (_opt.check_every <= 1 || seq % _opt.check_every == 0);
    example::EchoService_Stub stub(ch);
    stub.Echo(&cntl, &call->echo_req, &call->echo_res, done);
}

void PressSession::finish(PressCall* call) {
    const int64_t lat = monotonic_us() - call->t0;
    if (FLAGS_press_slow_trace_us > 0 && lat >= FLAGS_press_slow_trace_us) RecordSlowCall(call->t0, lat);
    Controller& cntl = call->cntl;
    bool ok = !cntl.Failed();
    if (ok && call->check && !_method) {
        if (call->echo_res.message() != _echo_message) {
            ok = false;
            cntl.SetFailed(ERESPONSE, "echoed message mismatch");
        } else if (call->echo_res.ids() != _ids) {
            ok = false;
            cntl.SetFailed(ERESPONSE, "echoed ids mismatch (%d of %zu)", call->echo_res.ids_size(), _ids.size());
        } else if (!_attachment.empty()) {
            std::string got, want;
            if (_opt.scatter) {
                want = _attachment;  // slices gathered back in channel order
            } else {
                for (int k = 0; k < _fanout; ++k) want += _attachment;  // gathered in channel order
            }
            const DevicePayloadIndex& ix = cntl.device_payload_index();
            if (gpu::CopyBufToHost(cntl.response_attachment(), &got) != 0 || got != want) {
                ok = false;
                cntl.SetFailed(ERESPONSE, "echoed attachment mismatch (%zu bytes)", got.size());
            } else if (_device_attachment && _opt.device_scan && _fanout == 1 &&
                       !cntl.response_attachment().all_host_accessible() &&
                       (ix.nfields != 1 || ix.fields.size() < 2 || ix.fields[0] != ((1u << 3) | 2) ||
                        (ix.fields[1] & 0xffffffffu) != (uint64_t)(_attachment.size() - (ix.fields[1] >> 32)))) {
                // the reply's device field table: one length-delimited field 1
                // running to the end of the message
                ok = false;
                cntl.SetFailed(ERESPONSE, "device pb index of the echoed attachment is wrong (nfields %d)", ix.nfields);
            } else if ((_opt.gpu_process || _opt.cpu_process) &&
                       call->echo_res.crc32c() != crc32c::Value(want.data(), want.size())) {
                ok = false;
                cntl.SetFailed(ERESPONSE, "device CRC32C 0x%08x does not match the host's", call->echo_res.crc32c());
            }
        }
    }
    call->w->add(lat, ok, cntl.ErrorCode(), ok ? std::string() : cntl.ErrorText(), call->nbytes);
}

void PressCall::Run() {
    s->finish(this);
    std::atomic<int64_t>* f = inflight;
    delete this;
    if (f) f->fetch_sub(1, std::memory_order_release);
}

// Closed-loop worker: one synchronous call at a time.
static void* closed_loop(void* arg) {
    PressSession::Worker* w = static_cast<PressSession::Worker*>(arg);
    PressSession* s = w->s;
    int64_t seq = w->index;
    for (;;) {
        if (w->remaining) {
            if (w->deadline_us && monotonic_us() >= w->deadline_us) break;
            if (w->remaining->fetch_sub(1, std::memory_order_relaxed) <= 0) break;
        } else if (w->stop->load(std::memory_order_relaxed)) {
            break;
        }
        PressCall call;
        s->issue(w, seq++, &call, false);
        s->finish(&call);
        // a refused write fails at once: back off instead of spinning the
        // worker (which would starve the fibers that drain the socket)
        if (call.cntl.ErrorCode() == EOVERCROWDED) fiber::usleep(200);
    }
    return nullptr;
}

// Open-loop sender: one async call every pace_us, independent of replies
// (rpc_press -qps semantics; latency includes queueing at the server).
static void* open_loop(void* arg) {
    PressSession::Worker* w = static_cast<PressSession::Worker*>(arg);
    PressSession* s = w->s;
    int64_t seq = w->index;
    int64_t next = monotonic_us() + (int64_t)(fast_rand() % (uint64_t)std::max<int64_t>(1, w->pace_us));
    while (!w->stop->load(std::memory_order_relaxed)) {
        const int64_t now = monotonic_us();
        if (now < next) {
            fiber::usleep(next - now);
            continue;
        }
        next += w->pace_us;
        if (next < now - 1000000) next = now;  // do not burst after a long stall
        PressCall* call = new PressCall;
        call->inflight = s->inflight();
        s->inflight()->fetch_add(1, std::memory_order_relaxed);
        s->issue(w, seq++, call, true);
    }
    return nullptr;
}

void PressSession::collect(std::vector<std::unique_ptr<Worker>>& ws) {
    std::lock_guard<std::mutex> g(_mu);
    for (auto& w : ws) {
        std::lock_guard<std::mutex> g2(w->mu);
        _hist.merge(w->total);
        _sent += w->sent;
        _ok += w->ok;
        _err += w->err;
        _bytes += w->bytes;
        if (w->last_code) {
            _last_code = w->last_code;
            _last_error = w->last_error;
        }
        for (const auto& kv : w->codes) {
            auto& c = _error_codes[kv.first];
            c.first += kv.second.first;
            c.second = kv.second.second;
        }
    }
}

int64_t PressSession::RunRequests(int64_t n, int64_t deadline_us) {
    if (_channels.empty() || n <= 0) return -1;
    std::atomic<int64_t> remaining{n};
    const int nw = (int)std::min<int64_t>(_opt.concurrency, n);
    std::vector<std::unique_ptr<Worker>> ws;
    const int64_t t0 = monotonic_us();
    for (int i = 0; i < nw; ++i) {
        ws.emplace_back(new Worker);
        Worker* w = ws.back().get();
        w->s = this;
        w->index = i;
        w->remaining = &remaining;
        w->deadline_us = deadline_us;
    }
    for (auto& w : ws) {
        fiber::Attr attr(fiber::STACK_NORMAL, fiber::ATTR_NOSIGNAL);
        if (fiber::start_background(&w->tid, &attr, closed_loop, w.get()) != 0) {
            closed_loop(w.get());
            w->tid = 0;
        }
    }
    fiber::flush();
    for (auto& w : ws) {
        if (w->tid) fiber::join(w->tid);
    }
    collect(ws);
    std::lock_guard<std::mutex> g(_mu);
    _busy_s += (monotonic_us() - t0) / 1e6;
    return std::max<int64_t>(0, remaining.load(std::memory_order_relaxed));
}

int PressSession::RunFor(double seconds,
                         const std::function<void(const Snapshot& interval, const Snapshot& total)>& tick) {
    if (_channels.empty()) return -1;
    std::atomic<bool> stop{false};
    const int nw = std::max(1, _opt.concurrency);
    std::vector<std::unique_ptr<Worker>> ws;
    const bool open = _opt.qps > 0;
    for (int i = 0; i < nw; ++i) {
        ws.emplace_back(new Worker);
        Worker* w = ws.back().get();
        w->s = this;
        w->index = i;
        w->stop = &stop;
        if (open) w->pace_us = std::max<int64_t>(1, (int64_t)(1e6 * nw / _opt.qps));
    }
    const int64_t t0 = monotonic_us();
    for (auto& w : ws) {
        fiber::Attr attr(fiber::STACK_NORMAL, fiber::ATTR_NOSIGNAL);
        fiber::start_background(&w->tid, &attr, open ? open_loop : closed_loop, w.get());
    }
    fiber::flush();
    const int64_t end = seconds > 0 ? t0 + (int64_t)(seconds * 1e6) : INT64_MAX;
    int64_t last = t0;
    var::LatencyHistogram run_hist;
    int64_t rs = 0, rok = 0, rerr = 0, rbytes = 0;
    for (;;) {
        int64_t now = monotonic_us();
        if (now >= end) break;
        const int64_t wake = std::min(end, last + 1000000);
        if (wake > now) {
            timespec ts{(time_t)((wake - now) / 1000000), (long)((wake - now) % 1000000) * 1000};
            nanosleep(&ts, nullptr);
        }
        now = monotonic_us();
        if (!tick) {
            last = now;
            continue;
        }
        var::LatencyHistogram ih;
        int64_t s = 0, ok = 0, er = 0, by = 0;
        int code = 0;
        std::string etext;
        for (auto& w : ws) {
            std::lock_guard<std::mutex> g(w->mu);
            ih.merge(w->interval);
            w->interval.clear();
            s += w->i_sent;
            ok += w->i_ok;
            er += w->i_err;
            by += w->i_bytes;
            w->i_sent = w->i_ok = w->i_err = w->i_bytes = 0;
            if (w->last_code) {
                code = w->last_code;
                etext = w->last_error;
            }
        }
        run_hist.merge(ih);
        rs += s;
        rok += ok;
        rerr += er;
        rbytes += by;
        Snapshot iv = summarize(ih, s, ok, er, by, (now - last) / 1e6);
        Snapshot tot = summarize(run_hist, rs, rok, rerr, rbytes, (now - t0) / 1e6);
        iv.last_error_code = tot.last_error_code = code;
        iv.last_error = tot.last_error = etext;
        tick(iv, tot);
        last = now;
    }
    stop.store(true);
    for (auto& w : ws) fiber::join(w->tid);
    // drain async calls
    while (_inflight.load(std::memory_order_acquire) > 0) {
        timespec ts{0, 200000};
        nanosleep(&ts, nullptr);
    }
    collect(ws);
    std::lock_guard<std::mutex> g(_mu);
    _busy_s += (monotonic_us() - t0) / 1e6;
    return 0;
}

Snapshot PressSession::summarize(const var::LatencyHistogram& h, int64_t sent, int64_t ok, int64_t err,
                                 int64_t bytes, double secs) const {
    Snapshot s;
    s.sent = sent;
    s.success = ok;
    s.error = err;
    s.bytes = bytes;
    s.elapsed_s = secs;
    s.qps = secs > 0 ? ok / secs : 0;
    s.avg_us = h.mean();
    s.min_us = h.min();
    s.p50_us = h.percentile(0.5);
    s.p70_us = h.percentile(0.7);
    s.p90_us = h.percentile(0.9);
    s.p95_us = h.percentile(0.95);
    s.p97_us = h.percentile(0.97);
    s.p99_us = h.percentile(0.99);
    s.p999_us = h.percentile(0.999);
    s.p9999_us = h.percentile(0.9999);
    s.max_us = h.max();
    return s;
}

Snapshot PressSession::Stats() const {
    std::lock_guard<std::mutex> g(_mu);
    Snapshot s = summarize(_hist, _sent, _ok, _err, _bytes, _busy_s);
    s.last_error_code = _last_code;
    s.last_error = _last_error;
    s.error_codes = _error_codes;
    return s;
}

void PressSession::ResetStats() {
    std::lock_guard<std::mutex> g(_mu);
    _hist.clear();
    _sent = _ok = _err = _bytes = 0;
    _busy_s = 0;
    _last_code = 0;
    _last_error.clear();
    _error_codes.clear();
}

std::string FormatLatencyTable(const Snapshot& s) {
    char buf[1024];
    snprintf(buf, sizeof(buf),
             "[Latency]\n"
             "  avg     %10.0f us\n  50%%     %10lld us\n  70%%     %10lld us\n  90%%     %10lld us\n"
             "  95%%     %10lld us\n  97%%     %10lld us\n  99%%     %10lld us\n  99.9%%   %10lld us\n"
             "  99.99%%  %10lld us\n  max     %10lld us\n",
             s.avg_us, (long long)s.p50_us, (long long)s.p70_us, (long long)s.p90_us, (long long)s.p95_us,
             (long long)s.p97_us, (long long)s.p99_us, (long long)s.p999_us, (long long)s.p9999_us,
             (long long)s.max_us);
    return buf;
}

}  // namespace press
}  // namespace mrpc
