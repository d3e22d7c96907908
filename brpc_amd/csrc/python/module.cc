// pybind11 bindings: the Python face of the native runtime (bench.py,
// tests, and torch-side GPU ops). Every call that can block drops the GIL.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <sstream>
#include <unistd.h>

#include "base/crc32c.h"
#include "builtin/cpu_profiler.h"
#include "base/snappy.h"
#include "base/flags.h"
#include "base/logging.h"
#include "fiber/fiber.h"
#include "gpu/gpu.h"
#include "gpu/copy_engine.h"
#include "rpc/compress.h"
#include "gpu/hbm_pool.h"
#include "gpu/snappy_offload.h"
#include "gpu/json_offload.h"
#include "gpu/codec_batch.h"
#include "gpu/device_codec.h"
#include "json/json2pb.h"
#include "pb/descriptor.h"
#include "pb/parser.h"
#include "gpu/xgmi.h"
#include "policy/device_payload.h"
#include "gpu/rccl_plane.h"
#include "rdma/rdma.h"
#include "mrpc/proto/echo.pb.h"
#include "base/time.h"
#include "press/press.h"
#include "press/stream_press.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/protocol.h"
#include "rpc/server.h"
#include "rpc/span.h"
#include "rpc/span_db.h"
#include "services/echo_service.h"
#include "var/variable.h"

namespace py = pybind11;

DECLARE_string(rdma_verbs_library);
using namespace mrpc;

void bind_gpu_ops(py::module_& m);  // gpu_ops.cc

namespace {

class PyServer {
public:
    PyServer() { GlobalInitializeOrDie(); }
    ~PyServer() { stop(); }
    void add_echo_service() {
        if (!_echo) {
            _echo.reset(new EchoServiceImpl);
            if (_server.AddService(_echo.get(), SERVER_DOESNT_OWN_SERVICE) != 0) throw std::runtime_error("AddService failed");
        }
    }
    int start(const std::string& addr, int num_threads, int gpu_device, int idle_timeout_s, bool use_rdma,
              int max_concurrency) {
        ServerOptions opt;
        opt.num_threads = num_threads;
        if (max_concurrency > 0) opt.max_concurrency = max_concurrency;
        if (_echo) _echo->set_gpu_device(gpu_device);
        opt.gpu_device = gpu_device;
        opt.idle_timeout_sec = idle_timeout_s;
        opt.use_rdma = use_rdma;
        int rc;
        {
            py::gil_scoped_release nogil;
            rc = addr.find(':') == std::string::npos ? _server.Start(std::stoi(addr), &opt)
                                                     : _server.Start(addr.c_str(), &opt);
        }
        if (rc != 0) throw std::runtime_error("fail to start server on " + addr);
        _running = true;
        return _server.listen_address().port;
    }
    void stop() {
        if (!_running) return;
        py::gil_scoped_release nogil;
        _server.Stop(0);
        _server.Join();
        _running = false;
    }
    int port() const { return _server.listen_address().port; }
    std::string address() const { return _server.listen_address().to_string(); }
    int64_t echo_calls() const { return _echo ? _echo->ncalls() : 0; }
    int64_t gpu_calls() const { return _echo ? _echo->gpu_calls() : 0; }

private:
    Server _server;
    std::unique_ptr<EchoServiceImpl> _echo;
    bool _running = false;
};

class PyChannel {
public:
    PyChannel(const std::string& server, const std::string& lb, const std::string& protocol,
              const std::string& connection_type, int timeout_ms, int max_retry) {
        GlobalInitializeOrDie();
        ChannelOptions o;
        o.protocol = protocol;
        o.connection_type = connection_type;
        o.timeout_ms = timeout_ms;
        o.max_retry = max_retry;
        const int rc = lb.empty() ? _ch.Init(server.c_str(), &o) : _ch.Init(server.c_str(), lb.c_str(), &o);
        if (rc != 0) throw std::runtime_error("fail to init channel to " + server);
    }
    // Returns (message, attachment, latency_us); raises on RPC failure.
    py::tuple echo(const std::string& message, py::bytes attachment, int64_t sleep_us) {
        example::EchoRequest req;
        example::EchoResponse res;
        Controller cntl;
        req.set_message(message);
        if (sleep_us > 0) req.set_sleep_us(sleep_us);
        std::string att = attachment;
        cntl.request_attachment().append(att);
        {
            py::gil_scoped_release nogil;
            example::EchoService_Stub stub(&_ch);
            stub.Echo(&cntl, &req, &res, nullptr);
        }
        if (cntl.Failed()) {
            throw std::runtime_error("[E" + std::to_string(cntl.ErrorCode()) + "] " + cntl.ErrorText());
        }
        return py::make_tuple(res.message(), py::bytes(cntl.response_attachment().to_string()), cntl.latency_us());
    }

private:
    Channel _ch;
};

press::PressOptions press_options(const py::dict& d) {
    press::PressOptions o;
    for (auto item : d) {
        const std::string k = py::str(item.first);
        py::handle v = item.second;
        if (k == "server") o.server = v.cast<std::string>();
        else if (k == "lb_policy") o.lb_policy = v.cast<std::string>();
        else if (k == "protocol") o.protocol = v.cast<std::string>();
        else if (k == "connection_type") o.connection_type = v.cast<std::string>();
        else if (k == "timeout_ms") o.timeout_ms = v.cast<int>();
        else if (k == "connect_timeout_ms") o.connect_timeout_ms = v.cast<int>();
        else if (k == "max_retry") o.max_retry = v.cast<int>();
        else if (k == "request_compress_type") o.request_compress_type = v.cast<int>();
        else if (k == "response_compress_type") o.response_compress_type = v.cast<int>();
        else if (k == "concurrency") o.concurrency = v.cast<int>();
        else if (k == "qps") o.qps = v.cast<double>();
        else if (k == "num_channels") o.num_channels = v.cast<int>();
        else if (k == "request_size") o.request_size = v.cast<int>();
        else if (k == "body") o.body = v.cast<std::string>();
        else if (k == "attachment_size") o.attachment_size = v.cast<int>();
        else if (k == "packed_ids") o.packed_ids = v.cast<int>();
        else if (k == "device_attachment") o.device_attachment = v.cast<bool>();
        else if (k == "attachment_body") o.attachment_body = v.cast<std::string>();
        else if (k == "attachment_pb") o.attachment_pb = v.cast<bool>();
        else if (k == "device_compress") o.device_compress = v.cast<int>();
        else if (k == "device_scan") o.device_scan = v.cast<bool>();
        else if (k == "verify_device_payload") o.verify_device_payload = v.cast<bool>();
        else if (k == "gpu_device") o.gpu_device = v.cast<int>();
        else if (k == "check_echo") o.check_echo = v.cast<bool>();
        else if (k == "fanout_servers") o.fanout_servers = v.cast<std::string>();
        else if (k == "scatter") o.scatter = v.cast<bool>();
        else if (k == "gpu_process") o.gpu_process = v.cast<bool>();
        else if (k == "cpu_process") o.cpu_process = v.cast<bool>();
        else if (k == "check_every") o.check_every = v.cast<int>();
        else if (k == "use_rdma") o.use_rdma = v.cast<bool>();
        else if (k == "proto_file") o.proto_file = v.cast<std::string>();
        else if (k == "include_paths") o.include_paths = v.cast<std::string>();
        else if (k == "method") o.method = v.cast<std::string>();
        else if (k == "input") o.input = v.cast<std::string>();
        else throw std::invalid_argument("unknown press option: " + k);
    }
    return o;
}

py::dict snapshot_dict(const press::Snapshot& s) {
    py::dict d;
    d["sent"] = s.sent;
    d["success"] = s.success;
    d["error"] = s.error;
    d["elapsed_s"] = s.elapsed_s;
    d["qps"] = s.qps;
    d["avg_us"] = s.avg_us;
    d["min_us"] = s.min_us;
    d["p50_us"] = s.p50_us;
    d["p70_us"] = s.p70_us;
    d["p90_us"] = s.p90_us;
    d["p95_us"] = s.p95_us;
    d["p97_us"] = s.p97_us;
    d["p99_us"] = s.p99_us;
    d["p999_us"] = s.p999_us;
    d["p9999_us"] = s.p9999_us;
    d["max_us"] = s.max_us;
    d["bytes"] = s.bytes;
    d["last_error_code"] = s.last_error_code;
    d["last_error"] = s.last_error;
    py::dict codes;
    for (const auto& kv : s.error_codes) codes[py::str(std::to_string(kv.first))] = py::make_tuple(kv.second.first, kv.second.second);
    d["error_codes"] = codes;
    return d;
}

class PyPress {
public:
    explicit PyPress(const py::dict& d) {
        GlobalInitializeOrDie();
        press::PressOptions o = press_options(d);
        std::string err;
        int rc;
        {
            py::gil_scoped_release nogil;
            rc = _s.Init(o, &err);
        }
        if (rc != 0) throw std::runtime_error("press init failed: " + err);
    }
    // Returns the calls never issued because max_seconds (>0) ran out
    // (0: all n ran).
    int64_t run_requests(int64_t n, double max_seconds) {
        py::gil_scoped_release nogil;
        const int64_t deadline = max_seconds > 0 ? monotonic_us() + (int64_t)(max_seconds * 1e6) : 0;
        return _s.RunRequests(n, deadline);
    }
    void run_for(double seconds) {
        py::gil_scoped_release nogil;
        _s.RunFor(seconds, nullptr);
    }
    py::dict stats() const { return snapshot_dict(_s.Stats()); }
    void reset_stats() { _s.ResetStats(); }

private:
    press::PressSession _s;
};

// Streaming-RPC throughput driver (press/stream_press.h).
class PyStreamPress {
public:
    explicit PyStreamPress(const py::dict& d) {
        GlobalInitializeOrDie();
        press::StreamPressOptions o;
        for (auto item : d) {
            const std::string k = py::str(item.first);
            py::handle v = item.second;
            if (k == "server") o.server = v.cast<std::string>();
            else if (k == "chunk_size") o.chunk_size = v.cast<int>();
            else if (k == "chunks_per_step") o.chunks_per_step = v.cast<int>();
            else if (k == "timeout_ms") o.timeout_ms = v.cast<int>();
            else if (k == "max_buf_size") o.max_buf_size = v.cast<int64_t>();
            else if (k == "pipeline_rounds") o.pipeline_rounds = v.cast<int>();
            else if (k == "device_chunks") o.device_chunks = v.cast<bool>();
            else if (k == "gpu_device") o.gpu_device = v.cast<int>();
            else if (k == "relay_chain") o.relay_chain = v.cast<std::string>();
            else throw std::invalid_argument("unknown stream press option: " + k);
        }
        _s.reset(new press::StreamPress);
        std::string err;
        int rc;
        {
            py::gil_scoped_release nogil;
            rc = _s->Init(o, &err);
        }
        if (rc != 0) throw std::runtime_error("stream press init failed: " + err);
    }
    // Steps completed; fewer than `steps` when max_seconds (>0) ran out
    // before the rest started.
    int run_steps(int steps, double max_seconds) {
        std::string err;
        int rc, done = 0;
        {
            py::gil_scoped_release nogil;
            const int64_t deadline = max_seconds > 0 ? monotonic_us() + (int64_t)(max_seconds * 1e6) : 0;
            rc = _s->RunSteps(steps, &err, deadline, &done);
        }
        if (rc != 0) throw std::runtime_error(err);
        return done;
    }
    py::dict stats() {
        py::dict d;
        d["bytes_sent"] = _s->bytes_sent();
        d["bytes_acked"] = _s->bytes_acked();
        d["steps"] = _s->steps_done();
        d["streams"] = _s->num_streams();
        return d;
    }
    void close() {
        py::gil_scoped_release nogil;
        _s.reset();
    }

private:
    std::unique_ptr<press::StreamPress> _s;
};

}  // namespace

PYBIND11_MODULE(_native, m) {
    m.doc() = "brpc_amd native runtime (fibers, RPC, press, MI355X device ops)";
    m.def("global_init", [] { GlobalInitializeOrDie(); });
    m.def("set_concurrency", [](int n) { return fiber::set_concurrency(n); });
    m.def("get_concurrency", [] { return fiber::get_concurrency(); });
    m.def("set_flag", [](const std::string& name, const std::string& value) {
        std::string err;
        if (!SetFlag(name, value, false, &err)) throw std::invalid_argument("set_flag " + name + ": " + err);
    });
    // placement on shared hosts: wake-up lateness per CPU, re-confinement
    m.def("probe_cpu_wake", [](const std::vector<int>& cpus, int duration_ms, int period_us, int threshold_us) {
        std::vector<fiber::CpuWakeProbe> r;
        {
            py::gil_scoped_release nogil;
            r = fiber::ProbeCpuWake(cpus, duration_ms, period_us, threshold_us);
        }
        py::list out;
        for (const auto& p : r) {
            py::dict d;
            d["cpu"] = p.cpu;
            d["wakes"] = p.wakes;
            d["late_p50_us"] = p.late_p50_us;
            d["late_p99_us"] = p.late_p99_us;
            d["late_max_us"] = p.late_max_us;
            d["late_over"] = p.late_over;
            d["run_delay_us"] = p.run_delay_us;
            d["nivcsw"] = p.nivcsw;
            out.append(d);
        }
        return out;
    }, py::arg("cpus"), py::arg("duration_ms") = 500, py::arg("period_us") = 1000, py::arg("threshold_us") = 150);
    m.def("rebind_l3_domain", [](int k) { return fiber::RebindL3Domain(k); });
    m.def("get_flag", [](const std::string& name) {
        std::string v;
        if (!GetFlag(name, &v)) throw std::invalid_argument("no flag " + name);
        return v;
    });
    // rpcz: recent spans (memory), spans by trace id / end time (disk store)
    m.def("press_slow_calls", [] { return press::TakeSlowCalls(); });
    // sampling CPU profile of the whole process (folded stacks), e.g. while a
    // press runs in another Python thread
    m.def("profile_cpu", [](double seconds, int hz) {
        std::string folded;
        int64_t n = 0;
        bool ok;
        {
            py::gil_scoped_release nogil;
            ok = profiler::ProfileCpu(seconds, hz, &folded, nullptr, &n);
        }
        if (!ok) throw std::runtime_error("another CPU profile is running");
        return py::make_tuple(folded, n);
    }, py::arg("seconds"), py::arg("hz") = 999);
    m.def("monotonic_us", [] { return monotonic_us(); });
    m.def("rpcz_recent", [](size_t max) { return ListRecentSpans(max, 0); }, py::arg("max") = 100);
    m.def("rpcz_trace", [](uint64_t trace, size_t max) { return span_db::FindTrace(trace, max); },
          py::arg("trace_id"), py::arg("max") = 100, py::call_guard<py::gil_scoped_release>());
    m.def("rpcz_before", [](int64_t before_us, size_t max) { return span_db::ListBefore(before_us, max); },
          py::arg("before_us") = 0, py::arg("max") = 100, py::call_guard<py::gil_scoped_release>());
    m.def("rpcz_flush", [] { span_db::Flush(); }, py::call_guard<py::gil_scoped_release>());
    m.def("rpcz_stats", [] {
        const span_db::Stats st = span_db::GetStats();
        py::dict d;
        d["written"] = st.written;
        d["dropped"] = st.dropped;
        d["indexed"] = st.indexed;
        d["files"] = st.files;
        d["bytes"] = st.bytes;
        d["reloaded"] = st.reloaded;
        d["dir"] = st.dir;
        return d;
    });
    m.def("list_flags", [] {
        py::dict d;
        for (auto& f : ListFlags()) d[py::str(f.name)] = f.current_value;
        return d;
    });
    m.def("dump_vars", [](const std::string& filter) {
        std::vector<std::pair<std::string, std::string>> out;
        var::Variable::dump_exposed(&out, filter);
        py::dict d;
        for (auto& kv : out) d[py::str(kv.first)] = kv.second;
        return d;
    }, py::arg("filter") = "");
    m.def("dump_prometheus", [] { return var::Variable::dump_prometheus(); });
    m.def("crc32c", [](py::bytes b) {
        std::string s = b;
        return crc32c::Value(s.data(), s.size());
    });
    // Host snappy codec (the CPU half; the GPU decompressor is gpu.snappy_*).
    m.def("echo_body", [](const std::string& kind, size_t size) { return py::bytes(press::EchoBody(kind, size)); });
    m.def("snappy_compress", [](py::bytes b) {
        std::string s = b, out;
        snappy::Compress(s.data(), s.size(), &out);
        return py::bytes(out);
    });
    m.def("snappy_uncompress", [](py::bytes b) {
        std::string s = b, out;
        if (!snappy::Uncompress(s.data(), s.size(), &out)) throw std::invalid_argument("malformed snappy stream");
        return py::bytes(out);
    });
    // The body codec registry (rpc/compress.h) exactly as protocols call it:
    // a registered offload (GPU snappy) applies here too.
    // JSON -> message (type from a .proto loaded at run time) -> JSON, plus
    // the message's wire bytes and the JSON of those bytes parsed back —
    // parity checks against the reference's own JSON fixtures
    m.def("json_proto_roundtrip", [](const std::string& proto_dir, const std::string& proto_file,
                                     const std::string& type_name, py::bytes text, bool base64_to_bytes) {
        pb::Importer imp({proto_dir});
        std::string err;
        if (!imp.Import(proto_file, &err)) throw std::runtime_error("import " + proto_file + ": " + err);
        const pb::Descriptor* d = imp.FindMessageTypeByName(type_name);
        if (!d || !d->prototype) throw std::invalid_argument("unknown message type " + type_name);
        std::unique_ptr<pb::Message> msg(d->prototype->New());
        std::unique_ptr<pb::Message> back(d->prototype->New());
        std::string in = text, out, wire, out2;
        json2pb::Json2PbOptions jo;
        jo.base64_to_bytes = base64_to_bytes;
        json2pb::Pb2JsonOptions po;
        po.bytes_to_base64 = base64_to_bytes;
        bool ok;
        {
            py::gil_scoped_release nogil;
            ok = json2pb::JsonToProtoMessage(in, msg.get(), jo, &err) &&
                 json2pb::ProtoMessageToJson(*msg, &out, po, &err) && msg->SerializeToString(&wire) &&
                 back->ParseFromString(wire) && json2pb::ProtoMessageToJson(*back, &out2, po, &err);
        }
        if (!ok) throw std::runtime_error(err);
        return py::make_tuple(out, py::bytes(wire), out2);
    }, py::arg("proto_dir"), py::arg("proto_file"), py::arg("type_name"), py::arg("json"),
       py::arg("base64_to_bytes") = false);
    // JsonToProtoMessage's verdict and error text (soft errors of optional
    // fields come back with ok=True), plus the message as JSON
    m.def("json_proto_parse", [](const std::string& proto_dir, const std::string& proto_file,
                                 const std::string& type_name, py::bytes text, bool base64_to_bytes) {
        pb::Importer imp({proto_dir});
        std::string err;
        if (!imp.Import(proto_file, &err)) throw std::runtime_error("import " + proto_file + ": " + err);
        const pb::Descriptor* d = imp.FindMessageTypeByName(type_name);
        if (!d || !d->prototype) throw std::invalid_argument("unknown message type " + type_name);
        std::unique_ptr<pb::Message> msg(d->prototype->New());
        std::string in = text, out, err2;
        json2pb::Json2PbOptions jo;
        jo.base64_to_bytes = base64_to_bytes;
        const bool ok = json2pb::JsonToProtoMessage(in, msg.get(), jo, &err);
        json2pb::Pb2JsonOptions po;
        po.bytes_to_base64 = base64_to_bytes;
        if (ok) json2pb::ProtoMessageToJson(*msg, &out, po, &err2);
        return py::make_tuple(ok, err, out);
    }, py::arg("proto_dir"), py::arg("proto_file"), py::arg("type_name"), py::arg("json"),
       py::arg("base64_to_bytes") = true);
    // wire bytes -> message -> JSON: ProtoMessageToJson's verdict and error
    // (a missing required field is one) plus the JSON
    m.def("json_proto_from_wire", [](const std::string& proto_dir, const std::string& proto_file,
                                     const std::string& type_name, py::bytes wire, bool bytes_to_base64) {
        pb::Importer imp({proto_dir});
        std::string err;
        if (!imp.Import(proto_file, &err)) throw std::runtime_error("import " + proto_file + ": " + err);
        const pb::Descriptor* d = imp.FindMessageTypeByName(type_name);
        if (!d || !d->prototype) throw std::invalid_argument("unknown message type " + type_name);
        std::unique_ptr<pb::Message> msg(d->prototype->New());
        const std::string in = wire;
        if (!msg->ParsePartialFromArray(in.data(), in.size())) throw std::runtime_error("bad wire bytes for " + type_name);
        std::string out;
        json2pb::Pb2JsonOptions po;
        po.bytes_to_base64 = bytes_to_base64;
        const bool ok = json2pb::ProtoMessageToJson(*msg, &out, po, &err);
        return py::make_tuple(ok, err, out);
    }, py::arg("proto_dir"), py::arg("proto_file"), py::arg("type_name"), py::arg("wire"),
       py::arg("bytes_to_base64") = false);
    m.def("json_to_pb_to_json", [](const std::string& type_name, py::bytes text) {
        const pb::Descriptor* d = pb::DescriptorPool::generated_pool()->FindMessageTypeByName(type_name);
        if (!d || !d->prototype) throw std::invalid_argument("unknown message type " + type_name);
        std::unique_ptr<pb::Message> msg(d->prototype->New());
        std::string in = text, err, out;
        bool ok;
        {
            py::gil_scoped_release nogil;
            ok = json2pb::JsonToProtoMessage(in, msg.get(), json2pb::Json2PbOptions(), &err) &&
                 json2pb::ProtoMessageToJson(*msg, &out, json2pb::Pb2JsonOptions(), &err);
        }
        if (!ok) throw std::runtime_error(err);
        return out;
    });
    m.def("compress", [](int type, py::bytes b) {
        std::string s = b;
        Buf in(s), out;
        bool ok;
        {
            py::gil_scoped_release nogil;
            ok = CompressBuf((CompressType)type, in, &out);
        }
        if (!ok) throw std::invalid_argument("compression failed");
        return py::bytes(out.to_string());
    });
    m.def("decompress", [](int type, py::bytes b) {
        std::string s = b;
        Buf in(s), out;
        bool ok;
        {
            py::gil_scoped_release nogil;
            ok = DecompressBuf((CompressType)type, in, &out);
        }
        if (!ok) throw std::invalid_argument("decompression failed");
        return py::bytes(out.to_string());
    });
    m.def("fiber_stats", [] {
        py::dict d;
        d["fibers"] = fiber::fiber_count();
        d["switches"] = fiber::switch_count();
        d["steals"] = fiber::steal_count();
        d["workers"] = fiber::get_concurrency();
        return d;
    });

    py::class_<PyServer>(m, "Server")
        .def(py::init<>())
        .def("add_echo_service", &PyServer::add_echo_service)
        .def("start", &PyServer::start, py::arg("addr"), py::arg("num_threads") = -1, py::arg("gpu_device") = -1,
             py::arg("idle_timeout_s") = -1, py::arg("use_rdma") = false, py::arg("max_concurrency") = 0)
        .def("stop", &PyServer::stop)
        .def_property_readonly("port", &PyServer::port)
        .def_property_readonly("address", &PyServer::address)
        .def_property_readonly("echo_calls", &PyServer::echo_calls)
        .def_property_readonly("gpu_calls", &PyServer::gpu_calls);

    py::class_<PyChannel>(m, "Channel")
        .def(py::init<const std::string&, const std::string&, const std::string&, const std::string&, int, int>(),
             py::arg("server"), py::arg("lb") = "", py::arg("protocol") = "baidu_std",
             py::arg("connection_type") = "", py::arg("timeout_ms") = 1000, py::arg("max_retry") = 3)
        .def("echo", &PyChannel::echo, py::arg("message"), py::arg("attachment") = py::bytes(),
             py::arg("sleep_us") = 0);

    py::class_<PyStreamPress>(m, "StreamPress")
        .def(py::init<const py::dict&>())
        .def("run_steps", &PyStreamPress::run_steps, py::arg("steps"), py::arg("max_seconds") = 0.0)
        .def("stats", &PyStreamPress::stats)
        .def("close", &PyStreamPress::close);

    py::class_<PyPress>(m, "Press")
        .def(py::init<const py::dict&>())
        .def("run_requests", &PyPress::run_requests, py::arg("n"), py::arg("max_seconds") = 0.0)
        .def("run_for", &PyPress::run_for)
        .def("stats", &PyPress::stats)
        .def("reset_stats", &PyPress::reset_stats);

    py::module_ g = m.def_submodule("gpu", "MI355X device runtime");
    g.def("device_count", [] { return gpu::DeviceCount(); });
    g.def("available", [] { return gpu::Available(); });
    g.def("init", [](int dev) {
        std::string err;
        if (gpu::Init(dev, &err) != 0) throw std::runtime_error(err);
    }, py::arg("device") = -1);
    g.def("device_arch", [](int dev) { return gpu::DeviceArch(dev); }, py::arg("device") = 0);
    g.def("device_name", [](int dev) { return gpu::DeviceName(dev); }, py::arg("device") = 0);
    g.def("pci_bus_id", [](int dev) { return gpu::PciBusId(dev); }, py::arg("device") = 0);
    g.def("polled_events", [] { return gpu::PolledEvents(); });
    g.def("enable_xgmi", [](int dev) {
        std::string err;
        if (gpu::EnableXgmiTransport(dev, &err) != 0) throw std::runtime_error(err);
    }, py::arg("device") = 0);
    g.def("xgmi_stats", [] {
        const gpu::XgmiStats s = gpu::GetXgmiStats();
        py::dict d;
        d["sent_bytes"] = s.sent_bytes;
        d["recv_bytes"] = s.recv_bytes;
        d["sent_payloads"] = s.sent_payloads;
        d["recv_payloads"] = s.recv_payloads;
        d["ring_full_fallbacks"] = s.ring_full_fallbacks;
        d["crc_failures"] = s.crc_failures;
        d["lent_outstanding"] = s.lent_outstanding;
        d["copied_into_arena"] = s.copied_into_arena;
        d["released_unconsumed"] = s.released_unconsumed;
        d["cross_device_payloads"] = s.cross_device_payloads;
        d["cross_device_bytes"] = s.cross_device_bytes;
        d["cross_device_pull_failures"] = s.cross_device_pull_failures;
        d["peer_access_enabled"] = s.peer_access_enabled;
        d["attach_failures"] = s.attach_failures;
        d["peer_maps"] = s.peer_maps;
        d["compressed_sent"] = s.compressed_sent;
        d["compressed_recv"] = s.compressed_recv;
        d["compress_skipped_raw"] = s.compress_skipped_raw;
        d["compress_failures"] = s.compress_failures;
        d["compress_skipped_adaptive"] = s.compress_skipped_adaptive;
        int64_t staged = 0, staged_bytes = 0;
        GetStagedStats(&staged, &staged_bytes);
        d["staged_payloads"] = staged;
        d["staged_bytes"] = staged_bytes;
        const gpu::CopyEngineStats c = gpu::GetCopyEngineStats();
        d["copy_submits"] = c.submits;
        d["copy_launches"] = c.launches;
        d["copy_segments"] = c.segments;
        d["copy_bytes"] = c.bytes;
        d["copy_queue_us"] = c.queue_us;
        d["copy_api_us"] = c.api_us;
        d["copy_gpu_us"] = c.gpu_us;
        d["copy_wake_us"] = c.wake_us;
        d["copy_kernel_ticks"] = c.kernel_ticks;
        d["copy_kernel_timed"] = c.kernel_timed;
        d["copy_start_delay_us"] = c.start_delay_us;
        d["copy_notice_us"] = c.notice_us;
        return d;
    });
    g.def("reap_lent", [] { gpu::ReapLentBlocks(); });
    // RCCL data plane (gpu/rccl_plane.h): collective init from every rank
    g.def("rccl_unique_id", [] {
        std::string err;
        std::string id = gpu::rccl::UniqueId(&err);
        if (id.empty()) throw std::runtime_error(err);
        return py::bytes(id);
    });
    g.def("rccl_init", [](int rank, int world, py::bytes uid, int dev) {
        std::string err, id = uid;
        int rc;
        {
            py::gil_scoped_release nogil;  // blocks until every rank joined
            rc = gpu::rccl::Init(rank, world, id, dev, &err);
        }
        if (rc != 0) throw std::runtime_error(err);
    }, py::arg("rank"), py::arg("world"), py::arg("unique_id"), py::arg("device"));
    // GPUDirect RDMA registration of REAL HBM (arena memory) through the HIP
    // dmabuf export (hipMemGetHandleForAddressRange) and the ibverbs
    // provider loaded from `verbs_library` (the stub on hosts without an HCA)
    g.def("dmabuf_register_probe", [](const std::string& verbs_library, size_t nbytes, int dev) {
        py::dict d;
        std::string err;
        if (gpu::Init(dev, &err) != 0 || gpu::InitHbmPool(dev, &err) != 0) throw std::runtime_error(err);
        Buf hold;
        void* p = gpu::AppendNewDeviceBlock(&hold, nbytes, dev);
        if (!p) throw std::runtime_error("no HBM");
        d["arena_offset"] = gpu::ArenaOffset(p, dev);
        // the export itself: a dmabuf fd naming the HBM range
        int fd = -1;
        uint64_t off = 0;
        rdma::DmabufExportFn ex = rdma::GetDmabufExportHook();
        d["export_rc"] = ex ? ex(p, nbytes, dev, &fd, &off) : -100;
        d["export_offset"] = off;
        std::string kind;
        if (fd >= 0) {
            char link[256] = {0};
            const std::string path = "/proc/self/fd/" + std::to_string(fd);
            const ssize_t n = readlink(path.c_str(), link, sizeof(link) - 1);
            if (n > 0) kind.assign(link, (size_t)n);
            close(fd);
        }
        d["fd_target"] = kind;
        // registration through the provider (ibv_reg_dmabuf_mr)
        FLAGS_rdma_verbs_library = verbs_library;
        std::string why;
        std::unique_ptr<rdma::Provider> pr = rdma::CreateIbverbsProvider(&why);
        d["provider"] = pr ? std::string(pr->name()) : "none: " + why;
        if (pr) {
            uint32_t lkey = 0;
            d["register_rc"] = pr->RegisterMemory(p, nbytes, true, dev, &lkey);
            d["lkey"] = lkey;
            pr->DeregisterMemory(p);
        }
        return d;
    }, py::arg("verbs_library"), py::arg("nbytes") = 1 << 20, py::arg("device") = 0);
    g.def("rccl_active", [] { return gpu::rccl::Active(); });
    g.def("rccl_abort_for_test", [](const std::string& why) { gpu::rccl::AbortForTest(why); });
    g.def("rccl_shutdown", [] {
        py::gil_scoped_release nogil;
        gpu::rccl::Shutdown();
    });
    g.def("rccl_stats", [] {
        const gpu::rccl::Stats s = gpu::rccl::GetStats();
        py::dict d;
        d["sent_payloads"] = s.sent_payloads;
        d["sent_bytes"] = s.sent_bytes;
        d["recv_payloads"] = s.recv_payloads;
        d["recv_bytes"] = s.recv_bytes;
        d["discarded"] = s.discarded;
        d["rounds"] = s.rounds;
        d["payload_rounds"] = s.payload_rounds;
        d["pair_rounds"] = s.pair_rounds;
        d["withdrawals"] = s.withdrawals;
        d["group_us"] = s.group_us;
        d["aborts"] = s.aborts;
        d["credit_stalls"] = s.credit_stalls;
        d["stash_expired"] = s.stash_expired;
        d["recv_timeouts"] = s.recv_timeouts;
        d["doorbells"] = s.doorbells;
        d["withdrawn"] = s.withdrawn;
        d["stash_payloads"] = s.stash_payloads;
        d["stash_bytes"] = s.stash_bytes;
        d["world"] = s.world;
        d["host_memory"] = s.host_memory;
        return d;
    });
    // packed_only (-gpu_snappy_packed_only): the device codec takes only
    // messages with large packed numeric fields; False forces every snappy
    // body of at least min_bytes onto the device (the A/B and the tests)
    g.def("enable_snappy", [](int dev, size_t min_bytes, bool packed_only) {
        std::string err;
        SetFlag("gpu_snappy_packed_only", packed_only ? "true" : "false");
        if (gpu::EnableGpuSnappy(dev, min_bytes, &err) != 0) throw std::runtime_error(err);
    }, py::arg("device") = 0, py::arg("min_bytes") = 32768, py::arg("packed_only") = true);
    g.def("disable_snappy", [] { gpu::DisableGpuSnappy(); });
    g.def("snappy_stats", [] {
        const gpu::GpuSnappyStats s = gpu::GetGpuSnappyStats();
        py::dict d;
        d["compress_calls"] = s.compress_calls;
        d["decompress_calls"] = s.decompress_calls;
        d["fallbacks"] = s.fallbacks;
        d["indexed_parses"] = s.indexed_parses;
        d["plain_routed"] = s.plain_routed;
        d["index_fallbacks"] = s.index_fallbacks;
        d["packs"] = s.packs;
        d["pack_runs"] = s.pack_runs;
        d["pack_run_chunks"] = s.pack_run_chunks;
        d["unpack_runs"] = s.unpack_runs;
        d["unpack_fallbacks"] = s.unpack_fallbacks;
        return d;
    });
    g.def("device_codec_stats", [] {
        const gpu::DeviceCodecStats s = gpu::GetDeviceCodecStats();
        py::dict d;
        d["encodes"] = s.encodes;
        d["encoded_bytes"] = s.encoded_bytes;
        d["encoded_out_bytes"] = s.encoded_out_bytes;
        d["decodes"] = s.decodes;
        d["decoded_bytes"] = s.decoded_bytes;
        d["bad_tables"] = s.bad_tables;
        d["decode_errors"] = s.decode_errors;
        d["scans"] = s.scans;
        d["packed_runs"] = s.packed_runs;
        d["packed_bytes"] = s.packed_bytes;
        d["packed_elems"] = s.packed_elems;
        d["packed_errors"] = s.packed_errors;
        return d;
    });
    g.def("codec_batch_stats", [] {
        const gpu::CodecBatchStats s = gpu::GetCodecBatchStats();
        py::dict d;
        d["requests"] = s.requests;
        d["launches"] = s.launches;
        d["run_chunks"] = s.run_chunks;
        d["decode_chunks"] = s.decode_chunks;
        d["fused_launches"] = s.fused_launches;
        d["timed"] = s.timed;
        d["queue_us"] = s.queue_us;
        d["api_us"] = s.api_us;
        d["gpu_us"] = s.gpu_us;
        d["wake_us"] = s.wake_us;
        return d;
    });
    // numeric run (vector layout bytes) -> varints / JSON numbers on the device (tests)
    g.def("pb_run_encode", [](py::bytes values, size_t n, uint32_t kind, uint32_t format, int dev) {
        std::string v = values;
        std::string out;
        int rc;
        {
            py::gil_scoped_release nogil;
            rc = gpu::EncodeRunOnDevice(v.data(), n, kind, format, &out, dev);
        }
        if (rc != 0) throw std::runtime_error("pb_run_encode failed");
        return py::bytes(out);
    }, py::arg("values"), py::arg("n"), py::arg("kind"), py::arg("format") = 0, py::arg("device") = 0);
    g.def("pb_run_decode", [](py::bytes payload, uint32_t kind, int dev) {
        std::string v = payload;
        std::string out;
        int rc;
        {
            py::gil_scoped_release nogil;
            rc = gpu::DecodeRunOnDevice(v.data(), v.size(), kind, &out, dev);
        }
        if (rc != 0) throw std::runtime_error("pb_run_decode failed (malformed run or device error)");
        return py::bytes(out);
    }, py::arg("payload"), py::arg("kind"), py::arg("device") = 0);
    g.def("enable_json_index", [](int dev, size_t min_bytes) {
        std::string err;
        if (gpu::EnableGpuJsonIndex(dev, min_bytes, &err) != 0) throw std::runtime_error(err);
    }, py::arg("device") = 0, py::arg("min_bytes") = 65536);
    g.def("disable_json_index", [] { gpu::DisableGpuJsonIndex(); });
    g.def("json_stats", [] {
        const gpu::GpuJsonStats s = gpu::GetGpuJsonStats();
        py::dict d;
        d["indexed_bodies"] = s.indexed_bodies;
        d["indexed_bytes"] = s.indexed_bytes;
        d["failures"] = s.failures;
        d["pb2json_arrays"] = s.pb2json_arrays;
        d["pb2json_elems"] = s.pb2json_elems;
        d["pb2json_failures"] = s.pb2json_failures;
        d["int_arrays"] = s.int_arrays;
        d["int_array_fallbacks"] = s.int_array_fallbacks;
        d["sparse_skips"] = s.sparse_skips;
        return d;
    });
    // host bytes -> structural positions through the device (tests)
    g.def("json_index_bytes", [](py::bytes b, int dev) {
        std::string data = b;
        std::vector<uint32_t> pos;
        int rc;
        {
            py::gil_scoped_release nogil;
            rc = gpu::JsonIndex(data.data(), data.size(), &pos, dev);
        }
        if (rc != 0) throw std::runtime_error("json index failed (device error or unterminated string)");
        return pos;
    }, py::arg("data"), py::arg("device") = 0);
    g.def("hbm_pool_stats", [](int dev) {
        const gpu::HbmPoolStats s = gpu::GetHbmPoolStats(dev);
        py::dict d;
        d["arena_bytes"] = s.arena_bytes;
        d["carved_bytes"] = s.carved_bytes;
        d["live_blocks"] = s.live_blocks;
        d["live_bytes"] = s.live_bytes;
        d["fallback_allocs"] = s.fallback_allocs;
        d["splits"] = s.splits;
        d["pinned_bytes"] = gpu::PinnedBytes();
        d["pinned_blocks_in_use"] = gpu::PinnedBlocksInUse();
        return d;
    }, py::arg("device") = 0);
    bind_gpu_ops(g);
}
