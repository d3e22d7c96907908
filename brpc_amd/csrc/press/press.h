// Load generator behind the rpc_press tool and bench.py (role of the
// reference's tools/rpc_press/rpc_press_impl.{h,cpp} + info_thread.cpp).
//
// Differences from the reference, by design:
//  * senders are fibers, not pthreads: `concurrency` closed-loop workers (or
//    paced open-loop senders in qps mode) all live on the M:N runtime, so a
//    1-GPU box's CPU share is not burnt on idle threads;
//  * latencies go into an exact log-linear histogram (var::LatencyHistogram)
//    per worker and are merged at the end, so p99/p99.9 are exact to 1/64;
//  * RunRequests(n) issues exactly n calls and returns, which is the unit a
//    benchmark "step" is made of (bench.py times K such steps);
//  * echo payloads may be device-resident (HBM) attachments that travel the
//    xGMI transport (ChannelOptions::use_device_transport).
#pragma once

#include <atomic>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "base/buf.h"
#include "var/percentile.h"

namespace mrpc {

class ChannelBase;
namespace pb {
class Message;
class MethodDescriptor;
class Importer;
}  // namespace pb

namespace press {

struct PressOptions {
    std::string server = "127.0.0.1:8002";  // ip:port, or naming-service url when lb_policy set
    std::string lb_policy;
    std::string protocol = "baidu_std";
    std::string connection_type;  // single | pooled | short
    int timeout_ms = 1000;
    int connect_timeout_ms = 500;
    int max_retry = 3;
    int request_compress_type = 0;
    int response_compress_type = 0;
    int concurrency = 50;  // closed-loop workers (or open-loop senders)
    double qps = 0;        // >0: open loop paced at this rate; 0: closed loop
    int num_channels = 1;  // independent channels (connections for "single")
    // echo workload (used when proto_file is empty)
    int request_size = 32;     // bytes in EchoRequest.message
    // contents of EchoRequest.message (EchoBody): "const" (one repeated
    // byte: the best case for any compressor), "text" (log/JSON-like
    // records, ~2-4x snappy-compressible), "random" (incompressible bytes)
    std::string body = "const";
    int attachment_size = 0;   // bytes of attachment per request
    int packed_ids = 0;        // int64 ids per request (EchoRequest.ids, a packed varint run), echoed back
    bool device_attachment = false;  // attachment lives in HBM (needs GPU)
    // attachment contents: "" (pseudo-random bytes), or an EchoBody kind
    // ("const", "text", "random")
    std::string attachment_body;
    // the attachment is one serialized EchoRequest whose message is that
    // body (a protobuf the receiver can index on the device: device_scan)
    bool attachment_pb = false;
    // device attachments: snappy-encode on the device before lending
    // (Controller::set_device_payload_compress_type; the server mirrors it)
    int device_compress = 0;
    // device attachments: the receiver pb_scan-indexes the payload (the
    // server mirrors it; check_echo verifies the reply's field table)
    bool device_scan = false;
    // device attachments: CRC32C-verified on the device by the receiver
    bool verify_device_payload = false;
    int gpu_device = -1;
    bool check_echo = false;   // verify the echoed payload
    int check_every = 1;       // ... of every n-th call (bench legs sample; tests check all)
    bool gpu_process = false;  // ask the server to run the attachment through its GPU
    bool cpu_process = false;  // ask the server to checksum the attachment on its CPU
    bool use_rdma = false;     // verbs data plane (server needs use_rdma too)
    // Fan-out (ParallelChannel, the DP analog of SURVEY §2.10): every call is
    // broadcast to all of these comma-separated servers — on one node the
    // xGMI-direct channels to the peer GPUs — and the echoed attachments are
    // gathered. Empty: plain calls to `server`.
    std::string fanout_servers;
    // With fanout_servers: scatter instead of broadcast — server i gets the
    // i-th slice of the attachment (ScatterAttachmentMapper, the TP analog)
    // and the echoed slices are gathered back in order.
    bool scatter = false;
    // generic workload (dynamic messages)
    std::string proto_file;    // .proto path
    std::string include_paths; // ';' separated
    std::string method = "example.EchoService.Echo";
    std::string input;         // file with json requests, or inline json
};

struct PressCall;

// The echo message of `size` bytes for a body kind (see PressOptions::body);
// deterministic. Empty string for an unknown kind.
std::string EchoBody(const std::string& kind, size_t size);

struct Snapshot {
    int64_t sent = 0;
    int64_t success = 0;
    int64_t error = 0;
    double elapsed_s = 0;
    double qps = 0;             // successes per second over elapsed_s
    double avg_us = 0;
    int64_t p50_us = 0, p70_us = 0, p90_us = 0, p95_us = 0, p97_us = 0;
    int64_t p99_us = 0, p999_us = 0, p9999_us = 0, max_us = 0, min_us = 0;
    int64_t bytes = 0;          // request+response payload bytes moved
    int last_error_code = 0;
    std::string last_error;
    // failed calls by error code, each with the text of its latest failure
    // (rpc_press prints error counts next to every latency line:
    // tools/rpc_press/info_thread.cpp:60-92)
    std::map<int, std::pair<int64_t, std::string>> error_codes;
};

class PressSession {
public:
    PressSession();
    ~PressSession();
    // Returns 0 on success, else fills *error.
    int Init(const PressOptions& opt, std::string* error);
    // Closed loop: issue exactly n calls over `concurrency` workers, return
    // when all finished. Stats accumulate until ResetStats(). With a
    // deadline (monotonic us, 0: none) workers stop issuing once it passed
    // and the calls in flight finish (each bounded by timeout_ms): returns
    // the number of calls never issued (0 when all n ran), -1 on misuse.
    int64_t RunRequests(int64_t n, int64_t deadline_us = 0);
    // Run for `seconds` (closed loop, or paced when qps>0); `tick` gets the
    // per-interval snapshot every second (rpc_press's info thread).
    int RunFor(double seconds, const std::function<void(const Snapshot& interval, const Snapshot& total)>& tick);
    Snapshot Stats() const;
    void ResetStats();
    const PressOptions& options() const { return _opt; }

    struct Worker;
    // internal (used by the worker fibers)
    void issue(Worker* w, int64_t seq, PressCall* call, bool async);
    void finish(PressCall* call);
    std::atomic<int64_t>* inflight() { return &_inflight; }

private:
    void collect(std::vector<std::unique_ptr<Worker>>& ws);
    Snapshot summarize(const var::LatencyHistogram& h, int64_t sent, int64_t ok, int64_t err, int64_t bytes,
                       double secs) const;

    PressOptions _opt;
    std::vector<std::unique_ptr<ChannelBase>> _channels;
    int _fanout = 1;  // sub calls per call
    // generic mode
    std::unique_ptr<pb::Importer> _importer;
    const pb::MethodDescriptor* _method = nullptr;
    std::vector<std::unique_ptr<pb::Message>> _requests;
    std::string _echo_message;
    std::string _attachment;
    std::vector<int64_t> _ids;  // EchoRequest.ids of every call
    Buf _attachment_buf;                 // _attachment as one shared block
    void* _device_attachment = nullptr;  // HBM copy of _attachment when device_attachment

    mutable std::mutex _mu;
    var::LatencyHistogram _hist;
    int64_t _sent = 0, _ok = 0, _err = 0, _bytes = 0;
    double _busy_s = 0;
    int _last_code = 0;
    std::string _last_error;
    std::map<int, std::pair<int64_t, std::string>> _error_codes;
    std::atomic<int64_t> _inflight{0};
};

// Formats the latency table the way rpc_press prints it.
std::string FormatLatencyTable(const Snapshot& s);

// Diagnostics: calls slower than -press_slow_trace_us, as (monotonic start
// us, latency us); taking them clears the list.
void RecordSlowCall(int64_t t0_us, int64_t lat_us);
std::vector<std::pair<int64_t, int64_t>> TakeSlowCalls();

}  // namespace press
}  // namespace mrpc
