// rpc_press: load generator for any pb method (role of the reference's
// tools/rpc_press/rpc_press.cpp:27-46 flags + info_thread.cpp:60-80 output).
// With -proto empty it drives example.EchoService.Echo with -request_size
// bytes of message and -attachment_size bytes of attachment (HBM-resident
// with -device_attachment).
#include <cstdio>
#include <fstream>

#include "base/flags.h"
#include "base/logging.h"
#include "press/press.h"
#include "rpc/server.h"

DEFINE_int32(dummy_port, -1, "Start a builtin-service dummy server on this port (-1: off)");
DEFINE_string(proto, "", "user's .proto file (empty = built-in echo workload)");
DEFINE_string(inc, "", "include paths for -proto, separated by ';'");
DEFINE_string(method, "example.EchoService.Echo", "full method name");
DEFINE_string(server, "127.0.0.1:8002", "ip:port, or a naming service url when -lb_policy is set");
DEFINE_string(input, "", "file of json requests, or an inline json request");
DEFINE_string(lb_policy, "", "rr random wrr wr la c_murmurhash c_md5 c_ketama");
DEFINE_int32(thread_num, 0, "concurrent senders (0: 50 closed loop / derived from -qps)");
DEFINE_string(protocol, "baidu_std", "protocol name");
DEFINE_string(connection_type, "", "single | pooled | short");
DEFINE_int32(timeout_ms, 1000, "RPC timeout in ms");
DEFINE_int32(connection_timeout_ms, 500, "connect timeout in ms");
DEFINE_int32(max_retry, 3, "max retries");
DEFINE_int32(request_compress_type, 0, "0 none, 1 snappy, 2 gzip, 3 zlib");
DEFINE_int32(response_compress_type, 0, "0 none, 1 snappy, 2 gzip, 3 zlib");
DEFINE_int32(request_size, 32, "echo message bytes (built-in workload)");
DEFINE_string(body, "const", "echo message contents: const, text (log records) or random");
DEFINE_int32(attachment_size, 0, "attachment bytes per request");
DEFINE_bool(device_attachment, false, "keep the attachment in HBM (MI355X)");
DEFINE_int32(duration, 0, "seconds to run (0: until killed)");
DEFINE_double(qps, 0, "target qps (0: closed loop as fast as possible)");
DEFINE_int32(channels, 1, "independent channels (connections)");
DEFINE_bool(check, false, "verify echoed payloads");
DEFINE_bool(use_rdma, false, "move the connection onto RDMA verbs (server needs -use_rdma as well)");

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    mrpc::GlobalInitializeOrDie();
    if (FLAGS_dummy_port >= 0) mrpc::StartDummyServerAt(FLAGS_dummy_port);
    mrpc::press::PressOptions o;
    o.server = FLAGS_server;
    o.lb_policy = FLAGS_lb_policy;
    o.protocol = FLAGS_protocol;
    o.connection_type = FLAGS_connection_type;
    o.use_rdma = FLAGS_use_rdma;
    o.timeout_ms = FLAGS_timeout_ms;
    o.connect_timeout_ms = FLAGS_connection_timeout_ms;
    o.max_retry = FLAGS_max_retry;
    o.request_compress_type = FLAGS_request_compress_type;
    o.response_compress_type = FLAGS_response_compress_type;
    o.concurrency = FLAGS_thread_num;
    o.qps = FLAGS_qps;
    o.num_channels = FLAGS_channels;
    o.request_size = FLAGS_request_size;
    o.body = FLAGS_body;
    o.attachment_size = FLAGS_attachment_size;
    o.device_attachment = FLAGS_device_attachment;
    o.check_echo = FLAGS_check;
    o.proto_file = FLAGS_proto;
    o.include_paths = FLAGS_inc;
    o.method = FLAGS_method;
    o.input = FLAGS_input;
    mrpc::press::PressSession s;
    std::string err;
    if (s.Init(o, &err) != 0) {
        fprintf(stderr, "rpc_press: %s\n", err.c_str());
        return 1;
    }
    int64_t total_err = 0, total_sent = 0;
    s.RunFor(FLAGS_duration, [&](const mrpc::press::Snapshot& iv, const mrpc::press::Snapshot& tot) {
        total_err = tot.error;
        total_sent = tot.sent;
        printf("sent:%-10lld success:%-10lld error:%-6lld total_error:%-10lld total_sent:%-10lld qps:%.0f\n",
               (long long)iv.sent, (long long)iv.success, (long long)iv.error, (long long)tot.error,
               (long long)tot.sent, iv.qps);
        if (iv.error && !iv.last_error.empty()) printf("  last error: [E%d] %s\n", iv.last_error_code, iv.last_error.c_str());
        fflush(stdout);
    });
    mrpc::press::Snapshot st = s.Stats();
    printf("[Summary] sent:%lld success:%lld error:%lld elapsed:%.2fs qps:%.0f throughput:%.1fMB/s\n",
           (long long)st.sent, (long long)st.success, (long long)st.error, st.elapsed_s, st.qps,
           st.elapsed_s > 0 ? st.bytes / st.elapsed_s / 1e6 : 0.0);
    printf("%s", mrpc::press::FormatLatencyTable(st).c_str());
    return st.success > 0 ? 0 : 2;
}
