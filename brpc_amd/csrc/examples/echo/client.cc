// Echo client (the reference's example/echo_c++/client.cpp): one synchronous
// call per -interval_ms, logging latency and the echoed attachment size.
#include <unistd.h>

#include <cstdio>

#include "base/flags.h"
#include "base/logging.h"
#include "mrpc/proto/echo.pb.h"
#include "rpc/channel.h"
#include "rpc/controller.h"

DEFINE_string(server, "127.0.0.1:8002", "IP address of server");
DEFINE_string(load_balancer, "", "load balancer name (with a naming service url in -server)");
DEFINE_string(protocol, "baidu_std", "protocol");
DEFINE_string(connection_type, "", "single | pooled | short");
DEFINE_string(attachment, "", "carry this along with requests");
DEFINE_int32(timeout_ms, 100, "RPC timeout in ms");
DEFINE_int32(max_retry, 3, "max retries");
DEFINE_int32(interval_ms, 1000, "milliseconds between consecutive requests");
DEFINE_int32(count, -1, "number of requests (-1: forever)");

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    mrpc::Channel channel;
    mrpc::ChannelOptions options;
    options.protocol = FLAGS_protocol;
    options.connection_type = FLAGS_connection_type;
    options.timeout_ms = FLAGS_timeout_ms;
    options.max_retry = FLAGS_max_retry;
    const int rc = FLAGS_load_balancer.empty()
                       ? channel.Init(FLAGS_server.c_str(), &options)
                       : channel.Init(FLAGS_server.c_str(), FLAGS_load_balancer.c_str(), &options);
    if (rc != 0) {
        LOG(ERROR) << "Fail to initialize channel";
        return -1;
    }
    example::EchoService_Stub stub(&channel);
    int failures = 0;
    for (int i = 0; FLAGS_count < 0 || i < FLAGS_count; ++i) {
        example::EchoRequest request;
        example::EchoResponse response;
        mrpc::Controller cntl;
        request.set_message("hello world");
        cntl.request_attachment().append(FLAGS_attachment);
        stub.Echo(&cntl, &request, &response, nullptr);
        if (!cntl.Failed()) {
            LOG(INFO) << "Received response from " << cntl.remote_side() << ": " << response.message()
                      << " (attached=" << cntl.response_attachment().size() << ")"
                      << " latency=" << cntl.latency_us() << "us";
        } else {
            ++failures;
            LOG(WARNING) << cntl.ErrorText();
        }
        if (FLAGS_interval_ms > 0) usleep(FLAGS_interval_ms * 1000L);
    }
    return failures ? 1 : 0;
}
