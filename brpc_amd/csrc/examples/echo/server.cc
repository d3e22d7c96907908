// Echo server (the reference's example/echo_c++/server.cpp workload): echoes
// message + attachment; -gpu_device routes HBM attachments through the GPU
// echo handler (checksum on device, response stays in HBM).
#include <csignal>
#include <unistd.h>

#include <cstdio>

#include "base/flags.h"
#include "base/logging.h"
#include "fiber/fiber.h"
#include "rpc/server.h"
#include "services/echo_service.h"

DEFINE_int32(port, 8002, "TCP port of this server");
DEFINE_string(listen_addr, "", "ip:port / unix:path; overrides -port");
DEFINE_int32(idle_timeout_s, -1, "close connections idle this long (-1: never)");
DEFINE_int32(num_threads, -1, "fiber worker pthreads (-1: default)");
DEFINE_int32(gpu_device, -1, "GPU ordinal for device attachments (-1: host only)");

static volatile sig_atomic_t g_quit = 0;
static void on_signal(int) { g_quit = 1; }

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    mrpc::Server server;
    mrpc::EchoServiceImpl echo;
    if (server.AddService(&echo, mrpc::SERVER_DOESNT_OWN_SERVICE) != 0) {
        LOG(ERROR) << "Fail to add service";
        return -1;
    }
    mrpc::ServerOptions opt;
    opt.idle_timeout_sec = FLAGS_idle_timeout_s;
    opt.num_threads = FLAGS_num_threads;
    opt.gpu_device = FLAGS_gpu_device;
    const int rc = FLAGS_listen_addr.empty() ? server.Start(FLAGS_port, &opt)
                                             : server.Start(FLAGS_listen_addr.c_str(), &opt);
    if (rc != 0) {
        LOG(ERROR) << "Fail to start EchoServer";
        return -1;
    }
    printf("EchoServer listening on %s\n", server.listen_address().to_string().c_str());
    fflush(stdout);
    signal(SIGINT, on_signal);
    signal(SIGTERM, on_signal);
    while (!g_quit) usleep(100000);
    server.Stop(0);
    server.Join();
    return 0;
}
