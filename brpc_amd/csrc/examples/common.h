// Shared helpers of the self-contained examples (each example starts the
// servers it needs in-process, runs its client, prints what happened and
// exits 0 on success, so `build/bin/<example>_main` is both a demo and a
// smoke test). Mirrors the reference's example/* programs.
#pragma once

#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <string>

#include "base/flags.h"
#include "base/logging.h"
#include "fiber/fiber.h"
#include "mrpc/proto/echo.pb.h"
#include "rpc/channel.h"
#include "rpc/controller.h"
#include "rpc/errno.h"
#include "rpc/server.h"

namespace demo {

// Echo that tags responses with the server's name and honors sleep_us /
// server_fail, like the fault-injecting servers of the reference's tests.
class TaggedEcho : public example::EchoService {
public:
    explicit TaggedEcho(std::string tag, int delay_us = 0) : _tag(std::move(tag)), _delay_us(delay_us) {}
    void Echo(mrpc::RpcController* c, const example::EchoRequest* req, example::EchoResponse* res,
              mrpc::Closure* done) override {
        mrpc::ClosureGuard g(done);
        mrpc::Controller* cntl = static_cast<mrpc::Controller*>(c);
        if (req->sleep_us() > 0) mrpc::fiber::usleep((uint64_t)req->sleep_us());
        if (_delay_us > 0) mrpc::fiber::usleep((uint64_t)_delay_us);
        if (req->server_fail()) {
            cntl->SetFailed(mrpc::EINTERNAL, "asked to fail");
            return;
        }
        res->set_message(req->message() + "@" + _tag);
        cntl->response_attachment().append(cntl->request_attachment());
    }

private:
    std::string _tag;
    int _delay_us;
};

struct LocalServer {
    mrpc::Server server;
    TaggedEcho echo;
    explicit LocalServer(const std::string& tag, int delay_us = 0, mrpc::ServerOptions opt = mrpc::ServerOptions())
        : echo(tag, delay_us) {
        server.AddService(&echo, mrpc::SERVER_DOESNT_OWN_SERVICE);
        if (server.Start("127.0.0.1:0", &opt) != 0) LOG(FATAL) << "fail to start " << tag;
    }
    std::string addr() const { return "127.0.0.1:" + std::to_string(server.listen_port()); }
};

// A crashing demo prints where it crashed (no debugger on the test boxes).
inline void CrashHandler(int sig) {
    void* frames[64];
    const int n = backtrace(frames, 64);
    fprintf(stderr, "*** signal %d, backtrace:\n", sig);
    backtrace_symbols_fd(frames, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}
struct CrashHandlerInstaller {
    CrashHandlerInstaller() {
        signal(SIGSEGV, CrashHandler);
        signal(SIGABRT, CrashHandler);
        signal(SIGBUS, CrashHandler);
    }
};
static CrashHandlerInstaller g_crash_handler_installer;

inline int Check(bool ok, const char* what) {
    printf("%-48s %s\n", what, ok ? "OK" : "FAILED");
    return ok ? 0 : 1;
}

}  // namespace demo
