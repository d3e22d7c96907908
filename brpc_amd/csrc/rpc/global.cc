// Process-wide initialization (role of src/brpc/global.cpp:207-622):
// ignore SIGPIPE, register error texts, compressors, load balancers, naming
// services, concurrency limiters, every protocol, the client-side response
// handlers, and the runtime metrics.
#include <signal.h>
#include <sys/stat.h>

#include <algorithm>
#include <fstream>
#include <mutex>

#include "base/buf.h"
#include "base/flags.h"
#include "base/logging.h"
#include "base/time.h"
#include "cluster/load_balancer.h"
#include "cluster/naming_service.h"
#include "fiber/fiber.h"
#include "fiber/sync.h"
#include "net/input_messenger.h"
#include "net/socket.h"
#include "policy/policies.h"
#include "rpc/compress.h"
#include "rpc/concurrency_limiter.h"
#include "rpc/errno.h"
#include "rpc/periodic_task.h"
#include "rpc/protocol.h"
#include "rpc/server.h"
#include "rpc/stream_internal.h"
#include "var/var.h"

DEFINE_string(dummy_server_port_file, "dummy_server.port",
              "while no server runs in the process, creating (or touching) this file with a port number in it "
              "starts a server of builtin services on that port (reference global.cpp DUMMY_SERVER_PORT_FILE)");
DEFINE_int32(dummy_server_watch_ms, 1000, "how often the dummy server port file is checked");

namespace mrpc {

// Optional protocol modules register themselves through this list so that
// the core does not need to know about them at compile time.
typedef void (*ProtocolRegistrar)();
static std::vector<ProtocolRegistrar>& extra_registrars() {
    static std::vector<ProtocolRegistrar>* v = new std::vector<ProtocolRegistrar>;
    return *v;
}
int AddProtocolRegistrar(ProtocolRegistrar fn) {
    extra_registrars().push_back(fn);
    return 0;
}

static void expose_runtime_vars() {
    new var::PassiveStatus<int64_t>("fiber_count", [] { return fiber::fiber_count(); });
    new var::PassiveStatus<int64_t>("fiber_switch_count", [] { return fiber::switch_count(); });
    new var::PassiveStatus<int64_t>("fiber_steal_count", [] { return fiber::steal_count(); });
    new var::PassiveStatus<int>("fiber_concurrency", [] { return fiber::get_concurrency(); });
    new var::PassiveStatus<double>("fiber_worker_usage", [] { return fiber::worker_usage(); });
    new var::PassiveStatus<int64_t>("buf_block_count", [] { return Buf::block_count(); });
    new var::PassiveStatus<int64_t>("buf_block_memory", [] { return Buf::block_memory(); });
    new var::PassiveStatus<int64_t>("socket_count", [] { return Socket::nsocket(); });
    new var::PassiveStatus<int64_t>("contention_count", [] { return fiber::ContentionCount(); });
}

namespace {
// The dummy_server.port watcher (reference global.cpp:117,226-254 with
// butil::FileWatcher::init_from_not_exist): a file that appears, or whose
// modification time changes, is read once; its first integer is the port.
class GlobalUpdate : public PeriodicTask {
public:
    bool OnTriggeringTask(timespec* next) override {
        check();
        *next = realtime_after_us((int64_t)std::max(10, FLAGS_dummy_server_watch_ms) * 1000);
        return true;
    }
    void OnDestroyingTask() override { delete this; }

private:
    void check() {
        struct stat st;
        const std::string path = FLAGS_dummy_server_port_file;
        if (path.empty() || stat(path.c_str(), &st) != 0) {
            _seen = false;  // gone: a later creation counts again
            return;
        }
        const int64_t mtime = (int64_t)st.st_mtim.tv_sec * 1000000000LL + st.st_mtim.tv_nsec;
        if (_seen && mtime == _mtime) return;
        if (IsDummyServerRunning() || RunningServerCount() > 0) return;  // consumed only when it can act
        _seen = true;
        _mtime = mtime;
        std::ifstream in(path);
        long port = -1;
        if (!(in >> port) || port < 0 || port > 65535) {
            LOG(WARNING) << "ignore " << path << ": no port in it";
            return;
        }
        if (StartDummyServerAt((int)port) == 0) {
            LOG(INFO) << "dummy server started on port " << port << " (" << path << ")";
        } else {
            LOG(WARNING) << "fail to start the dummy server on port " << port;
        }
    }
    bool _seen = false;
    int64_t _mtime = 0;
};
}  // namespace

void StartGlobalUpdate() {
    PeriodicTaskManager::StartTaskAt(new GlobalUpdate, realtime_after_us(1000));
}

void GlobalInitializeOrDie() {
    static std::once_flag once;
    std::call_once(once, [] {
        signal(SIGPIPE, SIG_IGN);
        RegisterRpcErrnoTexts();
        RegisterBuiltinCompressHandlers();
        RegisterBuiltinLoadBalancers();
        RegisterBuiltinNamingServices();
        RegisterBuiltinConcurrencyLimiters();
        policy::RegisterBaiduStdProtocol();
        RegisterStreamingProtocol();
        policy::RegisterHttpProtocol();
        policy::RegisterH2Protocol();
        policy::RegisterRedisProtocol();
        policy::RegisterMemcacheProtocol();
        policy::RegisterHuluProtocol();
        policy::RegisterSofaProtocol();
        policy::RegisterNsheadProtocols();  // nshead, nova, public_pbrpc, nshead_mcpack, ubrpc_*
        policy::RegisterEspProtocol();
        policy::RegisterMongoProtocol();
        policy::RegisterThriftProtocol();
        policy::RegisterRtmpProtocol();
        for (ProtocolRegistrar r : extra_registrars()) r();
        // Client-side messenger handles responses of every protocol.
        std::vector<std::pair<ProtocolType, Protocol>> protocols;
        ListProtocols(&protocols);
        InputMessenger* cm = get_client_side_messenger();
        for (auto& p : protocols) {
            if (!p.second.process_response) continue;
            InputMessageHandler h;
            h.parse = p.second.parse;
            h.process = p.second.process_response;
            h.verify = nullptr;
            h.arg = nullptr;
            h.name = p.second.name;
            cm->AddHandler(h);
        }
        var::ExposeDefaultVariables();
        expose_runtime_vars();
        fiber::init_runtime();
        StartGlobalUpdate();
    });
}

}  // namespace mrpc
