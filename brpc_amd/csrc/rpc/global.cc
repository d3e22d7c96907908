// Process-wide initialization (role of src/brpc/global.cpp:207-622):
// ignore SIGPIPE, register error texts, compressors, load balancers, naming
// services, concurrency limiters, every protocol, the client-side response
// handlers, and the runtime metrics.
#include <signal.h>

#include <mutex>

#include "base/buf.h"
#include "base/logging.h"
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
#include "rpc/protocol.h"
#include "rpc/stream_internal.h"
#include "var/var.h"

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
    });
}

}  // namespace mrpc
