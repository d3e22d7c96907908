// rpc_dump: sample live server requests into recordio files for later
// replay by tools/rpc_replay (role of the reference's src/brpc/rpc_dump.h/.cpp).
//
//   -rpc_dump                    turn sampling on (reloadable)
//   -rpc_dump_dir                directory of the dump files
//   -rpc_dump_max_files          keep at most this many files (oldest removed)
//   -rpc_dump_max_requests_in_one_file
//   -rpc_dump_max_samples_per_second (collector speed limit)
//
// Protocols ask AskToBeSampled() per request (one relaxed load when off);
// a sampled request is filled and submitted to the var::Collector thread,
// which appends {meta: RpcDumpMeta, payload: body+attachment} records.
#pragma once

#include <string>

#include "base/buf.h"
#include "base/flags.h"
#include "mrpc/proto/rpc_dump.pb.h"
#include "var/collector.h"

DECLARE_bool(rpc_dump);
DECLARE_string(rpc_dump_dir);

namespace mrpc {

class SampledRequest : public var::Collected {
public:
    RpcDumpMeta meta;
    Buf request;  // serialized (possibly compressed) body + attachment
    void dump_and_destroy(size_t round) override;
    var::CollectorSpeedLimit* speed_limit() override;
};

// nullptr unless -rpc_dump is on and this request is picked by the limiter.
SampledRequest* AskToBeSampled();

// Files written so far (for tests / builtin pages).
std::vector<std::string> ListRpcDumpFiles(const std::string& dir);
// Flushes buffered records (tests).
void FlushRpcDump();

}  // namespace mrpc
