// Periodic version reporting to -trackme_server (reference src/brpc/trackme.cpp:
// 36-39 flags, :118 TrackMe). A running Server registers its address; one
// background fiber per process sends TrackMeRequest{rpc_version,
// server_addr} every -trackme_interval seconds and logs the verdict
// (warning / fatal text) the tracking server returns; the server may change
// the interval.
#pragma once

#include <cstdint>

#include "base/endpoint.h"

namespace mrpc {

// Version number reported (major * 10000 + minor * 100 + patch).
int64_t RpcVersionNumber();
// Called by Server::Start; a no-op unless -trackme_server is set.
void SetTrackMeAddress(const EndPoint& ep);
// Reports sent so far (tests).
int64_t TrackMeReportsSent();

}  // namespace mrpc
