// Glue between baidu_std and streams.
#pragma once

#include "mrpc/proto/streaming_rpc_meta.pb.h"
#include "net/socket.h"
#include "rpc/stream.h"

namespace mrpc {

class Controller;

void FillStreamSettings(StreamId sid, StreamSettings* settings);
// server: request carried client stream settings (kept until StreamAccept)
void OnRequestStreamSettings(Controller* cntl, Socket* host, const StreamSettings& s);
// server: response with our stream sent on host socket -> stream connected
void OnServerStreamCreated(StreamId sid, SocketId host);
// client: response carried server stream settings -> connect
void OnResponseStreamSettings(Controller* cntl, Socket* host, const StreamSettings& s);
// client: the call carrying the stream ended; close it if it never connected
void OnRequestStreamCallEnded(StreamId sid);
void RegisterStreamingProtocol();

}  // namespace mrpc
