// Echo service implementation shared by examples, tests, rpc_press and
// bench.py (the workload of the reference's example/echo_c++ and
// multi_threaded_echo_c++: echo the message and the attachment).
#pragma once

#include <atomic>

#include "mrpc/proto/echo.pb.h"

namespace mrpc {

class EchoServiceImpl : public example::EchoService {
public:
    void Echo(RpcController* controller, const example::EchoRequest* request, example::EchoResponse* response,
              Closure* done) override;
    int64_t ncalls() const { return _ncalls.load(); }
    // Optional device handler: when set (gpu/gpu_echo.cc), attachments are
    // processed on the GPU (checksum + copy into HBM) before echoing.
    static void (*device_hook)(RpcController* cntl, example::EchoResponse* response);

private:
    std::atomic<int64_t> _ncalls{0};
};

}  // namespace mrpc
