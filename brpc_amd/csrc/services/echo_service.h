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
    int64_t gpu_calls() const { return _gpu_calls.load(); }
    // GPU that serves requests with gpu_process set (-1: none, such
    // requests fail with EREQUEST). The attachment is gathered into HBM by
    // a kernel that also checksums it, and echoed from HBM
    // (gpu/device_handler.h).
    void set_gpu_device(int device) { _gpu_device = device; }

private:
    std::atomic<int64_t> _ncalls{0};
    std::atomic<int64_t> _gpu_calls{0};
    int _gpu_device = -1;
};

}  // namespace mrpc
