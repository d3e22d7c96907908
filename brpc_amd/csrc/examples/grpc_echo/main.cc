// gRPC (reference example/grpc_c++): the same pb service served over h2 with
// the gRPC framing; the client uses protocol "h2:grpc" and optional gzip
// message compression (-gzip). Interop with grpcio is covered by
// tests/test_grpc_interop.py.
#include "examples/common.h"
#include "rpc/compress.h"

DEFINE_bool(gzip, true, "compress messages with gzip (grpc-encoding)");
DEFINE_int32(calls, 50, "calls to make");

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    demo::LocalServer s("grpc");
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.protocol = "h2:grpc";
    opt.timeout_ms = 2000;
    if (ch.Init(s.addr().c_str(), &opt) != 0) return 1;
    example::EchoService_Stub stub(&ch);
    int ok = 0;
    for (int i = 0; i < FLAGS_calls; ++i) {
        mrpc::Controller cntl;
        if (FLAGS_gzip) cntl.set_request_compress_type(mrpc::COMPRESS_TYPE_GZIP);
        example::EchoRequest req;
        example::EchoResponse res;
        req.set_message(std::string(1000, 'g') + std::to_string(i));
        stub.Echo(&cntl, &req, &res, nullptr);
        ok += !cntl.Failed() && res.message() == req.message() + "@grpc";
    }
    // a failing call maps to a grpc-status error
    mrpc::Controller cntl;
    example::EchoRequest req;
    example::EchoResponse res;
    req.set_message("fail");
    req.set_server_fail(true);
    stub.Echo(&cntl, &req, &res, nullptr);
    printf("%d/%d grpc calls ok; failing call -> %s\n", ok, FLAGS_calls, cntl.ErrorText().c_str());
    return demo::Check(ok == FLAGS_calls && cntl.Failed(), "h2:grpc echo");
}
