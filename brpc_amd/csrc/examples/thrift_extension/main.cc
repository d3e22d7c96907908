// Framed thrift (reference example/thrift_extension_c++): an EchoService
// defined in thrift IDL as
//     struct EchoRequest  { 1: required string data; 2: optional i32 need_by_proxy }
//     struct EchoResponse { 1: required string data }
//     service EchoService { EchoResponse Echo(1: EchoRequest request) }
// served by a ThriftService (ServerOptions::thrift_service) and called
// three ways:
//   * a Channel with protocol "thrift" (ThriftFramedMessage request),
//   * a "native" client writing TFramedTransport + TBinaryProtocol bytes on
//     a plain socket (wire compatibility with stock thrift clients),
//   * the same Channel against a "native" server that is nothing but a
//     socket loop speaking the framed binary protocol (stock servers).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>

#include <atomic>
#include <thread>
#include <vector>

#include "base/time.h"
#include "builtin/cpu_profiler.h"
#include "fiber/fiber.h"

#include "examples/common.h"
#include "thrift/thrift.h"

using mrpc::thrift::Value;

DEFINE_int32(thread_num, 0, "load phase: fibers echoing \"hello\" through the framework client (0: none)");
DEFINE_int32(repeat, 1, "load phase: the string is \"hello\" repeated this many times (the reference: 1 and 1000)");
DEFINE_double(duration_s, 1.0, "load phase: seconds");
DEFINE_string(profile_folded, "", "load phase: write a CPU profile (folded stacks) to this file");

namespace {

class EchoThrift : public mrpc::ThriftService {
public:
    void ProcessThriftFramedRequest(mrpc::Controller* cntl, mrpc::ThriftFramedMessage* req,
                                    mrpc::ThriftFramedMessage* res, mrpc::Closure* done) override {
        mrpc::ClosureGuard g(done);
        if (req->method_name != "Echo") {
            cntl->SetFailed(mrpc::ENOMETHOD, "unknown method %s", req->method_name.c_str());
            return;
        }
        const Value* arg = req->body.find(1);
        const Value* data = arg ? arg->find(1) : nullptr;
        if (!data || data->type() != mrpc::thrift::T_STRING) {
            cntl->SetFailed(mrpc::EREQUEST, "EchoRequest.data missing");
            return;
        }
        Value out = Value::Struct();
        out.field(1) = Value::String(data->as_string());
        res->body.field(0) = out;  // success
    }
};

Value MakeArgs(const std::string& s) {
    Value req = Value::Struct();
    req.field(1) = Value::String(s);
    Value args = Value::Struct();
    args.field(1) = req;
    return args;
}

int Connect(int port) {
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (connect(fd, (sockaddr*)&a, sizeof(a)) != 0) {
        close(fd);
        return -1;
    }
    return fd;
}

bool ReadFull(int fd, char* p, size_t n) {
    while (n) {
        const ssize_t r = read(fd, p, n);
        if (r <= 0) return false;
        p += r;
        n -= (size_t)r;
    }
    return true;
}

bool WriteFrame(int fd, const std::string& msg) {
    uint32_t len = htonl((uint32_t)msg.size());
    std::string frame(reinterpret_cast<char*>(&len), 4);
    frame += msg;
    return write(fd, frame.data(), frame.size()) == (ssize_t)frame.size();
}

bool ReadFrame(int fd, std::string* msg) {
    uint32_t len;
    if (!ReadFull(fd, reinterpret_cast<char*>(&len), 4)) return false;
    msg->resize(ntohl(len));
    return ReadFull(fd, &(*msg)[0], msg->size());
}

// A stock-style framed binary server: one thread, one connection at a time.
class NativeServer {
public:
    NativeServer() {
        _lfd = socket(AF_INET, SOCK_STREAM, 0);
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        socklen_t len = sizeof(a);
        bind(_lfd, (sockaddr*)&a, sizeof(a));
        listen(_lfd, 8);
        getsockname(_lfd, (sockaddr*)&a, &len);
        port = ntohs(a.sin_port);
        _t = std::thread([this] {
            for (;;) {
                _cfd = accept(_lfd, nullptr, nullptr);
                if (_cfd < 0) return;
                std::string msg;
                while (ReadFrame(_cfd, &msg)) {
                    mrpc::thrift::MessageHeader h;
                    Value args;
                    if (!mrpc::thrift::ReadMessage(msg.data(), msg.size(), &h, &args)) break;
                    const Value* r = args.find(1);
                    Value out = Value::Struct();
                    out.field(1) = Value::String("native:" + (r && r->find(1) ? r->find(1)->as_string() : ""));
                    Value result = Value::Struct();
                    result.field(0) = out;
                    mrpc::thrift::MessageHeader rh{h.name, mrpc::thrift::T_REPLY, h.seqid};
                    std::string reply;
                    mrpc::thrift::WriteMessage(&reply, rh, result);
                    if (!WriteFrame(_cfd, reply)) break;
                }
                const int c = _cfd.exchange(-1);
                close(c);
            }
        });
    }
    ~NativeServer() {
        const int c = _cfd.load();
        if (c >= 0) shutdown(c, SHUT_RDWR);  // the client may keep its connection
        shutdown(_lfd, SHUT_RDWR);
        close(_lfd);
        _t.join();
    }
    int port = 0;

private:
    int _lfd = -1;
    std::atomic<int> _cfd{-1};
    std::thread _t;
};

}  // namespace

int main(int argc, char** argv) {
    mrpc::ParseCommandLineFlags(&argc, &argv);
    EchoThrift svc;
    mrpc::Server server;
    mrpc::ServerOptions so;
    so.thrift_service = &svc;
    if (server.Start("127.0.0.1:0", &so) != 0) return 1;
    const int port = server.listen_port();

    // 1) framework client
    mrpc::Channel ch;
    mrpc::ChannelOptions opt;
    opt.protocol = "thrift";
    opt.timeout_ms = 2000;
    if (ch.Init(("127.0.0.1:" + std::to_string(port)).c_str(), &opt) != 0) return 1;
    bool ok = true;
    for (int i = 0; i < 20 && ok; ++i) {
        mrpc::ThriftFramedMessage req, res;
        mrpc::Controller cntl;
        req.method_name = "Echo";
        req.body = MakeArgs("hi " + std::to_string(i));
        ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
        ok = !cntl.Failed() && res.success() && res.success()->find(1) &&
             res.success()->find(1)->as_string() == "hi " + std::to_string(i);
    }
    {  // unknown method -> TApplicationException -> failed controller
        mrpc::ThriftFramedMessage req, res;
        mrpc::Controller cntl;
        req.method_name = "Nope";
        ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
        ok = ok && cntl.Failed();
        printf("unknown method: %s\n", cntl.ErrorText().c_str());
    }
    printf("framework client: %s\n", ok ? "20 echoes ok" : "FAILED");

    // 2) native client: raw framed binary bytes on a socket
    bool native_ok = false;
    const int fd = Connect(port);
    if (fd >= 0) {
        std::string msg, reply;
        mrpc::thrift::WriteMessage(&msg, mrpc::thrift::MessageHeader{"Echo", mrpc::thrift::T_CALL, 77},
                                   MakeArgs("from a stock client"));
        mrpc::thrift::MessageHeader h;
        Value result;
        if (WriteFrame(fd, msg) && ReadFrame(fd, &reply) &&
            mrpc::thrift::ReadMessage(reply.data(), reply.size(), &h, &result)) {
            const Value* s = result.find(0);
            native_ok = h.type == mrpc::thrift::T_REPLY && h.seqid == 77 && h.name == "Echo" && s && s->find(1) &&
                        s->find(1)->as_string() == "from a stock client";
        }
        close(fd);
    }
    printf("native client -> framework server: %s\n", native_ok ? "ok" : "FAILED");

    // 3) framework client -> native server
    NativeServer native;
    mrpc::Channel nch;
    bool to_native = nch.Init(("127.0.0.1:" + std::to_string(native.port)).c_str(), &opt) == 0;
    for (int i = 0; i < 5 && to_native; ++i) {
        mrpc::ThriftFramedMessage req, res;
        mrpc::Controller cntl;
        req.method_name = "Echo";
        req.body = MakeArgs(std::to_string(i));
        nch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
        to_native = !cntl.Failed() && res.success() && res.success()->find(1) &&
                    res.success()->find(1)->as_string() == "native:" + std::to_string(i);
    }
    printf("framework client -> native server: %s\n", to_native ? "ok" : "FAILED");

    // 4) load: the reference's thrift figure (docs/en/thrift.md) echoes
    // "hello" (and "hello" x 1000) from 60 threads
    if (FLAGS_thread_num > 0 && ok) {
        std::string hello;
        for (int i = 0; i < FLAGS_repeat; ++i) hello += "hello";
        std::atomic<bool> stop{false};
        std::atomic<int64_t> n{0}, errors{0}, lat_sum{0};
        std::vector<mrpc::fiber::fiber_t> fs(FLAGS_thread_num);
        for (auto& f : fs) {
            mrpc::fiber::start(
                [&] {
                    while (!stop.load(std::memory_order_relaxed)) {
                        mrpc::ThriftFramedMessage req, res;
                        mrpc::Controller cntl;
                        req.method_name = "Echo";
                        req.body = MakeArgs(hello);
                        ch.CallMethod(nullptr, &cntl, &req, &res, nullptr);
                        if (cntl.Failed() || !res.success()) {
                            errors.fetch_add(1);
                        } else {
                            n.fetch_add(1);
                            lat_sum.fetch_add(cntl.latency_us());
                        }
                    }
                },
                false, nullptr, &f);
        }
        if (!FLAGS_profile_folded.empty()) {
            std::string folded;
            int64_t nsamples = 0;
            mrpc::profiler::ProfileCpu(FLAGS_duration_s, 997, &folded, nullptr, &nsamples);
            if (FILE* pf = fopen(FLAGS_profile_folded.c_str(), "w")) {
                fwrite(folded.data(), 1, folded.size(), pf);
                fclose(pf);
            }
        } else {
            mrpc::fiber::usleep((uint64_t)(FLAGS_duration_s * 1e6));
        }
        stop = true;
        for (auto f : fs) mrpc::fiber::join(f);
        printf("load: %lld QPS, avg %lld us, \"hello\" x %d, %d fibers, %lld failed calls\n",
               (long long)(n.load() / FLAGS_duration_s), n.load() ? (long long)(lat_sum.load() / n.load()) : 0ll,
               FLAGS_repeat, FLAGS_thread_num, (long long)errors.load());
        ok = errors.load() == 0 && n.load() > 0;
    }
    server.Stop(0);
    server.Join();
    return demo::Check(ok && native_ok && to_native, "framed thrift interop");
}
