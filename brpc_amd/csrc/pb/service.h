// Generic RPC service interfaces used by generated code (the roles of
// google::protobuf::Service/RpcChannel/RpcController/Closure that the
// reference builds on, plus brpc's NewCallback/ClosureGuard from
// src/brpc/callback.h and closure_guard.h).
#pragma once

#include <functional>
#include <string>
#include <utility>

#include "pb/descriptor.h"
#include "pb/message.h"

namespace mrpc {

class Closure {
public:
    virtual ~Closure() {}
    virtual void Run() = 0;
};

// Self-deleting closure over any callable.
template <typename F>
class FunctionClosure : public Closure {
public:
    explicit FunctionClosure(F&& f) : _f(std::move(f)) {}
    void Run() override {
        F f = std::move(_f);
        delete this;
        f();
    }
private:
    F _f;
};

template <typename F>
Closure* NewCallback(F&& f) {
    return new FunctionClosure<typename std::decay<F>::type>(std::forward<F>(f));
}
template <typename F, typename... Args>
Closure* NewCallback(F&& f, Args&&... args) {
    auto bound = std::bind(std::forward<F>(f), std::forward<Args>(args)...);
    return new FunctionClosure<decltype(bound)>(std::move(bound));
}
// A closure that does nothing (for sync calls that want to pass a non-null done).
Closure* NewDoNothingClosure();

// Runs done->Run() on scope exit unless released.
class ClosureGuard {
public:
    ClosureGuard() : _done(nullptr) {}
    explicit ClosureGuard(Closure* d) : _done(d) {}
    ~ClosureGuard() {
        if (_done) _done->Run();
    }
    Closure* release() {
        Closure* d = _done;
        _done = nullptr;
        return d;
    }
    void reset(Closure* d) {
        if (_done) _done->Run();
        _done = d;
    }
    bool empty() const { return _done == nullptr; }
    ClosureGuard(const ClosureGuard&) = delete;
    ClosureGuard& operator=(const ClosureGuard&) = delete;
private:
    Closure* _done;
};

class RpcController {
public:
    virtual ~RpcController() {}
    virtual void Reset() = 0;
    virtual bool Failed() const = 0;
    virtual std::string ErrorText() const = 0;
    virtual void StartCancel() = 0;
    virtual void SetFailed(const std::string& reason) = 0;
    virtual bool IsCanceled() const = 0;
    virtual void NotifyOnCancel(Closure* callback) = 0;
};

class RpcChannel {
public:
    virtual ~RpcChannel() {}
    virtual void CallMethod(const pb::MethodDescriptor* method, RpcController* controller,
                            const pb::Message* request, pb::Message* response, Closure* done) = 0;
};

class Service {
public:
    virtual ~Service() {}
    virtual const pb::ServiceDescriptor* GetDescriptor() = 0;
    virtual void CallMethod(const pb::MethodDescriptor* method, RpcController* controller,
                            const pb::Message* request, pb::Message* response, Closure* done) = 0;
    virtual const pb::Message& GetRequestPrototype(const pb::MethodDescriptor* method) const = 0;
    virtual const pb::Message& GetResponsePrototype(const pb::MethodDescriptor* method) const = 0;
};

}  // namespace mrpc
