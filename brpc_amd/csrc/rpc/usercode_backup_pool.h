// -usercode_in_pthread support (role of the reference's
// src/brpc/details/usercode_backup_pool.h/.cpp).
//
// With the flag on, user callbacks (service methods, async client `done`)
// are assumed to block their pthread (e.g. legacy code calling blocking
// syscalls or pthread locks). They run in place on a fiber worker only while
// fewer than (workers - usercode_backup_threads) of them are running there,
// so some workers always stay free to drive I/O; the excess is queued to a
// pool of backup pthreads. When that queue grows past
// usercode_backup_threads * max_pending_in_each_backup_thread, servers
// reject new requests with ELIMIT (TooManyUserCode).
#pragma once

#include <utility>

#include "base/flags.h"
#include "pb/service.h"

DECLARE_bool(usercode_in_pthread);
DECLARE_int32(usercode_backup_threads);

namespace mrpc {

// true: caller runs the code in place and must call EndRunningUserCodeInPlace.
bool BeginRunningUserCode();
void EndRunningUserCodeInPlace();
// Hands fn(arg) to a backup pthread (after a false BeginRunningUserCode).
void EndRunningUserCodeInPool(void (*fn)(void*), void* arg);
bool TooManyUserCode();

// Runs fn(arg) in place or in the backup pool as described above. Without
// -usercode_in_pthread it simply calls fn(arg).
void RunUserCode(void (*fn)(void*), void* arg);

// Convenience for std::function callers.
template <typename F>
void RunUserCodeF(F&& f) {
    if (!FLAGS_usercode_in_pthread) {
        f();
        return;
    }
    struct Box {
        F fn;
    };
    Box* b = new Box{std::forward<F>(f)};
    RunUserCode(
        [](void* a) {
            Box* bx = static_cast<Box*>(a);
            bx->fn();
            delete bx;
        },
        b);
}

int64_t UserCodeInPlaceCount();
int64_t UserCodeQueueSize();

// Server protocols call service methods through this (RunUserCode aware).
inline void CallServiceMethod(Service* svc, const pb::MethodDescriptor* method, RpcController* cntl,
                              const pb::Message* req, pb::Message* res, Closure* done) {
    if (!FLAGS_usercode_in_pthread) {
        svc->CallMethod(method, cntl, req, res, done);
        return;
    }
    RunUserCodeF([=] { svc->CallMethod(method, cntl, req, res, done); });
}

}  // namespace mrpc
