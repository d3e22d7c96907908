// RetryPolicy (role of src/brpc/retry_policy.h, retry_policy.cpp:33-45).
#pragma once

namespace mrpc {

class Controller;

class RetryPolicy {
public:
    virtual ~RetryPolicy() {}
    // Called with the error set on the controller; true => retry.
    virtual bool DoRetry(const Controller* cntl) const = 0;
};

// Retries connection-level errors: EFAILEDSOCKET, EEOF, EHOSTDOWN, ELOGOFF,
// ETIMEDOUT (connect, not RPC timeout), ELIMIT, ENOENT, EPIPE, ECONNREFUSED,
// ECONNRESET, ENODATA, EOVERCROWDED, EH2RUNOUTSTREAMS.
const RetryPolicy* DefaultRetryPolicy();

}  // namespace mrpc
