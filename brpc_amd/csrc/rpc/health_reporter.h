// User hook for /health (role of src/brpc/health_reporter.h): fill the
// response (http status + body in cntl) and run done.
#pragma once

#include "pb/service.h"

namespace mrpc {

class Controller;

class HealthReporter {
public:
    virtual ~HealthReporter() {}
    virtual void GenerateReport(Controller* cntl, Closure* done) = 0;
};

}  // namespace mrpc
