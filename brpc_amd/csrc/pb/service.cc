#include "pb/service.h"

namespace mrpc {

namespace {
class DoNothing : public Closure {
public:
    void Run() override { delete this; }
};
}  // namespace

Closure* NewDoNothingClosure() { return new DoNothing; }

}  // namespace mrpc
