// Wake a pthread out of a blocking system call (role of the reference's
// src/bthread/interrupt_pthread.cpp:37): SIGURG with an empty handler
// installed WITHOUT SA_RESTART, so read/epoll_wait/nanosleep/... return
// EINTR. Used when the runtime stops (a worker stuck in a syscall of user
// code must still reach its join, task_control.cpp:246) and by
// fiber::interrupt() on a fiber that is running on its worker, i.e. not
// parked on a butex or a timer the runtime could cancel.
#pragma once

#include <pthread.h>

namespace mrpc {
namespace fiber {

int interrupt_pthread(pthread_t th);
// How many SIGURGs this process handled (tests).
long interrupt_pthread_signals();

}  // namespace fiber
}  // namespace mrpc
