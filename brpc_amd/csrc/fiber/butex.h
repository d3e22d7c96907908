// Butex: a futex that works for both fibers and pthreads (role of
// bthread/butex.h:45-71, reference butex.cpp:244-700). A fiber waiter is
// queued by a "remained" callback *after* it has switched off its stack, so
// a concurrent wake can never resume a fiber that is still running.
// Every blocking primitive in the runtime (mutex, cond, join, call-id, fd
// wait, GPU event wait) is built on it.
#pragma once

#include <time.h>

#include <atomic>

#include "fiber/fiber.h"

namespace mrpc {
namespace fiber {

// Returns the address of the 32-bit value word. Butexes are pooled and never
// freed, so waking a destroyed butex is harmless.
std::atomic<int>* butex_create();
void butex_destroy(std::atomic<int>* b);
// Wake at most one waiter. Returns number woken.
int butex_wake(std::atomic<int>* b, bool nosignal = false);
int butex_wake_all(std::atomic<int>* b, bool nosignal = false);
// Wake all except the fiber `excluded`.
int butex_wake_except(std::atomic<int>* b, fiber_t excluded);
// Wake one waiter of b1 and move the rest to b2.
int butex_requeue(std::atomic<int>* b1, std::atomic<int>* b2);
// Wait while *b == expected. Returns 0 when woken, -1 with errno
// EWOULDBLOCK (value mismatch), ETIMEDOUT, EINTR (interrupted).
int butex_wait(std::atomic<int>* b, int expected, const timespec* abstime = nullptr);

// Internal: used by interrupt().
struct ButexWaiter;
bool erase_from_butex_because_of_interruption(ButexWaiter* w);

}  // namespace fiber
}  // namespace mrpc
