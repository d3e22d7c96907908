#include "fiber/interrupt_pthread.h"

#include <signal.h>

#include <atomic>
#include <cstring>

namespace mrpc {
namespace fiber {

namespace {
std::atomic<long> g_handled{0};

// Does nothing but exist: its delivery interrupts the syscall in progress.
void on_sigurg(int) { g_handled.fetch_add(1, std::memory_order_relaxed); }

pthread_once_t g_once = PTHREAD_ONCE_INIT;

void install() {
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_handler = on_sigurg;
    sigemptyset(&sa.sa_mask);
    sa.sa_flags = 0;  // no SA_RESTART: the interrupted call returns EINTR
    sigaction(SIGURG, &sa, nullptr);
}
}  // namespace

int interrupt_pthread(pthread_t th) {
    pthread_once(&g_once, install);
    return pthread_kill(th, SIGURG);
}

long interrupt_pthread_signals() { return g_handled.load(std::memory_order_relaxed); }

}  // namespace fiber
}  // namespace mrpc
