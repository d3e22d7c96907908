// Happens-before annotations for ThreadSanitizer builds (no-ops otherwise).
// Used where the synchronisation goes through the kernel in a way the TSan
// runtime does not intercept (epoll_pwait2, shared-memory flags polled by a
// peer process's writes), so the race detector sees the same ordering the
// hardware and the kernel guarantee.
#pragma once

#if defined(__SANITIZE_THREAD__)
#include <sanitizer/tsan_interface.h>
#define MRPC_TSAN_RELEASE(addr) __tsan_release((void*)(addr))
#define MRPC_TSAN_ACQUIRE(addr) __tsan_acquire((void*)(addr))
#else
#define MRPC_TSAN_RELEASE(addr) (void)0
#define MRPC_TSAN_ACQUIRE(addr) (void)0
#endif
