// Common macros for the mrpc native runtime.
#pragma once

#include <cstddef>
#include <cstdint>

#define MRPC_LIKELY(x) __builtin_expect(!!(x), 1)
#define MRPC_UNLIKELY(x) __builtin_expect(!!(x), 0)
#define MRPC_CACHELINE 64
#define MRPC_CACHELINE_ALIGNED alignas(MRPC_CACHELINE)
#define MRPC_NOINLINE __attribute__((noinline))
#define MRPC_FORCE_INLINE inline __attribute__((always_inline))
#define MRPC_WEAK __attribute__((weak))

#define MRPC_DISALLOW_COPY(T) \
    T(const T&) = delete;     \
    T& operator=(const T&) = delete

#define MRPC_CONCAT_IMPL(a, b) a##b
#define MRPC_CONCAT(a, b) MRPC_CONCAT_IMPL(a, b)

namespace mrpc {

template <typename T, size_t N>
constexpr size_t arraysize(T (&)[N]) { return N; }

inline void cpu_relax() { __builtin_ia32_pause(); }

}  // namespace mrpc
