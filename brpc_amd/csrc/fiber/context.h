// User-level context switching for x86_64 SysV (role of bthread/context.h:56-60,
// reference context.cpp:337,381 — own implementation, not fcontext).
//
// A context is just a saved stack pointer. mrpc_fiber_jump() pushes the
// callee-saved registers and MXCSR/x87 control word onto the current stack,
// stores rsp in *from_sp, switches to to_sp, restores and returns `arg` in
// the resumed context. A fresh context built by make_context() starts in
// fn(arg) where arg is the value passed to the jump that first enters it.
#pragma once

#include <cstddef>
#include <cstdint>

extern "C" {
void* mrpc_fiber_jump(void** from_sp, void* to_sp, void* arg);
}

namespace mrpc {
namespace fiber {

typedef void (*ContextFn)(void* arg);

// Build an initial context at the top of [stack_base, stack_base+size).
void* make_context(void* stack_base, size_t size, ContextFn fn);

}  // namespace fiber
}  // namespace mrpc
