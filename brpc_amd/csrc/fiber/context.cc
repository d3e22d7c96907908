#include "fiber/context.h"

#include <cstring>

// Stack layout of a suspended context (low -> high):
//   [+0]  8 bytes pad | [+8] mxcsr (4) | [+12] x87 cw (2) | pad
//   [+16] r12 [+24] r13 [+32] r14 [+40] r15 [+48] rbx [+56] rbp [+64] ret
asm(R"(
    .text
    .globl mrpc_fiber_jump
    .type mrpc_fiber_jump,@function
    .align 16
mrpc_fiber_jump:
    pushq %rbp
    pushq %rbx
    pushq %r15
    pushq %r14
    pushq %r13
    pushq %r12
    subq $16, %rsp
    stmxcsr 8(%rsp)
    fnstcw 12(%rsp)
    movq %rsp, (%rdi)
    movq %rsi, %rsp
    ldmxcsr 8(%rsp)
    fldcw 12(%rsp)
    addq $16, %rsp
    popq %r12
    popq %r13
    popq %r14
    popq %r15
    popq %rbx
    popq %rbp
    movq %rdx, %rax
    movq %rdx, %rdi
    ret
    .size mrpc_fiber_jump,.-mrpc_fiber_jump

    .globl mrpc_fiber_trampoline
    .type mrpc_fiber_trampoline,@function
    .align 16
mrpc_fiber_trampoline:
    andq $-16, %rsp
    callq *%r12
    ud2
    .size mrpc_fiber_trampoline,.-mrpc_fiber_trampoline
    .section .note.GNU-stack,"",@progbits
    .text
)");

extern "C" void mrpc_fiber_trampoline();

namespace mrpc {
namespace fiber {

void* make_context(void* stack_base, size_t size, ContextFn fn) {
    uintptr_t top = ((uintptr_t)stack_base + size) & ~(uintptr_t)15;
    uint64_t* sp = (uint64_t*)top;
    *--sp = 0;                                      // pad (keeps ret slot 16-aligned)
    *--sp = (uint64_t)(uintptr_t)&mrpc_fiber_trampoline;  // return address
    *--sp = 0;                                      // rbp
    *--sp = 0;                                      // rbx
    *--sp = 0;                                      // r15
    *--sp = 0;                                      // r14
    *--sp = 0;                                      // r13
    *--sp = (uint64_t)(uintptr_t)fn;                // r12 -> called by trampoline
    sp -= 2;                                        // fpu control words
    uint32_t mxcsr = 0x1F80;
    uint16_t fcw = 0x037F;
    memcpy((char*)sp + 8, &mxcsr, 4);
    memcpy((char*)sp + 12, &fcw, 2);
    return sp;
}

}  // namespace fiber
}  // namespace mrpc
