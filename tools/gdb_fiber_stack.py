"""gdb commands for fibers of the mrpc runtime (role of the reference's
tools/gdb_bthread_stack.py).

    (gdb) source tools/gdb_fiber_stack.py
    (gdb) fiber_list                 # live fibers: tid, entry, saved sp, ...
    (gdb) fiber_frame <sp>           # switch registers to a suspended fiber
    (gdb) bt                         # ... and walk its stack
    (gdb) fiber_reset                # back to the thread's real registers

A suspended fiber's context is the frame pushed by mrpc_fiber_jump
(brpc_amd/csrc/fiber/context.cc): [sp+16] r12 [+24] r13 [+32] r14
[+40] r15 [+48] rbx [+56] rbp [+64] return address; the fiber resumes with
rsp = sp + 72. Works on a live process or a core file (x86-64).
"""
import gdb

_saved = None
_REGS = ("rsp", "rip", "rbp", "rbx", "r12", "r13", "r14", "r15")


def _read_u64(addr):
    return int(gdb.parse_and_eval("*(unsigned long long*)%d" % addr))


class FiberList(gdb.Command):
    """List live fibers (calls mrpc_fiber_dump() in the inferior)."""

    def __init__(self):
        super().__init__("fiber_list", gdb.COMMAND_USER)

    def invoke(self, arg, from_tty):
        try:
            s = gdb.parse_and_eval("(const char*)mrpc_fiber_dump()").string()
        except gdb.error as e:
            print("cannot call mrpc_fiber_dump() (core file?): %s" % e)
            return
        print(s if s else "no live fibers")


class FiberFrame(gdb.Command):
    """fiber_frame <saved sp>: load a suspended fiber's registers."""

    def __init__(self):
        super().__init__("fiber_frame", gdb.COMMAND_USER)

    def invoke(self, arg, from_tty):
        global _saved
        if not arg:
            print("usage: fiber_frame <sp from fiber_list>")
            return
        sp = int(gdb.parse_and_eval(arg))
        if _saved is None:
            _saved = {r: int(gdb.parse_and_eval("$" + r)) for r in _REGS}
        regs = {"r12": _read_u64(sp + 16), "r13": _read_u64(sp + 24), "r14": _read_u64(sp + 32),
                "r15": _read_u64(sp + 40), "rbx": _read_u64(sp + 48), "rbp": _read_u64(sp + 56),
                "rip": _read_u64(sp + 64), "rsp": sp + 72}
        for r, v in regs.items():
            gdb.execute("set $%s = %d" % (r, v))
        gdb.execute("frame 0")


class FiberReset(gdb.Command):
    """Restore the registers saved by the first fiber_frame."""

    def __init__(self):
        super().__init__("fiber_reset", gdb.COMMAND_USER)

    def invoke(self, arg, from_tty):
        global _saved
        if _saved is None:
            print("nothing to reset")
            return
        for r, v in _saved.items():
            gdb.execute("set $%s = %d" % (r, v))
        _saved = None


FiberList()
FiberFrame()
FiberReset()
