"""Runtime flags (the gflags analog): every DEFINE_* in the native code."""
from ..native import native


def set_flag(name, value):
    native.set_flag(name, str(value).lower() if isinstance(value, bool) else str(value))


def get_flag(name):
    return native.get_flag(name)


def list_flags():
    return native.list_flags()
