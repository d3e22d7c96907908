"""Runtime flags (the gflags analog, reference src/brpc/reloadable_flags.h and
the /flags builtin page): every DEFINE_* of the native code is settable at
run time by name. Values cross the boundary as strings; this module adds
typed reads, scoped overrides and the ``--name=value`` list syntax that the
tools and ``MRPC_FLAGS`` use."""
import contextlib
import os
import shlex

from ..native import native


def _text(value):
    if isinstance(value, bool):
        return "true" if value else "false"
    return str(value)


def set_flag(name, value):
    """Set a flag by name; raises ValueError for unknown flags or values the
    flag's validator rejects."""
    native.set_flag(name, _text(value))


def get_flag(name):
    """The flag's current value as text."""
    return native.get_flag(name)


def get_flag_typed(name):
    """The flag's value as bool, int, float or str (whichever parses)."""
    v = native.get_flag(name)
    if v in ("true", "false"):
        return v == "true"
    for conv in (int, float):
        try:
            return conv(v)
        except ValueError:
            pass
    return v


def list_flags():
    """name -> current value text for every flag."""
    return native.list_flags()


def parse_flag_args(text):
    """``"--a=1 -b --c=x y"`` -> ``[("a", "1"), ("b", "true"), ("c", "x y")]``
    (shell quoting honoured; a bare flag means true, ``--nob`` stays a name)."""
    out = []
    for item in shlex.split(text or ""):
        if not item.startswith("-"):
            raise ValueError("flag arguments look like --name=value, got %r" % item)
        k, eq, v = item.lstrip("-").partition("=")
        out.append((k, v if eq else "true"))
    return out


def apply_flag_args(text):
    """Set every flag of a ``--name=value`` list; returns the names set."""
    names = []
    for k, v in parse_flag_args(text):
        set_flag(k, v)
        names.append(k)
    return names


def apply_env_flags(var="MRPC_FLAGS"):
    """Apply ``$MRPC_FLAGS`` (same syntax as :func:`parse_flag_args`)."""
    return apply_flag_args(os.environ.get(var, ""))


@contextlib.contextmanager
def flag_overrides(**values):
    """Temporarily set flags; the previous values come back on exit, also
    when the body raises (a setting that fails leaves the earlier ones
    restored)."""
    saved = []
    try:
        for k, v in values.items():
            saved.append((k, native.get_flag(k)))
            set_flag(k, v)
        yield
    finally:
        for k, v in reversed(saved):
            native.set_flag(k, v)
