"""Loads the in-tree native extension ``brpc_amd/_native*.so``.

The extension (and ``lib/libmrpc.so`` it links) is produced by
``python build.py``; it is never installed into site-packages so the
round-end checks can see exactly which in-tree object was loaded. A missing
build is an error, never a silent fallback.
"""
import glob
import importlib.util
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))


def _load():
    name = "brpc_amd._native"
    if name in sys.modules:
        return sys.modules[name]
    # torch ships its own libamdhip64.so.7; load it first so the extension
    # binds to the SAME HIP runtime (same soname) instead of pulling a second
    # copy from /opt/rocm — one runtime per process, shared device contexts.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    cands = sorted(glob.glob(os.path.join(_HERE, "_native*.so")))
    if not cands:
        raise ImportError(
            "brpc_amd native extension not built: run `python build.py` at the repo root "
            "(expected brpc_amd/_native*.so)")
    spec = importlib.util.spec_from_file_location(name, cands[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules[name] = mod
    return mod


native = _load()
Server = native.Server
Channel = native.Channel
Press = native.Press


def library_path():
    """Path of the core runtime library the extension links."""
    return os.path.join(_HERE, "lib", "libmrpc.so")
