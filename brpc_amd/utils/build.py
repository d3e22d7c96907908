"""Drives the native build (``build.py`` at the repo root) from Python."""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def native_built():
    pkg = os.path.join(ROOT, "brpc_amd")
    return bool(glob.glob(os.path.join(pkg, "_native*.so"))) and os.path.exists(
        os.path.join(pkg, "lib", "libmrpc.so"))


def build_native(jobs=None, hip=True, check=True):
    """Compile libmrpc (host C++ + gfx950 HIP), the extension, tools and tests."""
    cmd = [sys.executable, os.path.join(ROOT, "build.py")]
    if jobs:
        cmd += ["-j", str(jobs)]
    if not hip:
        cmd.append("--no-hip")
    r = subprocess.run(cmd, cwd=ROOT)
    if check and r.returncode != 0:
        raise RuntimeError("native build failed (exit %d)" % r.returncode)
    return r.returncode
