"""Every self-contained example (brpc_amd/csrc/examples/<name>/main.cc, the
analog of the reference's example/*) runs its in-process servers + client
and must report success."""
import glob
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXAMPLES = sorted(glob.glob(os.path.join(ROOT, "build", "bin", "*_main")))


@pytest.mark.parametrize("path", EXAMPLES, ids=[os.path.basename(p) for p in EXAMPLES])
def test_example(path):
    r = subprocess.run([path], capture_output=True, text=True, timeout=120, cwd="/tmp")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.rstrip().endswith("OK"), r.stdout[-2000:]
