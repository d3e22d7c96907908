import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running")


def _ensure_built():
    from brpc_amd.utils.build import native_built
    if not native_built() or not os.path.exists(os.path.join(ROOT, "build", "bin", "mrpc_unittests")):
        import subprocess
        hip = os.path.exists("/opt/rocm/bin/hipcc")
        cmd = [sys.executable, os.path.join(ROOT, "build.py")] + ([] if hip else ["--no-hip"])
        subprocess.run(cmd, cwd=ROOT, check=True)


_ensure_built()


@pytest.fixture(scope="session")
def native():
    from brpc_amd import native as n
    return n


@pytest.fixture(scope="session")
def echo_server(native):
    from brpc_amd.models import start_echo_server
    s = start_echo_server("127.0.0.1:0")
    yield s
    s.stop()
