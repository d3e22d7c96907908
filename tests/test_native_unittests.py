"""Runs the C++ unit tests (brpc_amd/csrc/tests/*.cc, the analog of the
reference's test/*_unittest.cpp gtest binaries) one suite per pytest case,
each in its own process with a timeout."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "bin", "mrpc_unittests")


def _suites():
    out = subprocess.run([BIN, "--list"], capture_output=True, text=True, timeout=60).stdout
    suites = []
    for line in out.splitlines():
        line = line.strip()
        if "." in line:
            s = line.split(".")[0]
            if s not in suites:
                suites.append(s)
    return suites


@pytest.mark.parametrize("suite", _suites())
def test_suite(suite):
    r = subprocess.run([BIN, "--filter=%s.*" % suite], capture_output=True, text=True, timeout=300,
                       cwd="/tmp")
    assert r.returncode == 0, (r.stdout[-4000:] + r.stderr[-4000:])
