#!/usr/bin/env python3
"""Run every C++ unit suite (and optionally the stub-RCCL plane at 2/3/8
ranks) of a sanitizer build and count the sanitizer reports per suite.

Host code only: the tree is built with `python build.py --tsan` (or
--asan) in a copy of the repository, GPU kernels untouched. Writes one line
per suite: `<suite> rc=<exit code> <tsan|asan>=<reports> <summary line>`.

  python tools/sanitize_suites.py --tree /tmp/tsan/repo --kind tsan --jobs 4 --planes > profiles/tsan_r5.txt
"""
import argparse
import concurrent.futures as cf
import os
import re
import subprocess
import sys
import tempfile

SUPP = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tsan.supp")


def suites(binary):
    out = subprocess.run([binary, "--list"], capture_output=True, text=True, timeout=120).stdout
    seen = []
    for line in out.splitlines():
        s = line.strip().split(".")[0]
        if s and "." in line and s not in seen:
            seen.append(s)
    return seen


def run_suite(binary, suite, kind, timeout):
    env = dict(os.environ)
    if kind == "tsan":
        env["TSAN_OPTIONS"] = "halt_on_error=0 report_signal_unsafe=0 second_deadlock_stack=1 suppressions=" + SUPP
        pat = "WARNING: ThreadSanitizer"
    else:
        env["ASAN_OPTIONS"] = "detect_leaks=0"
        pat = "ERROR: AddressSanitizer"
    try:
        r = subprocess.run([binary, "--filter=%s.*" % suite], capture_output=True, text=True, timeout=timeout,
                           cwd="/tmp", env=env)
        text = r.stdout + r.stderr
        rc = r.returncode
    except subprocess.TimeoutExpired as e:
        text = (e.stdout or b"").decode(errors="replace") + (e.stderr or b"").decode(errors="replace")
        rc = "timeout"
    n = text.count(pat)
    summary = [l for l in text.splitlines() if l.startswith("[==========]")]
    first = ""
    if n:
        m = re.search(r"(WARNING: ThreadSanitizer[^\n]*|ERROR: AddressSanitizer[^\n]*)\n(?:.*\n){0,12}", text)
        first = m.group(0) if m else ""
    return suite, rc, n, summary[-1] if summary else "(no summary)", first


def run_planes(tree, kind):
    lib = subprocess.run(["g++", "-print-file-name=lib%s.so" % kind], capture_output=True, text=True).stdout.strip()
    out = []
    for nranks, extra in ((2, ["--calls", "80,8"]), (3, ["--calls", "80,8"]), (8, ["--calls", "40,4"])):
        # the sanitizer runtime is preloaded into the ranks only (through
        # `env`), not into the launcher
        env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
                   TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0 suppressions=" + SUPP, ASAN_OPTIONS="detect_leaks=0")
        with tempfile.TemporaryDirectory() as d:
            try:
                r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
                                    str(nranks), "--master-addr", "127.0.0.1", "--master-port", str(29700 + nranks),
                                    "--no-python", "env", "LD_PRELOAD=" + lib, sys.executable,
                                    os.path.join(tree, "tests", "plane_ranks.py"), "--out-dir", d] + extra,
                                   capture_output=True, text=True, timeout=900, cwd=tree, env=env)
                text, rc = r.stdout + r.stderr, r.returncode
                ranks = len([f for f in os.listdir(d) if f.startswith("rank")])
                text += "\n# rank reports: %d of %d\n" % (ranks, nranks)
            except subprocess.TimeoutExpired:
                text, rc = "", "timeout"
        pat = "WARNING: ThreadSanitizer" if kind == "tsan" else "ERROR: AddressSanitizer"
        n = text.count(pat)
        first = ""
        if n:
            i = text.find(pat)
            first = text[i:i + 1500]
        summary = [l for l in text.splitlines() if l.startswith("# rank reports")]
        out.append(("RcclPlaneStub%dRanks" % nranks, rc, n, summary[-1] if summary else "", first))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tree", required=True)
    ap.add_argument("--kind", choices=["tsan", "asan"], default="tsan")
    ap.add_argument("--jobs", type=int, default=4)
    ap.add_argument("--timeout", type=int, default=1200)
    ap.add_argument("--only", default="", help="comma-separated suites")
    ap.add_argument("--planes", action="store_true", help="also the stub-RCCL plane at 2, 3 and 8 ranks")
    a = ap.parse_args()
    binary = os.path.join(a.tree, "build", "bin", "mrpc_unittests")
    names = [s for s in suites(binary) if not a.only or s in a.only.split(",")]
    results = []
    with cf.ThreadPoolExecutor(a.jobs) as ex:
        for res in ex.map(lambda s: run_suite(binary, s, a.kind, a.timeout), names):
            results.append(res)
            print("%s rc=%s %s=%d %s" % (res[0], res[1], a.kind, res[2], res[3]), flush=True)
    if a.planes:
        for res in run_planes(a.tree, a.kind):
            results.append(res)
            print("%s rc=%s %s=%d %s" % (res[0], res[1], a.kind, res[2], res[3]), flush=True)
    total = sum(r[2] for r in results)
    print("# total %s reports: %d over %d runs" % (a.kind, total, len(results)))
    for r in results:
        if r[4]:
            print("# --- first report of %s:\n%s" % (r[0], "\n".join("# " + l for l in r[4].splitlines())))


if __name__ == "__main__":
    main()
