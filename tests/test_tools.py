"""Command-line tools as subprocesses (role of the reference's tools/):
trackme_server receiving reports from a server started with
-trackme_server, rpc_view relaying a target's builtin pages, parallel_http
fetching many urls concurrently."""
import os
import socket
import subprocess
import sys
import time
import urllib.request

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "bin")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _wait_port(port, timeout=10):
    end = time.time() + timeout
    while time.time() < end:
        try:
            socket.create_connection(("127.0.0.1", port), timeout=0.2).close()
            return
        except OSError:
            time.sleep(0.05)
    raise RuntimeError("port %d never opened" % port)


@pytest.fixture
def procs():
    started = []
    yield started
    for p in started:
        p.terminate()
        try:
            p.wait(timeout=5)
        except subprocess.TimeoutExpired:
            p.kill()


def _spawn(procs, args):
    p = subprocess.Popen(args, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, cwd="/tmp")
    procs.append(p)
    return p


def _get(url):
    with urllib.request.urlopen(url, timeout=5) as r:
        return r.status, r.read().decode()


def test_trackme_reports_and_bug_verdicts(procs, tmp_path):
    tport, sport = _free_port(), _free_port()
    bugs = tmp_path / "bugs.txt"
    bugs.write_text("# versions 10000..19999 have a known bug\n10000 19999 warning upgrade me please\n")
    tm = _spawn(procs, [os.path.join(BIN, "trackme_server"), "-port=%d" % tport, "-bug_file=%s" % bugs])
    _wait_port(tport)
    srv = _spawn(procs, [os.path.join(BIN, "echo_server"), "-port=%d" % sport,
                         "-trackme_server=127.0.0.1:%d" % tport, "-trackme_interval=1"])
    _wait_port(sport)
    time.sleep(2.5)
    srv.terminate()
    out_srv = srv.communicate(timeout=10)[0]
    tm.terminate()
    out_tm = tm.communicate(timeout=10)[0]
    assert "new reporter 0.0.0.0:%d" % sport in out_tm, out_tm
    assert "upgrade me please" in out_srv, out_srv  # the verdict reached the reporting server


def test_rpc_view_relays_builtin_pages(procs):
    sport, vport = _free_port(), _free_port()
    _spawn(procs, [os.path.join(BIN, "echo_server"), "-port=%d" % sport])
    _wait_port(sport)
    _spawn(procs, [os.path.join(BIN, "rpc_view"), "-port=%d" % vport, "-target=127.0.0.1:%d" % sport])
    _wait_port(vport)
    st, body = _get("http://127.0.0.1:%d/status" % vport)
    assert st == 200 and "EchoService" in body, body[:500]
    st, body = _get("http://127.0.0.1:%d/flags?name=port" % vport)
    assert st == 200 and "port" in body
    st, direct = _get("http://127.0.0.1:%d/version" % sport)
    st2, viewed = _get("http://127.0.0.1:%d/version" % vport)
    assert st2 == 200 and viewed == direct
    with pytest.raises(urllib.error.HTTPError):
        _get("http://127.0.0.1:%d/no_such_page_xyz" % vport)


def test_parallel_http(procs, tmp_path):
    sport = _free_port()
    _spawn(procs, [os.path.join(BIN, "echo_server"), "-port=%d" % sport])
    _wait_port(sport)
    urls = tmp_path / "urls.txt"
    pages = ["status", "vars", "flags", "version", "health", "connections"]
    urls.write_text("".join("http://127.0.0.1:%d/%s\n" % (sport, p) for p in pages * 20))
    r = subprocess.run([os.path.join(BIN, "parallel_http"), "-url_file=%s" % urls, "-thread_num=16"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "fetched 120 urls" in r.stdout and "failed=0" in r.stdout
    lines = [l for l in r.stdout.splitlines() if l.startswith("200 ")]
    assert len(lines) == 120


def test_sampling_heap_profiler():
    """heapprof/heapprof.cc linked into heapprof_demo: /hotspots/heap,
    /hotspots/growth and /pprof/heap attribute sampled bytes to the right
    functions (the demo checks the estimates against the true sizes)."""
    r = subprocess.run([os.path.join(BIN, "heapprof_demo")], capture_output=True, text=True, timeout=60, cwd="/tmp")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "KeepLiveBuffers" in r.stdout


def test_rpcz_pages_by_trace_and_time(procs, tmp_path):
    """/rpcz browsing of the on-disk span store: recent view, ?trace_id=,
    ?time= (epoch us or YYYY/MM/DD-HH:MM:SS) and ?stats."""
    import re
    from brpc_amd import native
    port = _free_port()
    _spawn(procs, [os.path.join(BIN, "echo_server"), "-port=%d" % port, "-enable_rpcz=true",
                   "-rpcz_database_dir=%s" % tmp_path])
    _wait_port(port)
    p = native.Press({"server": "127.0.0.1:%d" % port, "concurrency": 2})
    p.run_requests(20)
    assert p.stats()["error"] == 0
    time.sleep(0.3)
    mid_us = int(time.time() * 1e6)
    time.sleep(0.3)
    p.run_requests(5)
    time.sleep(1.2)
    st, recent = _get("http://127.0.0.1:%d/rpcz?max=500" % port)
    assert st == 200 and "EchoService.Echo" in recent, recent[:500]
    trace = re.search(r"trace=([0-9a-f]{16})", recent).group(1)
    _, by_trace = _get("http://127.0.0.1:%d/rpcz?trace_id=%s" % (port, trace))
    assert by_trace.strip() and all(("trace=" + trace) in line for line in by_trace.splitlines()
                                    if line.startswith(("S ", "C "))), by_trace
    _, before = _get("http://127.0.0.1:%d/rpcz?time=%d&max=500" % (port, mid_us))
    _, now = _get("http://127.0.0.1:%d/rpcz?time=%d&max=500" % (port, int(time.time() * 1e6)))
    n_before = sum(1 for l in before.splitlines() if l.startswith("S "))
    n_now = sum(1 for l in now.splitlines() if l.startswith("S "))
    assert n_before == 20 and n_now == 25, (n_before, n_now)
    _, stats = _get("http://127.0.0.1:%d/rpcz?stats" % port)
    assert "written: 25" in stats and "dir: %s" % tmp_path in stats, stats
    stamp = time.strftime("%Y/%m/%d-%H:%M:%S", time.localtime(time.time() + 5))
    _, by_date = _get("http://127.0.0.1:%d/rpcz?time=%s&max=500" % (port, stamp))
    assert sum(1 for l in by_date.splitlines() if l.startswith("S ")) == 25


_DUMMY_SCRIPT = r"""
import os, sys, time, urllib.request
sys.path.insert(0, sys.argv[1])
from brpc_amd import native
path, port = sys.argv[2], int(sys.argv[3])
native.set_flag("dummy_server_port_file", path)
native.set_flag("dummy_server_watch_ms", "50")
native.global_init()  # what every channel / server does first
time.sleep(0.3)
def health():
    try:
        return urllib.request.urlopen("http://127.0.0.1:%d/health" % port, timeout=1).read()
    except OSError:
        return None
assert health() is None  # no file yet, no server
with open(path, "w") as f:
    f.write("%d\n" % port)
for _ in range(100):
    if health():
        break
    time.sleep(0.05)
print("HEALTH", health())
"""


def test_dummy_server_port_file_starts_builtin_server(tmp_path):
    """The dummy_server.port watcher (reference src/brpc/global.cpp:223-260):
    while no server runs in the process, writing a port into the watched file
    starts a server of builtin services on it."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    path = str(tmp_path / "dummy_server.port")
    r = subprocess.run([sys.executable, "-c", _DUMMY_SCRIPT, ROOT, path, str(port)], capture_output=True, text=True,
                       timeout=120, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "HEALTH b'OK\\n'" in r.stdout, (r.stdout, r.stderr[-2000:])
