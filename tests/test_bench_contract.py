"""bench.py prints exactly one JSON line with the driver's contract keys;
the distributed path (ring over ranks) is exercised with gloo on CPU."""
import json
import os

import pytest
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_bench_single_rank():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
                        "--requests-per-step", "2000", "--requests-per-step-64k", "500", "--requests-per-step-grpc", "100",
                        "--latency-sample-s", "0.3"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    # nothing but the JSON line on stdout (library banners go to stderr)
    assert r.stdout.strip().splitlines() == [r.stdout.strip()], r.stdout[:500]
    j = lines[0]
    assert KEYS <= set(j)
    assert j["n_gpus"] == 1 and j["steps"] == 3 and j["value"] > 0 and j["errors"] == 0
    assert j["config"]["seq_len"] == 32


@pytest.mark.parametrize("nranks", [2, 3])
def test_bench_multi_rank_gloo(nranks):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nranks),
                        "--master-addr", "127.0.0.1", "--master-port", str(29517 + nranks),
                        os.path.join(ROOT, "bench.py"), "--gpus", str(nranks), "--steps", "2", "--warmup", "1",
                        "--requests-per-step", "1000", "--requests-per-step-64k", "300",
                        "--requests-per-step-fanout", "100", "--requests-per-step-grpc", "50",
                        "--latency-sample-s", "0.3", "--workers", "2", "--rccl-stub", "--requests-per-step-1m", "20",
                        "--sweep-seconds", "0.05", "--stream-min-s", "0.2"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    j = lines[0]
    assert j["n_gpus"] == nranks and j["value"] > 0 and j["errors"] == 0
    # multi-rank legs: stream fan-out to the other ranks, ParallelChannel fan-out
    assert j["stream_fanout_per_rank"] == nranks - 1 and j["stream_gbytes_per_s_64KB_chunks"] > 0
    assert j["fanout_peers_per_rank"] == nranks - 1 and j["fanout_errors"] == 0 and j["fanout_gbytes_per_s"] > 0
    assert j["scatter_errors"] == 0 and j["scatter_gbytes_per_s"] > 0
    assert j["route_errors"] == 0 and j["route_calls_per_s"] > 0
    # the RCCL payload plane (stub library on the CPU) carried the rccl legs
    # between all ranks, without aborts, and the JSON says so per leg
    assert j["rccl_world"] == nranks and j["rccl_aborts"] == 0 and j["rccl_64KB_errors"] == 0
    assert j["transport"]["rccl_64KB"]["rccl_payloads"] > 0
    assert j["rccl_1MB_errors"] == 0 and j["transport"]["rccl_1MB"]["rccl_payloads"] > 0
    assert j["errors_1MB"] == 0 and j["qps_1MB"] > 0
    assert all(p["errors"] == 0 for p in j["sweep"])
    assert "rccl_crossover_bytes" in j
    assert j["stream_timed_s"] >= 0.2
    # the host-only handler twin, and the CPU cost of every leg
    assert j["errors_64KB_cpu_handler"] == 0 and j["qps_64KB_cpu_handler"] > 0
    assert all(v > 0 for v in j["cpu_us_per_rpc"].values()) and "cpu_handler_64KB" in j["cpu_us_per_rpc"]
    # the codec paths per body kind (gRPC/baidu_std + snappy on text and
    # random bodies, http + json), CPU side here; compressed legs report
    # their body's snappy ratio
    for leg in ("grpc_snappy_64KB_text", "grpc_snappy_64KB_random", "baidu_std_snappy_64KB_text",
                "baidu_std_snappy_64KB_random", "http_json_64KB_text", "baidu_std_snappy_ids16k", "http_json_ids16k"):
        assert j[leg + "_errors"] == 0 and j[leg + "_qps_cpu"] > 0 and leg + "_cpu" in j["cpu_us_per_rpc"]
    assert 2.0 < j["baidu_std_snappy_64KB_text_snappy_ratio"] < 5.0
    assert j["grpc_snappy_64KB_random_snappy_ratio"] <= 1.01
    assert "error_detail" not in j and "vs_baseline_64KB" not in j
    assert j["p99_us_at_100qps_before_move"] > 0
    if nranks > 2:  # a relay chain needs at least two other ranks
        assert j["pipeline_hops"] == nranks - 1 and j["pipeline_gbytes_per_s"] > 0


SMALL = ["--steps", "3", "--warmup", "1", "--requests-per-step", "2000", "--requests-per-step-64k", "500",
         "--requests-per-step-grpc", "100", "--latency-sample-s", "0.3", "--skip-1m", "--skip-grpc"]


def test_bench_leg_deadline_cuts_a_stalled_leg():
    """A leg that overruns its deadline is cut, says so, and the run moves
    on to the next legs: the JSON line is complete."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + SMALL +
                       ["--leg-deadline-s", "3", "--stall-leg", "echo_64KB_host"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    j = lines[0]
    assert j["timed_out_legs"] == ["echo_64KB_host"] and "incomplete" not in j
    assert j["leg_wall_s"]["echo_64KB_host"] < 6.0
    # the legs after the stalled one ran
    assert j["qps_64KB_cpu_handler"] > 0 and j["stream_gbytes_per_s_64KB_chunks"] > 0 and j["p99_us_at_100qps"] > 0
    assert j["value"] > 0 and j["errors"] == 0


def test_bench_watchdog_prints_partial_json_on_hang():
    """A leg that never returns (a hung native call or collective): the
    watchdog prints what was measured, names the leg, and ends the rank."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + SMALL +
                       ["--hard-deadline-s", "30", "--stall-leg", "cpu_handler_64KB:hang"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    j = lines[0]
    assert j["incomplete"] is True and j["hung_leg"] == "cpu_handler_64KB"
    assert KEYS <= set(j) and j["value"] > 0 and j["qps_64KB"] > 0
    assert "qps_64KB_cpu_handler" not in j


def test_bench_watchdog_two_ranks():
    """The same at two ranks over gloo: every rank ends, torchrun returns,
    rank 0's JSON holds the legs before the hang."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29541",
                        os.path.join(ROOT, "bench.py"), "--gpus", "2"] + SMALL +
                       ["--workers", "2", "--requests-per-step-fanout", "100", "--stream-min-s", "0.2",
                        "--hard-deadline-s", "40", "--stall-leg", "scatter_64KB:hang"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    j = lines[0]
    assert j["incomplete"] is True and j["hung_leg"] == "scatter_64KB"
    assert j["n_gpus"] == 2 and j["fanout_errors"] == 0 and j["fanout_gbytes_per_s"] > 0


SPAWN = ["--steps", "2", "--warmup", "1", "--requests-per-step", "2000", "--requests-per-step-64k", "300",
         "--workers", "2", "--latency-sample-s", "0", "--skip-rccl"]


def _cpu_env(**kw):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(kw)
    return env


def test_bench_spawns_its_own_ranks():
    """`bench.py --gpus N` without torchrun starts N ranks itself: one JSON
    line (rank 0's), n_gpus == N, the ring over N ranks."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--only",
                        "echo_32B,echo_64KB_host"] + SPAWN,
                       capture_output=True, text=True, timeout=300, cwd="/tmp", env=_cpu_env())
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    j = lines[0]
    assert j["n_gpus"] == 3 and j["value"] > 0 and j["errors"] == 0
    assert j["config"]["parallelism"].startswith("ring3") and j["qps_64KB"] > 0
    assert "[Gloo]" not in r.stdout


def test_bench_rank_count_mismatch_fails():
    """A launcher that started a different number of ranks than --gpus asks
    for must not produce a curve point."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"] + SPAWN,
                       capture_output=True, text=True, timeout=120, cwd="/tmp", env=_cpu_env(WORLD_SIZE="1"))
    assert r.returncode != 0
    assert _json_lines(r.stdout) == []
    assert "refusing" in r.stderr


def test_bench_spawned_rank_failure_ends_the_job():
    """One self-launched rank dies before the rendezvous: the parent kills
    the rest after the grace period and exits non-zero (no hang)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--only", "echo_32B",
                        "--fail-rank", "1", "--spawn-grace-s", "3"] + SPAWN,
                       capture_output=True, text=True, timeout=120, cwd="/tmp", env=_cpu_env())
    assert r.returncode != 0
    assert _json_lines(r.stdout) == []
    assert "exited with status 3" in r.stderr
