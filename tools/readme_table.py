#!/usr/bin/env python3
"""Regenerate README.md's measured table from one bench.py JSON.

Every number in the table between the `<!-- bench-table:begin ... -->` and
`<!-- bench-table:end -->` markers comes from the JSON named on the command
line (default: the newest profiles/*bench*.json), so the README never quotes
a number the committed evidence does not hold. Legs the JSON lacks are left
out rather than filled from older runs.

  python tools/readme_table.py [--json profiles/r5_bench_final.json] [--check]
"""
import argparse
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BEGIN = "<!-- bench-table:begin"
END = "<!-- bench-table:end -->"


def k(v):
    return "%.1f k" % (v / 1e3) if v < 1e6 else "%.2f M" % (v / 1e6)


def us(d, key):
    v = (d.get("cpu_us_per_rpc") or {}).get(key)
    return "%.1f" % v if isinstance(v, (int, float)) else "—"


def rows(d):
    out = []

    def add(leg, value, host, ref="—"):
        out.append("| %s | %s | %s | %s |" % (leg, value, host, ref))

    if "value" in d:
        add("Echo 32 B (headline)", "**%s QPS**, p99 %s µs" % (k(d["value"]), d.get("p99_us")), us(d, "echo_32B"),
            "≈215 k QPS")
    if "qps_64KB" in d:
        add("Echo 64 KiB, HBM attachments lent zero-copy",
            "**%s QPS** (%.1f GB/s), p99 %s µs" % (k(d["qps_64KB"]), d.get("gbytes_per_s_64KB", 0), d.get("p99_us_64KB")),
            us(d, "echo_64KB"), "32 KB: ≈29 k single / ≈72 k pooled")
    if "qps_64KB_host_attachment" in d:
        add("Echo 64 KiB, host attachments (TCP)", "%s QPS, p99 %s µs" % (k(d["qps_64KB_host_attachment"]),
                                                                          d.get("p99_us_64KB_host_attachment")),
            us(d, "echo_64KB_host"))
    if "qps_1MB" in d:
        add("Echo 1 MiB, HBM attachments", "**%s QPS, %.0f GB/s**, p99 %s µs" % (k(d["qps_1MB"]),
                                                                                d.get("gbytes_per_s_1MB", 0),
                                                                                d.get("p99_us_1MB")),
            us(d, "echo_1MB"))
    for pre, proto in (("", "baidu_std"), ("grpc_", "h2/gRPC")):
        for body in ("text", "random"):
            leg = "%sdevice_snappy_64KB_%s" % (pre, body)
            q = d.get(leg + "_qps")
            if q is None:
                continue
            dev = d.get(leg + "_device") or {}
            add("Device-body codec over %s, 64 KiB protobuf in HBM, %s body (snappy on the device both ways, "
                "pb-indexed)" % (proto, body),
                "%s QPS, ratio %s, encoded %.0f%% / decoded %.0f%% of payloads" % (
                    k(q), dev.get("device_ratio", "?"), 100 * d.get(leg + "_encoded_fraction", 0),
                    100 * d.get(leg + "_decoded_fraction", 0)),
                us(d, leg))
    for proto in ("grpc", "baidu_std"):
        for body in ("text", "random"):
            base = "%s_snappy_64KB_%s" % (proto, body)
            if base + "_qps_cpu" not in d:
                continue
            g = d.get(base + "_qps_gpu")
            add("%s 64 KiB protobuf, snappy both ways, %s body (ratio %s)" % (proto, body, d.get(base + "_snappy_ratio")),
                "CPU codec %s%s" % (k(d[base + "_qps_cpu"]), "" if g is None else " vs GPU codec %s" % k(g)),
                "%s%s" % (us(d, base + "_cpu"), "" if g is None else " vs " + us(d, base + "_gpu")))
    for name, label in (("baidu_std_snappy_ids16k", "baidu_std + snappy, 16 k packed int64 ids"),
                        ("http_json_ids16k", "http + json, 16 k ids")):
        if name + "_qps_cpu" in d:
            g = d.get(name + "_qps_gpu")
            add(label, "CPU %s%s" % (k(d[name + "_qps_cpu"]), "" if g is None else " vs GPU %s" % k(g)),
                "%s%s" % (us(d, name + "_cpu"), "" if g is None else " vs " + us(d, name + "_gpu")))
    if "http_json_64KB_text_qps_cpu" in d:
        add("http + json, 64 KiB text string field (host only: the JSON offload's density gate leaves a long string "
            "field to the host)",
            "%s QPS" % k(d["http_json_64KB_text_qps_cpu"]), us(d, "http_json_64KB_text_cpu"))
    if "rccl_self_copy_64KB_qps" in d:
        add("Echo 64 KiB / 1 MiB through the one-rank RCCL plane: self payloads moved by the plane's copy kernel "
            "(NOT RCCL; -rccl_self_copy)",
            "%s QPS / %s QPS (%.0f GB/s), %s aborts" % (k(d["rccl_self_copy_64KB_qps"]),
                                                        k(d.get("rccl_self_copy_1MB_qps", 0)),
                                                        d.get("rccl_self_copy_1MB_gbytes_per_s", 0),
                                                        d.get("rccl_aborts")),
            us(d, "rccl_64KB"))
    if "rccl_nccl_self_64KB_qps" in d:
        add("Echo 64 KiB through ncclSend/ncclRecv to self (one-rank plane, -rccl_self_copy=false)",
            "%s QPS, p99 %s µs, %s µs per group" % (k(d["rccl_nccl_self_64KB_qps"]), d.get("rccl_nccl_self_64KB_p99_us"),
                                                    d.get("rccl_nccl_self_group_us_per_round")),
            us(d, "rccl_nccl_self_64KB"))
    if "rccl_64KB_qps" in d:
        add("Echo 64 KiB / 1 MiB over the RCCL plane (%s-rank communicator)" % d.get("rccl_world"),
            "%s QPS / %s QPS (%.0f GB/s), %s aborts" % (k(d["rccl_64KB_qps"]), k(d.get("rccl_1MB_qps", 0)),
                                                        d.get("rccl_1MB_gbytes_per_s", 0), d.get("rccl_aborts")),
            us(d, "rccl_64KB"))
    if "qps_64KB_gpu_handler" in d:
        add("GPU handler, TCP-delivered 64 KiB, CRC32C on the device (%s)" % d.get("gpu_handler_note", ""),
            "%s vs %s for the host-CRC twin" % (k(d["qps_64KB_gpu_handler"]), k(d.get("qps_64KB_cpu_handler", 0))),
            "%s vs %s" % (us(d, "gpu_handler_64KB"), us(d, "cpu_handler_64KB")))
    if "stream_gbytes_per_s_64KB_chunks" in d:
        add("Streaming RPC, 64 KiB HBM chunks", "%.1f GB/s per stream" % d["stream_gbytes_per_s_64KB_chunks"], "—")
    if "p99_us_at_100qps" in d:
        add("`rpc_press -qps=100` latency", "p50 %s µs, p99 %s µs, p999 %s µs" % (
            d["p50_us_at_100qps"], d["p99_us_at_100qps"], d.get("p999_us_at_100qps")),
            "%s%% of one CPU" % d.get("cpu_pct_at_100qps"), "p99 172 µs")
    return out


def newest():
    c = sorted(glob.glob(os.path.join(ROOT, "profiles", "*bench*.json")), key=os.path.getmtime)
    return c[-1] if c else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--readme", default=os.path.join(ROOT, "README.md"))
    ap.add_argument("--check", action="store_true", help="exit 1 if the README table differs")
    a = ap.parse_args()
    path = a.json or newest()
    if not path:
        sys.exit("no bench JSON")
    d = json.load(open(path))
    rel = os.path.relpath(path, ROOT)
    table = ["%s source=%s -->" % (BEGIN, rel),
             "Generated by `tools/readme_table.py` from `%s` (N=%s, %s warmup / %s timed steps)." % (
                 rel, d.get("n_gpus"), d.get("warmup"), d.get("steps")), "",
             "| Leg | Value | Host CPU µs/RPC | Reference (BASELINE.md) |", "|---|---|---|---|"]
    table += rows(d)
    table.append(END)
    text = open(a.readme).read()
    m = re.search(re.escape(BEGIN) + r".*?" + re.escape(END), text, re.S)
    if not m:
        sys.exit("README has no bench-table markers")
    new = text[:m.start()] + "\n".join(table) + text[m.end():]
    if a.check:
        sys.exit(0 if new == text else 1)
    open(a.readme, "w").write(new)
    print("README table <- %s (%d legs)" % (rel, len(table) - 6))


if __name__ == "__main__":
    main()
