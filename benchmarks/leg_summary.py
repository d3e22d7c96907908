#!/usr/bin/env python3
"""One line per leg of a bench.py JSON: QPS / GB/s, p99, errors, host
microseconds per RPC, transport verdict. Used by tools/gpurun/box.sh."""
import json
import sys


def main(path):
    j = json.loads(open(path).read().splitlines()[-1])
    cpu = j.get("cpu_us_per_rpc", {})
    tok = j.get("transport_ok", {})
    print("n_gpus=%s value=%s p99=%s wall=%s%s" % (j["n_gpus"], j["value"], j.get("p99_us"), j.get("wall_s"),
                                                  " INCOMPLETE" if j.get("incomplete") else ""))
    for k, v in sorted(j.items()):
        if isinstance(v, (int, float)) and any(s in k for s in ("qps", "gbytes", "calls_per_s", "ratio", "fraction")):
            leg = k
            print("  %-48s %12s" % (leg, v))
    for k, v in sorted(cpu.items()):
        print("  cpu_us %-41s %8s %s" % (k, v, "" if k not in tok else ("transport ok" if tok[k] else "TRANSPORT BAD")))
    for k in ("timed_out_legs", "failed_legs", "skipped_legs", "error_detail", "transport_problems", "perf_ok"):
        if k in j:
            print("  %s: %s" % (k, j[k]))
    for k, v in sorted(j.get("diag", {}).items()):
        print("  diag %-43s %s" % (k, v))
    for k, v in j.items():
        if k.endswith("_device") and isinstance(v, dict):
            print("  %s: %s" % (k, v))


if __name__ == "__main__":
    main(sys.argv[1])
