#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (run_counter_collection.csv from several
single-group runs of the same program) per kernel: average counters per
dispatch, duration, achieved HBM bandwidth (FETCH_SIZE + WRITE_SIZE are in
KiB) and instruction mix. Only this framework's kernels are reported.

usage: pmc_summary.py PASS_DIR [PASS_DIR ...] > summary.txt
"""
import collections
import csv
import re
import sys

OURS = re.compile(r"mrpc::gpu::\(anonymous namespace\)::(\w+)")
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E nominal


def short(name):
    m = OURS.search(name)
    return m.group(1) if m else None


def main():
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    counts = collections.defaultdict(lambda: collections.defaultdict(int))
    dur = collections.defaultdict(list)
    grid = {}
    for d in sys.argv[1:]:
        with open(d.rstrip("/") + "/run_counter_collection.csv") as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                if not k:
                    continue
                key = (k, row["Grid_Size"])
                c = row["Counter_Name"]
                sums[key][c] += float(row["Counter_Value"])
                counts[key][c] += 1
                grid[key] = (row["Grid_Size"], row["Workgroup_Size"], row["LDS_Block_Size"], row["VGPR_Count"],
                             row["SGPR_Count"])
                if c in ("SQ_WAVES", "FETCH_SIZE"):
                    dur[key].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    print("# per-kernel PMC summary (averages per dispatch); bandwidth = (FETCH_SIZE+WRITE_SIZE KiB) / duration,"
          " vs %.0f GB/s HBM3E nominal" % HBM_PEAK_GBPS)
    for key in sorted(sums):
        s, n = sums[key], counts[key]
        avg = {c: s[c] / max(1, n[c]) for c in s}
        us = sorted(dur[key])[len(dur[key]) // 2] if dur[key] else 0.0
        g, wg, lds, vgpr, sgpr = grid[key]
        line = "%-28s grid=%-8s wg=%-4s lds=%-6s vgpr=%-3s sgpr=%-3s dur_us=%-9.1f" % (key[0], g, wg, lds, vgpr, sgpr, us)
        if "SQ_WAVES" in avg:
            w = max(avg["SQ_WAVES"], 1)
            line += " waves=%.0f valu/wave=%.0f salu/wave=%.0f lds/wave=%.0f vmem_rd/wave=%.0f vmem_wr/wave=%.0f" % (
                avg["SQ_WAVES"], avg.get("SQ_INSTS_VALU", 0) / w, avg.get("SQ_INSTS_SALU", 0) / w,
                avg.get("SQ_INSTS_LDS", 0) / w, avg.get("SQ_INSTS_VMEM_RD", 0) / w, avg.get("SQ_INSTS_VMEM_WR", 0) / w)
            if avg.get("SQ_BUSY_CYCLES"):
                line += " wave_cycles/busy=%.1f" % (avg.get("SQ_WAVE_CYCLES", 0) / avg["SQ_BUSY_CYCLES"])
        fetch = avg.get("FETCH_SIZE")
        write = avg.get("WRITE_SIZE")
        if fetch is not None or write is not None:
            kib = (fetch or 0) + (write or 0)
            line += " fetch_MiB=%.1f write_MiB=%.1f" % ((fetch or 0) / 1024, (write or 0) / 1024)
            if us > 0:
                gbps = kib * 1024 / (us * 1e-6) / 1e9
                line += " hbm_GBps=%.0f (%.0f%% of peak)" % (gbps, 100 * gbps / HBM_PEAK_GBPS)
        print(line)


if __name__ == "__main__":
    main()
