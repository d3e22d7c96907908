#!/usr/bin/env python3
"""A/B of the fused workgroup-parallel codec (gpu/codec_fused.hip) against
the per-lane-segment snappy kernels at RPC batch shapes: kernel time per
launch (hipEvents around back-to-back launches), compressed size, parse
rounds. One JSON line per (body kind, block size, bodies per launch).

  python benchmarks/fused_codec_ab.py [--bodies 7,28] [--blocks 2048,4096,8192]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bodies", default="1,7,28")
    ap.add_argument("--blocks", default="2048,4096,8192")
    ap.add_argument("--kinds", default="text,random,const")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from brpc_amd import native
    for kind in a.kinds.replace("+", ",").split(","):
        for nb in [int(x) for x in a.bodies.replace("+", ",").split(",")]:
            bodies = [native.echo_body(kind, 65536) for _ in range(nb)]
            for blk in [int(x) for x in a.blocks.replace("+", ",").split(",")]:
                r = native.gpu.fused_codec_bench(bodies, blk, a.iters, 0)
                r.update({"kind": kind, "bodies": nb, "block": blk})
                print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
