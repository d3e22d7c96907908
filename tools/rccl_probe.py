#!/usr/bin/env python3
"""Probe: can two ranks share ONE GPU in an RCCL communicator (p2p
send/recv)? Run: torchrun --nproc-per-node 2 tools/rccl_probe.py"""
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    dev = int(os.environ.get("PROBE_DEVICE", "0"))
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
    t = torch.full((1 << 20,), rank + 1, dtype=torch.uint8, device="cuda")
    t0 = time.time()
    if rank == 0:
        dist.send(t, 1)
        r = torch.empty_like(t)
        dist.recv(r, 1)
    else:
        r = torch.empty_like(t)
        dist.recv(r, 0)
        dist.send(t, 0)
    torch.cuda.synchronize()
    print("rank %d got %d in %.3f s" % (rank, int(r[0].item()), time.time() - t0), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
