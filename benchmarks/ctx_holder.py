"""Holds a GPU context for N seconds (what another process on the same GPU
looks like to the hardware scheduler): `torch` (torch.cuda init + sync),
`native` (brpc_amd's runtime: HBM arena, xGMI lender, pool streams), or
`both`."""
import sys
import time

mode = sys.argv[1] if len(sys.argv) > 1 else "torch"
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
import torch  # noqa: E402
if mode in ("torch", "both"):
    torch.cuda.set_device(0)
    torch.ones(1, device="cuda").sum().item()
    torch.cuda.synchronize()
if mode in ("native", "both"):
    sys.path.insert(0, ".")
    from brpc_amd import native  # noqa: E402
    native.gpu.init(0)
    native.gpu.enable_xgmi(0)
print("holding %s context" % mode, flush=True)
time.sleep(secs)
