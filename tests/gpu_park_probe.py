"""Fiber-aware GPU waits, end to end (run by tests/test_gpu_ops.py in its own
process so the runtime can be sized to 2 workers): 8 fibers each wait for a
kernel that runs 100 ms while a closed-loop press keeps 32 B echo calls
flowing through the same 2 worker pthreads. If a waiting fiber blocked its
worker, the RPCs would stall for the whole 100 ms."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from brpc_amd import native
    from brpc_amd.models import start_echo_server
    native.set_flag("fiber_concurrency", "2")
    s = start_echo_server("127.0.0.1:0", num_threads=2, gpu_device=0)
    p = native.Press({"server": s.address, "concurrency": 4, "request_size": 32})
    p.run_requests(200)  # warm the connection
    p.reset_stats()
    h = native.gpu.park_start(8, 100000, 0)
    t0 = time.perf_counter()
    p.run_for(0.08)  # entirely inside the kernels' 100 ms
    dt = time.perf_counter() - t0
    st = p.stats()
    waited, rcs = native.gpu.park_join(h)
    s.stop()
    print(json.dumps({"calls": st["success"], "errors": st["error"], "p99_us": st["p99_us"], "max_us": st["max_us"],
                      "press_s": dt, "waited_us": waited, "rcs": rcs}))


if __name__ == "__main__":
    main()
