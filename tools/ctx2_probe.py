"""Dev: lc_check32 on the C2 batch from host memory in one context, in a
second context opened beside it, and again alone — does a second context in
the process slow the host path (bench.py's fanout_leg opens one beside the
main loop's)?  Median of 3 calls after a warm-up, with the per-device H2D rate.
    python tools/ctx2_probe.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402

ops, off, _, _ = abi.synth(10000, 1000, concurrency=20, seed=0x5EED0002)
o32, base = abi.pack32(ops, off)


def run(ctx, tag):
    ts, ds = [], []
    for i in range(4):
        t0 = time.perf_counter()
        ctx.check32(o32, off, base)
        if i:
            ts.append((time.perf_counter() - t0) * 1e3)
            ds.append(ctx.device_stats()[0])
    j = int(np.argsort(ts)[1])
    d = ds[j]
    print(json.dumps({"case": tag, "call_ms": ts[j],
                      "h2d_gb_per_s": d["h2d_bytes"] / (d["h2d_ms"] * 1e-3) / 1e9}), flush=True)


a = abi.Context(device_mask=1)
run(a, "first context alone")
b = abi.Context(device_mask=1)
run(b, "second context, first open")
run(a, "first context, second open")
b.close()
run(a, "first context, second closed")
a.close()
c = abi.Context(device_mask=1)
run(c, "fresh context")
c.close()
