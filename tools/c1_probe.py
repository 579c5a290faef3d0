"""Dev: where C1's host-buffer call goes (BASELINE configs[0]: 100 keys x 200
ops): lc_check and lc_check32 call times with the library's call profile and
per-device stats, median of 20 calls after warm-up.
    python tools/c1_probe.py"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402

ops, off, _, _ = abi.synth(100, 200, concurrency=10, seed=0x5EED0001)
o32, base = abi.pack32(ops, off)
out = {}
with abi.Context(device_mask=1) as ctx:
    for name, call in (("check", lambda: ctx.check(ops, off)),
                       ("check32", lambda: ctx.check32(o32, off, base))):
        for _ in range(5):
            call()
        ts, profs, stats = [], [], []
        for _ in range(20):
            t0 = time.perf_counter()
            call()
            ts.append((time.perf_counter() - t0) * 1e3)
            profs.append(ctx.call_profile())
            stats.append(ctx.stats())
        i = int(np.argsort(ts)[len(ts) // 2])
        out[name] = {"call_ms_median": float(np.median(ts)), "call_ms_min": float(min(ts)),
                     "profile": profs[i],
                     "stats": {k: v for k, v in stats[i].items() if isinstance(v, (int, float))}}
print(json.dumps(out, indent=1))
