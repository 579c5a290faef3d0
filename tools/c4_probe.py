"""Dev: C4 (bench.hot_key's two histories) call by call: wall time, the
gap tier's time and the call profile, --reps calls each after a warm-up.
Under rocprofv3 --kernel-trace, tools/kt_timeline.py lists the last call's
dispatches.

    python tools/c4_probe.py [--reps 5] [--only valid|invalid]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from jepsen.etcd_amd import abi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    out = {}
    with abi.Context(1) as ctx:
        for tag, anom, seed in (("valid", 0.0, 0x5EED0004), ("invalid", 1.0, 1007)):
            if a.only and a.only != tag:
                continue
            ops, off, _, _ = abi.synth(1, 5000, concurrency=50, p_info=0.2, info_frac=0.2,
                                       p_anomaly=anom, seed=seed)
            times, gap, kern = [], [], []
            for _ in range(a.reps + 1):
                t0 = time.perf_counter()
                _, r = ctx.check(ops, off)
                times.append((time.perf_counter() - t0) * 1e3)
                st = ctx.stats()
                gap.append(st["gap_kernel_ms"])
                kern.append(st["kernel_ms"])
            out[tag] = {"verdict": int(r["verdict"][0]), "fail_op": int(r["fail_op"][0]),
                        "call_ms": [round(x, 3) for x in times[1:]],
                        "median_ms": float(np.median(times[1:])),
                        "gap_kernel_ms": float(np.median(gap[1:])),
                        "kernel_ms": float(np.median(kern[1:])),
                        "profile": ctx.call_profile()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
