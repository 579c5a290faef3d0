"""Dev: the bench's oversized key through the frontier exchange, a warm-up
check and then --reps timed ones (for a kernel trace: tools/fx_gaps.py reads
rocprofv3 --kernel-trace's CSV of this run).

    python tools/fx_once.py [--reps 1]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from jepsen.etcd_amd import abi  # noqa: E402
from jepsen.etcd_amd.fx import FrontierExchange  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=1)
    a = ap.parse_args()
    ops, _ = bench.oversized_key_ops(abi)
    with FrontierExchange(device=0) as fx:
        fx.check(ops)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            r = fx.check(ops)
            ts.append((time.perf_counter() - t0) * 1e3)
        st = fx.stats()
    print(json.dumps({"ms": ts, "verdict": int(r["verdict"]), "explored": int(r["configs_explored"]),
                      "max_frontier": int(r["max_frontier"]), "stats": st}))


if __name__ == "__main__":
    main()
