"""Probe: one oversized version-less key through the frontier exchange
(whole GPU) vs lc_check's tiers (one cooperative workgroup per key), and
optionally the oracle's JITC on the host.

    python tools/fx_probe.py --ops 2000 --conc 24 --info 0.002 [--ranks 1] [--oracle]
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
from jepsen.etcd_amd.fx import FrontierExchange  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", type=int, default=2000)
    ap.add_argument("--conc", type=int, default=24)
    ap.add_argument("--info", type=float, default=0.002)
    ap.add_argument("--anomaly", type=float, default=0.0)
    ap.add_argument("--seed", type=int, default=0x5EED0004)
    ap.add_argument("--ranks", type=int, default=1)
    ap.add_argument("--part-above", type=int, default=-1)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("--no-tiers", action="store_true")
    a = ap.parse_args()
    ops, off, _, _ = abi.synth(1, a.ops, concurrency=a.conc, p_info=a.info,
                               p_anomaly=a.anomaly, seed=a.seed)
    ops = ops.copy()
    ops[:, 3] = -1  # cas-register model: no versions
    out = {"ops": a.ops, "conc": a.conc, "info": a.info, "crashed": int((ops[:, 5] == abi.LC_INF).sum())}
    with FrontierExchange(device=0, virtual_ranks=a.ranks, part_above=a.part_above) as fx:
        fx.check(ops)  # warm (allocations)
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            r = fx.check(ops)
            ts.append((time.perf_counter() - t0) * 1e3)
        out["fx"] = {"ms": min(ts), "verdict": int(r["verdict"]), "reason": int(r["reason"]),
                     "fail_op": int(r["fail_op"]), "explored": int(r["configs_explored"]),
                     "max_frontier": int(r["max_frontier"]), "stats": fx.stats()}
    if not a.no_tiers:
        with abi.Context(1) as ctx:
            ctx.check(ops, off)
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                _, res = ctx.check(ops, off)
                ts.append((time.perf_counter() - t0) * 1e3)
            st = ctx.stats()
        out["tiers"] = {"ms": min(ts), "verdict": int(res["verdict"][0]),
                        "reason": int(res["reason"][0]),
                        "explored": int(res["configs_explored"][0]),
                        "max_frontier": int(res["max_frontier"][0]),
                        "hbm_ms": st.get("hbm_kernel_ms") if isinstance(st, dict) else None}
    if a.oracle:
        import oracle
        t0 = time.perf_counter()
        _, ref = oracle.check(ops, off, algo=oracle.JITC, max_configs=1 << 24)
        out["oracle_jitc"] = {"ms": (time.perf_counter() - t0) * 1e3,
                              "verdict": int(ref["verdict"][0]),
                              "explored": int(ref["configs_explored"][0]),
                              "max_frontier": int(ref["max_frontier"][0])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
