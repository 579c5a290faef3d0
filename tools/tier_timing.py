"""Dev probe: per-tier device times on the BASELINE configs (C1, C4, C5) and
a crash-heavy C2 variant, with and without the gap tier."""
import json
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402

CFGS = {
    "C1": dict(n_keys=100, ops_per_key=200, concurrency=10, seed=0x5EED0001),
    "C4": dict(n_keys=1, ops_per_key=5000, concurrency=50, p_info=0.2, seed=0x5EED0004),
    "C4x": dict(n_keys=1, ops_per_key=5000, concurrency=50, p_info=0.2, p_anomaly=1.0, seed=1006),
    "C5": dict(n_keys=1000, ops_per_key=200, concurrency=10, p_anomaly=0.1, seed=0x5EED0005),
    "C2info": dict(n_keys=10000, ops_per_key=1000, concurrency=20, p_info=0.05, seed=0x5EED0012),
}
with abi.Context(device_mask=1) as ctx:
    for name, kw in CFGS.items():
        n_keys = kw.pop("n_keys")
        opk = kw.pop("ops_per_key")
        ops, off, lab, ninv = abi.synth(n_keys, opk, **kw)
        modes = [(0, "default")]
        if name != "C2info":  # the JIT + HBM tiers take minutes there
            modes.append((abi.LC_FLAG_NO_GAP_TIER, "no-gap"))
        for flags, tag in modes:
            o = abi.default_opts(flags=flags)
            ctx.check(ops, off, o)  # warm
            t = time.perf_counter()
            _, r = ctx.check(ops, off, o)
            wall = (time.perf_counter() - t) * 1e3
            s = ctx.stats()
            v = np.bincount(r["verdict"] + 1, minlength=3)
            print(json.dumps({"cfg": name, "mode": tag, "keys": n_keys, "ops": int(off[-1]),
                              "wall_ms": round(wall, 3),
                              "fast_ms": round(s["fast_kernel_ms"], 4),
                              "gap_ms": round(s["gap_kernel_ms"], 4), "n_gap": s["n_gap_keys"],
                              "jit_ms": round(s["jit_kernel_ms"], 4), "n_jit": s["n_jit_keys"],
                              "hbm_ms": round(s["hbm_kernel_ms"], 3), "n_hbm": s["n_hbm_keys"],
                              "unknown": int(v[0]), "invalid": int(v[1]), "valid": int(v[2])}))
            sys.stdout.flush()
