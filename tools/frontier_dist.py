"""Dev probe: max-frontier distribution of version-less (cas-register) keys
of the C2 shape, JIT + HBM tiers."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402

with abi.Context(device_mask=1) as ctx:
    for keys, opk, conc, pinf in ((1000, 1000, 20, 0.0), (1000, 1000, 10, 0.0), (1000, 200, 10, 0.0)):
        ops, off, _, _ = abi.synth(keys, opk, concurrency=conc, p_info=pinf, seed=7)
        ops = ops.copy()
        ops[:, 3] = -1
        t = time.perf_counter()
        _, r = ctx.check(ops, off, abi.default_opts(time_budget_ms=1000))
        wall = time.perf_counter() - t
        s = ctx.stats()
        mf = r["max_frontier"]
        print(json.dumps({"keys": keys, "opk": opk, "conc": conc, "wall_ms": round(wall * 1e3, 1),
                          "jit_ms": round(s["jit_kernel_ms"], 3), "hbm_ms": round(s["hbm_kernel_ms"], 1),
                          "n_hbm": s["n_hbm_keys"],
                          "mf_pct": [int(np.percentile(mf, q)) for q in (50, 90, 99, 100)],
                          "configs_pct": [int(np.percentile(r["configs_explored"], q)) for q in (50, 90, 99, 100)],
                          "verdicts": np.bincount(r["verdict"] + 1, minlength=3).tolist()}), flush=True)
