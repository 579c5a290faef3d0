"""Dev probe: the C2 batch with versions stripped (= knossos cas-register
model on the same histories): every key goes fast tier -> gap tier (not
applicable) -> JIT search.  Per-tier device times."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402

with abi.Context(device_mask=1) as ctx:
    for keys, opk, conc, pinf in ((10000, 1000, 20, 0.0), (10000, 1000, 20, 0.05), (1000, 200, 10, 0.0)):
        ops, off, _, _ = abi.synth(keys, opk, concurrency=conc, p_info=pinf, seed=7)
        ops = ops.copy()
        ops[:, 3] = -1  # no versions: cas-register
        for flags, tag in ((0, "default"), (abi.LC_FLAG_NO_GAP_TIER, "no-gap")):
            o = abi.default_opts(flags=flags, time_budget_ms=1000)
            ctx.check(ops, off, o)
            t = time.perf_counter()
            _, r = ctx.check(ops, off, o)
            wall = time.perf_counter() - t
            s = ctx.stats()
            print(json.dumps({"keys": keys, "opk": opk, "p_info": pinf, "mode": tag,
                              "wall_ms": round(wall * 1e3, 3), "fast_ms": round(s["fast_kernel_ms"], 4),
                              "gap_ms": round(s["gap_kernel_ms"], 4), "jit_ms": round(s["jit_kernel_ms"], 4),
                              "hbm_ms": round(s["hbm_kernel_ms"], 3), "n_jit": s["n_jit_keys"],
                              "verdicts": np.bincount(r["verdict"] + 1, minlength=3).tolist()}), flush=True)
