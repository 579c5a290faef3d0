import json, sys, time
sys.path.insert(0, ".")
import numpy as np
from jepsen.etcd_amd import abi
with abi.Context(device_mask=1) as ctx:
    for name, kw in (("C4", dict(p_info=0.2, info_frac=0.2, seed=0x5EED0004)),
                     ("C4r1", dict(p_info=0.2, seed=0x5EED0004))):
        ops, off, _, _ = abi.synth(1, 5000, concurrency=50, **kw)
        o = abi.default_opts(flags=abi.LC_FLAG_NO_GAP_TIER, time_budget_ms=40000)
        t = time.perf_counter()
        _, r = ctx.check(ops, off, o)
        s = ctx.stats()
        print(json.dumps({"cfg": name, "wall_s": round(time.perf_counter() - t, 2), "verdict": int(r["verdict"][0]),
                          "reason": int(r["reason"][0]), "explored": int(r["configs_explored"][0]),
                          "max_frontier": int(r["max_frontier"][0]), "hbm_ms": s["hbm_kernel_ms"],
                          "jit_ms": s["jit_kernel_ms"]}), flush=True)
