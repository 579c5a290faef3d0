"""Dev: version-less (cas-register) batches at several key counts: call time,
tier times, HBM keys (which tier shape the library picks)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jepsen.etcd_amd import abi  # noqa: E402

with abi.Context(device_mask=1) as ctx:
    for nk, n, conc in ((1000, 1000, 20), (4000, 1000, 20), (10000, 1000, 20), (10000, 200, 10)):
        ops, off, _, _ = abi.synth(nk, n, concurrency=conc, seed=7)
        ops = ops.copy()
        ops[:, 3] = abi.LC_NIL
        o = abi.default_opts(time_budget_ms=20000)
        ctx.check(ops, off, o)
        t = time.perf_counter()
        _, r = ctx.check(ops, off, o)
        ms = (time.perf_counter() - t) * 1e3
        s = ctx.stats()
        print(json.dumps({"keys": nk, "ops": n, "conc": conc, "call_ms": round(ms, 2),
                          "jit_ms": round(s["jit_kernel_ms"], 2), "hbm_ms": round(s["hbm_kernel_ms"], 2),
                          "n_jit": s["n_jit_keys"], "n_hbm": s["n_hbm_keys"],
                          "configs": int(r["configs_explored"].sum()),
                          "unknown": int((r["verdict"] == -1).sum())}), flush=True)
