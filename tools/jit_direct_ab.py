"""Dev A/B: frontier-search keys straight to the cooperative tier (default
for <= 4096 keys) against the LDS tier first (LC_JIT_DIRECT=0), on
version-less batches of several shapes: call time, tier times, verdicts."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402

CASES = [("model 1000x1000 c20", 1000, 1000, 20, 0.0),
         ("small 1000x200 c10", 1000, 200, 10, 0.0),
         ("small 4000x100 c8", 4000, 100, 8, 0.0),
         ("crashy 500x150 c10 info", 500, 150, 10, 0.05),
         ("few 64x1000 c16", 64, 1000, 16, 0.0)]
with abi.Context(device_mask=1) as ctx:
    for name, nk, n, conc, pinfo in CASES:
        ops, off, _, _ = abi.synth(nk, n, concurrency=conc, p_info=pinfo, seed=11)
        ops = ops.copy()
        ops[:, 3] = abi.LC_NIL
        o = abi.default_opts(time_budget_ms=20000)
        res = {}
        for mode in ("0", "1", "0", "1"):
            os.environ["LC_JIT_DIRECT"] = mode
            t = time.perf_counter()
            _, r = ctx.check(ops, off, o)
            ms = (time.perf_counter() - t) * 1e3
            s = ctx.stats()
            res.setdefault(mode, []).append(ms)
            key = (tuple(r["verdict"]), tuple(r["fail_op"]))
            res.setdefault("v" + mode, key)
        print(json.dumps({"case": name, "lds_first_ms": [round(x, 2) for x in res["0"]],
                          "direct_ms": [round(x, 2) for x in res["1"]],
                          "same_results": res["v0"] == res["v1"],
                          "valid": int((np.array(res["v1"][0]) == 1).sum()),
                          "unknown": int((np.array(res["v1"][0]) == -1).sum())}), flush=True)
