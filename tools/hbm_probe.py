"""Dev probe: workloads that push keys through the HBM tier (gap tier off),
with the tier's time and configurations explored."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402

with abi.Context(device_mask=1) as ctx:
    # LC_HBM_COOP: 0 wavefront per key, 4/16 workgroup of that many per key, 1 auto
    for mode in (sys.argv[1] if len(sys.argv) > 1 else "0,1").split(","):
        os.environ["LC_HBM_COOP"] = mode
        for keys, opk, conc, pinf, nover in ((256, 200, 12, 0.2, 0), (256, 300, 16, 0.2, 0),
                                             (64, 400, 20, 0.2, 0), (512, 150, 10, 0.3, 0),
                                             (64, 300, 20, 0.0, 1), (16, 1000, 20, 0.02, 1), (200, 1000, 20, 0.0, 1),
                                             (1000, 1000, 20, 0.0, 1), (2000, 1000, 20, 0.0, 1),
                                             (10000, 1000, 20, 0.0, 1)):
            ops, off, _, _ = abi.synth(keys, opk, concurrency=conc, p_info=pinf, seed=99)
            if nover:
                ops[:, 3] = -1
            o = abi.default_opts(flags=abi.LC_FLAG_NO_GAP_TIER, time_budget_ms=2000)
            t = time.perf_counter()
            _, r = ctx.check(ops, off, o)
            wall = time.perf_counter() - t
            s = ctx.stats()
            hot = r["reason"] != 0
            print(json.dumps({"coop": mode, "nover": nover, "keys": keys, "opk": opk, "conc": conc, "p_info": pinf,
                              "wall_s": round(wall, 3), "jit_ms": round(s["jit_kernel_ms"], 3),
                              "hbm_ms": round(s["hbm_kernel_ms"], 3), "n_hbm": s["n_hbm_keys"],
                              "configs": int(r["configs_explored"].sum()),
                              "max_frontier": int(r["max_frontier"].max()),
                              "verdicts": np.bincount(r["verdict"] + 1, minlength=3).tolist(),
                              "reasons": np.bincount(r["reason"], minlength=8).tolist()}), flush=True)
