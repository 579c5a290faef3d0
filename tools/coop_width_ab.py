"""Dev A/B: cooperative tier width (LC_HBM_COOP=4 vs 16) against the number
of frontier-search keys (version-less C2-shaped keys, concurrency 20)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jepsen.etcd_amd import abi  # noqa: E402

with abi.Context(device_mask=1) as ctx:
    for nk in (64, 200, 300, 400, 512):
        ops, off, _, _ = abi.synth(nk, 1000, concurrency=20, seed=7)
        ops = ops.copy()
        ops[:, 3] = abi.LC_NIL
        out = {"keys": nk}
        for mode in ("4", "16", "4", "16"):
            os.environ["LC_HBM_COOP"] = mode
            t = time.perf_counter()
            _, r = ctx.check(ops, off)
            out.setdefault(mode, []).append(round((time.perf_counter() - t) * 1e3, 2))
        print(json.dumps(out), flush=True)
