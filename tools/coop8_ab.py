"""Dev A/B: cooperative workgroup width 4 / 8 / 16 on version-less batches."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jepsen.etcd_amd import abi  # noqa: E402

with abi.Context(device_mask=1) as ctx:
    for nk, n, conc in ((64, 1000, 20), (128, 1000, 20), (256, 1000, 20), (400, 1000, 20), (512, 1000, 20), (700, 1000, 20)):
        ops, off, _, _ = abi.synth(nk, n, concurrency=conc, seed=7)
        ops = ops.copy()
        ops[:, 3] = abi.LC_NIL
        out = {"keys": nk}
        for mode in ("4", "8", "16", "8", "16"):
            os.environ["LC_HBM_COOP"] = mode
            t = time.perf_counter()
            _, r = ctx.check(ops, off)
            out.setdefault(mode, []).append(round(ctx.stats()["hbm_kernel_ms"], 2))
        print(json.dumps(out), flush=True)
