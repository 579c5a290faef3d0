"""Dev probe: gap-tier timings on C4 (valid), C4x (invalid) and C5 (mixed),
several calls each; with a GAP_PROFILE build (tools/build_variants.sh prof
-DGAP_PROFILE, LINCHECK_LIB=...) the kernel also prints per-stage clocks."""
import json
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import numpy as np  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402

CFGS = {
    "C4": dict(n_keys=1, ops_per_key=5000, concurrency=50, p_info=0.2, info_frac=0.2, seed=0x5EED0004),
    "C4x": dict(n_keys=1, ops_per_key=5000, concurrency=50, p_info=0.2, info_frac=0.2, p_anomaly=1.0, seed=1007),
    "C4x1004": dict(n_keys=1, ops_per_key=5000, concurrency=50, p_info=0.2, info_frac=0.2, p_anomaly=1.0, seed=1004),
    "C4r1": dict(n_keys=1, ops_per_key=5000, concurrency=50, p_info=0.2, seed=0x5EED0004),
    "C5": dict(n_keys=1000, ops_per_key=200, concurrency=10, p_anomaly=0.1, seed=0x5EED0005),
    "C5big": dict(n_keys=10000, ops_per_key=200, concurrency=10, p_info=0.1, p_anomaly=0.1, seed=77),
    "C2info": dict(n_keys=10000, ops_per_key=1000, concurrency=20, p_info=0.05, seed=0x5EED0012),
}
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
if len(sys.argv) > 2:
    CFGS = {k: v for k, v in CFGS.items() if k in sys.argv[2].split(",")}
with abi.Context(device_mask=1) as ctx:
    for name, kw in CFGS.items():
        kw = dict(kw)
        ops, off, _, _ = abi.synth(kw.pop("n_keys"), kw.pop("ops_per_key"), **kw)
        for i in range(reps):
            t = time.perf_counter()
            _, r = ctx.check(ops, off)
            wall = (time.perf_counter() - t) * 1e3
            s = ctx.stats()
            v = np.bincount(r["verdict"] + 1, minlength=3)
            print(json.dumps({"cfg": name, "rep": i, "wall_ms": round(wall, 3),
                              "gap_ms": round(s["gap_kernel_ms"], 4),
                              "fast_ms": round(s["fast_kernel_ms"], 4),
                              "jit_ms": round(s["jit_kernel_ms"], 4),
                              "nodes": int(r["configs_explored"].max()),
                              "invalid": int(v[1]), "valid": int(v[2]), "unknown": int(v[0]),
                              "reason": int(r["reason"].max())}),
                  flush=True)
