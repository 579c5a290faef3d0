"""Dev probe: run one bench.py leg's workload N times (for rocprofv3 passes
that must see only that leg's kernels).
  python tools/leg.py crash|crashdev|model|hot|hotx|mixed|search|fx [reps]
crash: C2 with 5 % crashed writes/CAS from host buffers (lc_check: chunked copies, a fused
       pass per chunk); crashdev: the same batch resident on the GPU (lc_check_device: one
       fused_tier_kernel launch per call, as bench.py's crash_leg)
mixed: C5, 1000 keys x 200 ops, 10 % anomalies (fast_tier_kernel, then
       gap_light_kernel: the first-failure rule)
model: cas-register model, 1000 keys x 1000 ops, concurrency 20 (lds_tier,
       hbm_coop_kernel<4>)
hot / hotx: C4 at 20 % crashed, valid / invalid (gap_tier_kernel)
search: C2 with the version-order and gap tiers off (lds_tier_kernel)
fx: bench.py's oversized key through the frontier exchange (fx_expand_kernel)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402

leg = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
if leg in ("crash", "crashdev"):
    ops, off, _, _ = abi.synth(10000, 1000, concurrency=20, p_info=0.05, seed=0x5EED0012)
elif leg == "mixed":
    ops, off, _, _ = abi.synth(1000, 200, concurrency=10, p_anomaly=0.1, seed=0x5EED0005)
elif leg == "model":
    ops, off, _, _ = abi.synth(1000, 1000, concurrency=20, seed=7)
    ops = ops.copy()
    ops[:, 3] = abi.LC_NIL
elif leg == "search":  # C2 through the JIT search tier only (lds_tier_kernel)
    ops, off, _, _ = abi.synth(10000, 1000, concurrency=20, seed=0x5EED0002)
elif leg == "fx":  # bench.py's oversized key through the frontier exchange (fx_expand_kernel)
    ops, off, _, _ = abi.synth(1, 2000, concurrency=50, seed=0x5EED0004)
    ops = ops.copy()
    ops[:, 3] = abi.LC_NIL
elif leg in ("hot", "hotx"):
    ops, off, _, _ = abi.synth(1, 5000, concurrency=50, p_info=0.2, info_frac=0.2,
                               p_anomaly=1.0 if leg == "hotx" else 0.0,
                               seed=1007 if leg == "hotx" else 0x5EED0004)
else:
    raise SystemExit("unknown leg " + leg)
if leg == "fx":
    from jepsen.etcd_amd.fx import FrontierExchange
    with FrontierExchange(device=0) as fx:
        for i in range(reps):
            t = time.perf_counter()
            r = fx.check(ops)
            print(json.dumps({"leg": leg, "rep": i, "wall_ms": (time.perf_counter() - t) * 1e3,
                              "configs": int(r["configs_explored"]), "verdict": int(r["verdict"]),
                              "stats": fx.stats()}))
    raise SystemExit(0)
if leg == "crashdev":  # as bench.py's crash_leg: resident records, lc_check_device (one fused launch)
    import torch
    dev = torch.device("cuda", 0)
    d_ops = torch.from_numpy(np.ascontiguousarray(ops)).to(dev)
    d_off = torch.from_numpy(np.ascontiguousarray(off)).to(dev)
    d_out = torch.zeros((len(off) - 1) * abi.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    with abi.Context(device_mask=1) as ctx:
        for i in range(reps + 1):  # the first call picks the fused pass for the next
            t = time.perf_counter()
            ctx.check_device(d_ops.data_ptr(), d_off.data_ptr(), len(off) - 1, d_out.data_ptr())
            torch.cuda.synchronize()
            s = ctx.stats()
            print(json.dumps({"leg": leg, "rep": i, "wall_ms": (time.perf_counter() - t) * 1e3,
                              "fast_ms": s["fast_kernel_ms"], "gap_ms": s["gap_kernel_ms"]}), flush=True)
    raise SystemExit(0)
opts = abi.default_opts(flags=abi.LC_FLAG_NO_FAST_PATH) if leg == "search" else None
with abi.Context(device_mask=1) as ctx:
    for i in range(reps):
        t = time.perf_counter()
        _, r = ctx.check(ops, off, opts)
        s = ctx.stats()
        print(json.dumps({"leg": leg, "rep": i, "wall_ms": (time.perf_counter() - t) * 1e3,
                          "fast_ms": s["fast_kernel_ms"], "gap_ms": s["gap_kernel_ms"],
                          "jit_ms": s["jit_kernel_ms"], "hbm_ms": s["hbm_kernel_ms"],
                          "configs": int(r["configs_explored"].sum()),
                          "verdicts": np.bincount(r["verdict"] + 1, minlength=3).tolist()}),
              flush=True)
