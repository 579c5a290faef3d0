import json, os, sys, time
sys.path.insert(0, ".")
from jepsen.etcd_amd import abi
with abi.Context(device_mask=1) as ctx:
    for nk, n, conc in ((10000, 1000, 20), (6000, 1000, 20), (10000, 300, 12)):
        ops, off, _, _ = abi.synth(nk, n, concurrency=conc, seed=7)
        ops = ops.copy(); ops[:, 3] = abi.LC_NIL
        o = abi.default_opts(time_budget_ms=20000)
        for mode in ("1", "4"):
            os.environ["LC_HBM_COOP"] = mode
            ctx.check(ops, off, o)
            t = time.perf_counter(); _, r = ctx.check(ops, off, o); ms = (time.perf_counter() - t) * 1e3
            s = ctx.stats()
            print(json.dumps({"keys": nk, "ops": n, "conc": conc, "coop": mode, "call_ms": round(ms, 2),
                              "jit_ms": round(s["jit_kernel_ms"], 2), "hbm_ms": round(s["hbm_kernel_ms"], 2),
                              "n_hbm": s["n_hbm_keys"], "configs": int(r["configs_explored"].sum())}), flush=True)
