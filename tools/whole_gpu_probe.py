"""Probe: several oversized version-less keys through lc_check with
LC_FLAG_WHOLE_GPU (concurrent frontier-exchange engines) against one
FrontierExchange engine taking them one after another.
    python tools/whole_gpu_probe.py [n_keys] [ops] [conc]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402
from jepsen.etcd_amd.fx import FrontierExchange  # noqa: E402

nk = int(sys.argv[1]) if len(sys.argv) > 1 else 4
nops = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
conc = int(sys.argv[3]) if len(sys.argv) > 3 else 40
ops, off, _, _ = abi.synth(nk, nops, concurrency=conc, seed=0x5EED0004)
ops = ops.copy()
ops[:, 3] = abi.LC_NIL
budget = 1 << 22
o = abi.default_opts(max_configs_per_key=budget, flags=abi.LC_FLAG_WHOLE_GPU)
with abi.Context(1) as ctx:
    ctx.check(ops, off, o)
    t0 = time.perf_counter()
    _, r = ctx.check(ops, off, o)
    t_conc = (time.perf_counter() - t0) * 1e3
    _, plain = ctx.check(ops, off, abi.default_opts(max_configs_per_key=budget))
with FrontierExchange(device=0) as fx:
    for k in range(nk):
        fx.check(ops[off[k]:off[k + 1]], abi.default_opts(max_configs_per_key=budget))
    t0 = time.perf_counter()
    seq = [fx.check(ops[off[k]:off[k + 1]], abi.default_opts(max_configs_per_key=budget))
           for k in range(nk)]
    t_seq = (time.perf_counter() - t0) * 1e3
same = all(int(seq[k][f]) == int(r[f][k]) for k in range(nk)
           for f in ("verdict", "configs_explored", "max_frontier"))
print(json.dumps({"keys": nk, "ops": nops, "conc": conc,
                  "tiers_unknown": int((plain["verdict"] == -1).sum()),
                  "whole_gpu_call_ms": t_conc, "fx_sequential_ms": t_seq, "same_results": same,
                  "verdicts": r["verdict"].tolist(),
                  "explored": r["configs_explored"].tolist()}))
