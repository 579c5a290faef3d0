"""Debug probe for the frontier exchange's queue path: the synthetic
version-less keys of test_fx against the oracle's JITC, per env setting."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle  # noqa: E402
from helpers import pack_keys  # noqa: E402
from jepsen.etcd_amd import abi  # noqa: E402
from jepsen.etcd_amd.fx import FrontierExchange  # noqa: E402

F = ("verdict", "fail_op", "configs_explored", "max_frontier")
keys = []
for seed in range(4):
    for i, conc in enumerate((8, 10, 12)):
        ops, off, _, _ = abi.synth(4, 300, concurrency=conc, p_info=0.01, p_anomaly=0.5,
                                   seed=seed * 7 + i + 0x700)
        ops = ops.copy()
        ops[:, 3] = -1
        keys += [ops[off[k]:off[k + 1]] for k in range(4)]
kops, koff = pack_keys([k.tolist() for k in keys])
_, o = oracle.check(kops, koff, algo=oracle.JITC, n_threads=8)
bad = 0
with FrontierExchange(device=0) as fx:
    for rep in range(3):
        for k, ops in enumerate(keys):
            r = fx.check(ops)
            if any(int(r[f]) != int(o[f][k]) for f in F):
                bad += 1
                if bad < 6:
                    print("  key", k, [int(r[f]) for f in F], [int(o[f][k]) for f in F])
print(os.environ.get("TAG", ""), "keys", len(keys) * 3, "mismatches", bad, flush=True)
