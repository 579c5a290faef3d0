"""Dev tool: print GPU/oracle mismatches for one synthetic configuration."""
import sys, numpy as np
sys.path.insert(0, '.')
from jepsen.etcd_amd import abi
import oracle
conc, pi, pa, seed = int(sys.argv[1]), float(sys.argv[2]), float(sys.argv[3]), int(sys.argv[4])
ops, off, lab, _ = abi.synth(400, 200, concurrency=conc, p_info=pi, p_anomaly=pa, seed=seed)
with abi.Context(1) as ctx:
    _, g = ctx.check(ops, off)
    print(ctx.stats())
_, j = oracle.check(ops, off, algo=oracle.JITC, n_threads=16, max_configs=1 << 21)
m = np.nonzero((j['verdict'] != -1) & ((g['verdict'] != j['verdict']) | (g['fail_op'] != j['fail_op'])))[0]
print("mismatches", len(m))
for k in m[:20]:
    print(k, "gpu", g[k], "oracle", j[k], "label", lab[k])
