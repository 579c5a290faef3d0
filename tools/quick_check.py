"""Dev tool: GPU vs oracle parity + timing on several synthetic workloads."""
import sys, time, numpy as np
sys.path.insert(0, '.')
from jepsen.etcd_amd import abi
import oracle
ctx = abi.Context(1)
cases = [
    ("C1", 100, 200, 10, 0.0, 0.0, 0x5EED0001),
    ("C5", 1000, 200, 10, 0.0, 0.1, 0x5EED0005),
    ("C2sub", 200, 1000, 20, 0.0, 0.0, 0x5EED0002),
    ("i1", 300, 100, 8, 0.1, 0.1, 7),
    ("i2", 300, 100, 8, 0.3, 0.1, 8),
    ("info40", 100, 150, 8, 0.4, 0.1, 0x5EED0013),
]
for (name, nk, n, conc, pi, pa, seed) in cases:
    ops, off, lab, _ = abi.synth(nk, n, concurrency=conc, p_info=pi, p_anomaly=pa, seed=seed)
    t = time.time(); rc, g = ctx.check(ops, off, raise_on_error=False); tg = time.time() - t
    st = ctx.stats()
    _, r = oracle.check(ops, off, algo=oracle.JITC, n_threads=16, max_configs=2000000)
    known = r['verdict'] != -1
    mism = np.nonzero(known & ((g['verdict'] != r['verdict']) | (g['fail_op'] != r['fail_op'])))[0]
    print(name, "rc", rc, "kernel_ms %.3f hbm_ms %.3f hbm_keys %d" % (st['kernel_ms'], st['hbm_kernel_ms'], st['n_hbm_keys']),
          "mismatch", len(mism), "oracle-unknown", int((~known).sum()),
          "gpu verdicts", dict(zip(*[a.tolist() for a in np.unique(g['verdict'], return_counts=True)])),
          "reasons", dict(zip(*[a.tolist() for a in np.unique(g['reason'], return_counts=True)])),
          "maxF", int(g['max_frontier'].max()), flush=True)
    for k in mism[:3]:
        print("  key", k, "gpu", g[k], "ref", r[k])
ops, off, lab, _ = abi.synth(10000, 1000, concurrency=20, seed=0x5EED0002)
for it in range(3):
    rc, g = ctx.check(ops, off)
    s = ctx.stats()
    print("C2 kernel_ms %.3f total_ms %.3f" % (s['kernel_ms'], s['total_ms']), np.unique(g['verdict'], return_counts=True), int(g['max_frontier'].max()))
