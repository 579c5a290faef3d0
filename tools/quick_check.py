import sys, time, numpy as np
sys.path.insert(0, '.')
from jepsen.etcd_amd import abi
import oracle
ctx = abi.Context(1)
for (nk, n, conc, pa, seed) in [(100,200,10,0.0,0x5EED0001),(1000,200,10,0.1,0x5EED0005),(200,1000,20,0.0,0x5EED0002)]:
    ops, off, lab, _ = abi.synth(nk, n, concurrency=conc, p_anomaly=pa, seed=seed)
    t=time.time(); rc, g = ctx.check(ops, off, raise_on_error=False); tg=time.time()-t
    st = ctx.stats()
    _, r = oracle.check(ops, off, algo=oracle.JIT, n_threads=8)
    mism = np.nonzero((g['verdict']!=r['verdict'])|(g['fail_op']!=r['fail_op']))[0]
    print(nk, n, conc, "rc", rc, "t", round(tg*1e3,2), "ms stats", st, "mismatch", len(mism), mism[:5], np.unique(g['verdict'],return_counts=True), "reasons", np.unique(g['reason'],return_counts=True), "maxF", g['max_frontier'].max())
    if len(mism):
        k=mism[0]; print("key",k,g[k],r[k])
ops, off, lab, _ = abi.synth(10000, 1000, concurrency=20, seed=0x5EED0002)
for it in range(3):
    rc, g = ctx.check(ops, off)
    print("C2", ctx.stats(), np.unique(g['verdict'],return_counts=True), g['max_frontier'].max())
