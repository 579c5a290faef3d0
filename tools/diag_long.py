"""Dev tool: find GPU/oracle mismatches on longer keys."""
import sys, numpy as np
sys.path.insert(0, '.')
from jepsen.etcd_amd import abi
import oracle
with abi.Context(1) as ctx:
    for (nk, n, conc, seed) in [(2, 200000, 40, 3), (50, 5000, 40, 3), (200, 2000, 40, 4), (200, 2000, 20, 5), (500, 300, 64, 6)]:
        ops, off, _, _ = abi.synth(nk, n, concurrency=conc, seed=seed)
        _, g = ctx.check(ops, off, raise_on_error=False)
        _, j = oracle.check(ops, off, algo=oracle.JITC, n_threads=16)
        bad = np.nonzero((g['verdict'] != j['verdict']) | (g['fail_op'] != j['fail_op']))[0]
        print(nk, n, conc, "mismatch", len(bad), "gpu", np.unique(g['verdict'], return_counts=True), "reasons", np.unique(g['reason'], return_counts=True), "maxF", g['max_frontier'].max(), j['max_frontier'].max(), flush=True)
        for k in bad[:3]:
            print("   key", k, "gpu", g[k], "ref", j[k])
