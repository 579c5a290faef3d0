"""Regenerates the committed golden fixtures (run from the repo root):

  c1.npz    BASELINE configs[0] shape: 100 keys x 200 ops, concurrency 10
  c5.npz    configs[4] shape (300-key slice): 10% keys with an injected stale
            read or lost CAS
  info.npz  300 keys x 100 ops, concurrency 8, 10% of mutations crashed
  tiny.npz  2000 random tiny histories (<= 6 ops) incl. nil fields and crashes

Each holds ops (n,6), key_off, and the expected verdict / fail_op per key.
Expected values come from the CPU oracle: JIT and WGL restatements must agree
on every key (and brute force on tiny.npz), else the script aborts.  The
generator is the product's own seeded lc_synth_register (deterministic).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from jepsen.etcd_amd import abi  # noqa: E402
import oracle  # noqa: E402
from oracle import brute  # noqa: E402
import helpers  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def agreed(ops, off, tiny=False):
    _, j = oracle.check(ops, off, algo=oracle.JIT, n_threads=8)
    _, w = oracle.check(ops, off, algo=oracle.WGL, n_threads=8)
    assert (j["verdict"] != -1).all() and (j["verdict"] == w["verdict"]).all()
    if tiny:
        for k in range(len(off) - 1):
            recs = [tuple(r) for r in ops[off[k]:off[k + 1]]]
            assert brute.check(recs) == (j["verdict"][k] == 1)
            assert brute.first_failure(recs) == j["fail_op"][k]
    return j["verdict"].astype(np.int32), j["fail_op"].astype(np.int64)


def save(name, ops, off, extra=None):
    v, f = agreed(ops, off, tiny=(name == "tiny"))
    np.savez_compressed(os.path.join(OUT, name + ".npz"), ops=ops, key_off=off,
                        verdict=v, fail_op=f, **(extra or {}))
    print(name, len(off) - 1, "keys", len(ops), "records", int((v == 0).sum()), "invalid")


if __name__ == "__main__":
    ops, off, lab, _ = abi.synth(100, 200, concurrency=10, seed=0x5EED0001)
    save("c1", ops, off)
    ops, off, lab, _ = abi.synth(300, 200, concurrency=10, p_anomaly=0.1, seed=0x5EED0005)
    save("c5", ops, off, {"label": lab})
    ops, off, lab, _ = abi.synth(300, 100, concurrency=8, p_info=0.1, p_anomaly=0.1, seed=7)
    save("info", ops, off)
    ops, off = helpers.pack_keys(helpers.tiny_batch(20261015, 2000))
    save("tiny", ops, off)
