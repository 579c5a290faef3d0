"""Regenerates tests/golden/branch.npz (run from the repo root): invalid
version-pinned keys whose failing prefix none of the fixed certificate kinds
covers — DUP, UNREACH, CLAIMS, PAIR, ORDER, HALL at the root — because its
infeasibility shows only in a search over who holds the open positions (the
gap matching's branching).  Their certificates are LC_CERT_PROOF
(include/lincheck.h).

Random crash-heavy keys with two or three values (helpers.random_tiny with
high crash and perturbation rates, and the product's seeded generator at
concurrency 4-8); the oracle's JIT and WGL restatements must agree on the
verdict and (JIT) give the failing return; tests/cert_ref.py's fixed stages
must find nothing at it.  Deterministic (seeded); stops at 120 keys.

Holds ops (n,6), key_off, verdict (all 0), fail_op and fail_prefix_end per key.
"""
import os
import random
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from jepsen.etcd_amd import abi  # noqa: E402
import oracle  # noqa: E402
import cert_ref  # noqa: E402
from helpers import INF, pack_keys, random_tiny  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
WANT = 120


def pinned_key(recs):
    return not any(r[5] != INF and r[3] == -1 and (r[0] != 0 or r[1] != -1) for r in recs)


def main():
    rng = random.Random(0x5EED00B1)
    found = []
    b = 0
    while len(found) < WANT:
        keys = [random_tiny(rng, rng.randrange(6, 13), p_info=rng.choice([0.3, 0.5, 0.7]),
                            p_perturb=0.8, n_values=rng.choice([2, 3])) for _ in range(2000)]
        ops, off, _, _ = abi.synth(300, rng.choice([40, 60, 90]), concurrency=rng.choice([4, 6, 8]),
                                   n_values=rng.choice([2, 3]), p_info=rng.choice([0.3, 0.5]),
                                   p_anomaly=1.0, seed=0x5EED00B1 + b)
        keys += [ops[off[k]:off[k + 1]].tolist() for k in range(300)]
        keys = [k for k in keys if pinned_key(k)]
        ops, off = pack_keys(keys)
        _, j = oracle.check(ops, off, algo=oracle.JIT, n_threads=8, max_configs=1 << 20)
        _, w = oracle.check(ops, off, algo=oracle.WGL, n_threads=8, max_configs=1 << 20)
        for i in np.nonzero((j["verdict"] == 0) & (w["verdict"] == 0))[0]:
            cut = int(j["fail_prefix_end"][i])
            # the fixed stages only (the proof search switched off)
            if cert_ref.find([tuple(r) for r in keys[i]], cut, proof=False)[0] == cert_ref.NONE:
                found.append((keys[i], int(j["fail_op"][i]), cut))
                if len(found) == WANT:
                    break
        b += 1
    ops, off = pack_keys([k for k, _, _ in found])
    np.savez_compressed(os.path.join(OUT, "branch.npz"), ops=ops, key_off=off,
                        verdict=np.zeros(len(found), dtype=np.int32),
                        fail_op=np.array([f for _, f, _ in found], dtype=np.int64),
                        fail_prefix_end=np.array([c for _, _, c in found], dtype=np.int64))
    print("branch.npz: %d keys, %d records, %d batches" % (len(found), len(ops), b))


if __name__ == "__main__":
    main()
