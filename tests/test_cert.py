"""Infeasibility certificates on the CPU: the certificate checker
(oracle/cert.c) against the oracle's decisions, and its soundness.

An invalid key's certificate names facts that rule out every linearization
of the prefix at its failing return (include/lincheck.h, LC_CERT_*).  The
checker accepts it from the records alone.  Here: the finder's restatement
(tests/cert_ref.py, the device's cert_kernel in Python) certifies the
oracle's own failing prefixes, and no certificate at all — the finder's, or
random ones — is ever accepted on a prefix the oracle finds linearizable
(the prefix just before each failing return, and valid keys' histories)."""
import os
import random

import numpy as np

import oracle
import cert_ref
from helpers import GOLDEN, INF, dup_versions, pack_keys, tiny_batch
from jepsen.etcd_amd import abi


def _sets():
    out = [("tiny", tiny_batch(4321, 3000, max_ops=8))]
    for (name, nk, n, conc, pi, pa, seed) in [
            ("c5", 300, 200, 10, 0.0, 0.5, 0x5EED0005),
            ("conc20", 150, 300, 20, 0.0, 0.6, 31),
            ("crash", 300, 80, 8, 0.2, 0.5, 32),
            ("crash_long", 60, 200, 12, 0.1, 0.6, 33)]:
        ops, off, _, _ = abi.synth(nk, n, concurrency=conc, p_info=pi, p_anomaly=pa, seed=seed)
        out.append((name, [ops[off[k]:off[k + 1]].tolist() for k in range(nk)]))
    out.append(("dup", dup_versions(out[1][1], 34, frac=0.8)))
    z = np.load(os.path.join(GOLDEN, "branch.npz"))
    out.append(("branch", [z["ops"][z["key_off"][k]:z["key_off"][k + 1]].tolist()
                           for k in range(len(z["key_off"]) - 1)]))
    return out


def _certs(keys, cuts):
    cert = np.zeros(4 * len(keys), dtype=np.int32)
    cset = np.zeros(sum(len(k) for k in keys), dtype=np.int32)
    base = 0
    for i, recs in enumerate(keys):
        if cuts[i] >= 0:
            kind, a, b, c, ps = cert_ref.find([tuple(r) for r in recs], int(cuts[i]))
            cert[4 * i: 4 * i + 4] = (kind, a, b, c)
            cset[base: base + len(ps)] = ps
        base += len(recs)
    return cert, cset


def _res(cuts):
    r = np.zeros(len(cuts), dtype=oracle.RESULT_DTYPE)
    r["fail_prefix_end"] = cuts
    return r


def pinned_key(recs):
    """Every :ok mutation carries a version and no read is [nil x]: the keys
    the version-order and gap tiers decide (the others only a search does;
    certificates do not cover them)."""
    return not any(r[5] != INF and r[3] == -1 and (r[0] != 0 or r[1] != -1) for r in recs)


def test_certificates_of_the_oracles_failing_prefixes():
    """Every invalid version-pinned key the oracle decides gets a certificate
    the checker accepts, at the oracle's failing return."""
    total = 0
    kinds = {}
    for name, keys in _sets():
        ops, off = pack_keys(keys)
        _, j = oracle.check(ops, off, algo=oracle.JITC, n_threads=8, max_configs=1 << 20)
        cuts = np.where(j["verdict"] == 0, j["fail_prefix_end"], -1)
        cert, cset = _certs(keys, cuts)
        st = oracle.check_certificate(ops, off, cert, cset, _res(cuts))
        inv = (j["verdict"] == 0) & np.array([pinned_key(k) for k in keys])
        bad = np.nonzero(inv & (st != oracle.CERT_OK))[0]
        assert len(bad) == 0, (name, [(int(k), cert[4 * k: 4 * k + 4].tolist()) for k in bad[:5]])
        assert not ((j["verdict"] == 0) & (st == oracle.CERT_BAD)).any(), name
        total += int(inv.sum())
        for k in np.nonzero(inv)[0]:
            kinds[oracle.CERT_KINDS[int(cert[4 * k])]] = kinds.get(oracle.CERT_KINDS[int(cert[4 * k])], 0) + 1
    assert total > 900, (total, kinds)
    assert {"dup", "pair", "order", "hall", "claims", "unreach", "proof"} <= set(kinds), kinds


def test_no_certificate_passes_on_a_linearizable_prefix():
    """Soundness: on the prefix just before each failing return (which the
    oracle finds linearizable) and on valid keys' whole histories, the
    checker rejects the finder's certificates from the failing prefix and
    random certificates of every kind."""
    rng = random.Random(5)
    checked = 0
    for name, keys in _sets():
        ops, off = pack_keys(keys)
        _, j = oracle.check(ops, off, algo=oracle.JITC, n_threads=8, max_configs=1 << 20)
        inv = j["verdict"] == 0
        cuts = np.where(inv, j["fail_prefix_end"], -1)
        cert, cset = _certs(keys, cuts)
        # the linearizable cuts: the return before each failing one; a valid
        # key's last event
        lin_cut = np.full(len(keys), -1, dtype=np.int64)
        for i, recs in enumerate(keys):
            rets = sorted(r[5] for r in recs if r[5] != INF)
            if inv[i]:
                earlier = [x for x in rets if x < cuts[i]]
                lin_cut[i] = earlier[-1] if earlier else -1
            elif j["verdict"][i] == 1 and recs:
                lin_cut[i] = max(max(r[4] for r in recs), rets[-1] if rets else 0)
        use = lin_cut >= 0
        st = oracle.check_certificate(ops, off, cert, cset, _res(lin_cut))
        assert not (use & (st == oracle.CERT_OK)).any(), name
        # the finder itself, run on the linearizable prefixes, finds nothing
        # the checker accepts (and nothing at all: its conditions are the
        # checker's)
        fc, fs = _certs(keys, lin_cut)
        st = oracle.check_certificate(ops, off, fc, fs, _res(lin_cut))
        assert not (use & (st == oracle.CERT_OK)).any(), name
        assert not (use & (fc[0::4] != 0) & np.array([pinned_key(k) for k in keys])).any(), name
        for trial in range(6):
            rc = np.zeros_like(cert)
            rs = np.zeros_like(cset)
            base = 0
            for i, recs in enumerate(keys):
                n = max(1, len(recs))
                kind = rng.randrange(1, 8)
                c = rng.randrange(0, n) if kind < 6 else rng.randrange(1, n + 1)
                rc[4 * i: 4 * i + 4] = (kind, rng.randrange(-1, n), rng.randrange(0, n), c)
                for g in range(len(recs)):
                    rs[base + g] = (rng.randrange(0, n + 1) if kind != 7 else
                                    cert_ref.tok(rng.randrange(1, 4), rng.randrange(0, n + 1),
                                                 rng.randrange(0, n)))
                base += len(recs)
            st = oracle.check_certificate(ops, off, rc, rs, _res(lin_cut))
            assert not (use & (st == oracle.CERT_OK)).any(), (name, trial)
        checked += int(use.sum())
    assert checked > 2000


def test_tampered_certificates_are_rejected():
    """Hand-made failing prefix: w1 ok [1 1], w2 ok [2 2], then a read of
    [1 1] invoked after both returned (KAT2's stale read).  ORDER(read, w2)
    is its certificate; the same facts with the records swapped, a read of
    another version, or a Hall set with a position some op can hold are not."""
    W, R = 1, 0
    recs = [[W, 1, -1, 1, 0, 1], [W, 2, -1, 2, 2, 3], [R, 1, -1, 1, 4, 5]]
    ops, off = pack_keys([recs])
    res = _res(np.array([5]))
    cases = [((5, 2, 1, 0), [], oracle.CERT_OK),       # the stale read after w2's return
             ((5, 1, 2, 0), [], oracle.CERT_BAD),      # swapped
             ((5, 2, 0, 0), [], oracle.CERT_BAD),      # w1 bounds nothing after the read
             ((1, 0, 1, 0), [], oracle.CERT_BAD),      # not one version
             ((6, -1, -1, 1), [0], oracle.CERT_BAD),   # position 0 is held
             ((4, 0, 2, 1), [], oracle.CERT_BAD),      # the read reads w1's value: no clash
             ((0, 0, 0, 0), [], oracle.CERT_NONE)]
    for c, ps, want in cases:
        cset = np.zeros(3, dtype=np.int32)
        cset[:len(ps)] = ps
        st = oracle.check_certificate(ops, off, np.array(c, dtype=np.int32), cset, res)
        assert st[0] == want, (c, st[0])
    got = cert_ref.find([tuple(r) for r in recs], 5)
    assert got[0] == cert_ref.ORDER and got[1:3] == (2, 1)


def test_branch_fixture_needs_and_gets_a_proof():
    """tests/golden/branch.npz (make_branch.py): invalid version-pinned keys
    whose failing prefix no fixed certificate kind covers — the fixed
    stages alone find nothing — get an LC_CERT_PROOF the checker accepts.
    The oracle's verdicts and failing returns are the fixture's."""
    z = np.load(os.path.join(GOLDEN, "branch.npz"))
    ops, off = z["ops"], z["key_off"]
    keys = [ops[off[k]:off[k + 1]].tolist() for k in range(len(off) - 1)]
    _, j = oracle.check(ops, off, algo=oracle.JITC, n_threads=8)
    assert (j["verdict"] == 0).all() and (j["fail_op"] == z["fail_op"]).all()
    assert (j["fail_prefix_end"] == z["fail_prefix_end"]).all()
    cuts = z["fail_prefix_end"]
    for i, recs in enumerate(keys):
        assert cert_ref.find([tuple(r) for r in recs], int(cuts[i]), proof=False)[0] == cert_ref.NONE
    cert, cset = _certs(keys, cuts)
    assert (cert[0::4] == cert_ref.PROOF).all()
    st = oracle.check_certificate(ops, off, cert, cset, _res(cuts))
    assert (st == oracle.CERT_OK).all(), np.nonzero(st != oracle.CERT_OK)[0][:5]


def test_tampered_proofs_are_rejected():
    """Every proof of the branch fixture, tampered: cut short, a case split
    counting one case fewer or more or of another kind, a token too many
    — the checker rejects each (it follows the proof step by step).  The
    finder's proofs themselves: most are propagation alone (no token)."""
    z = np.load(os.path.join(GOLDEN, "branch.npz"))
    ops, off = z["ops"], z["key_off"]
    keys = [ops[off[k]:off[k + 1]].tolist() for k in range(len(off) - 1)]
    cuts = z["fail_prefix_end"]
    cert, cset = _certs(keys, cuts)
    n_checked = 0
    lens = []
    for i in range(len(keys)):
        c, b = int(cert[4 * i + 3]), int(off[i])
        toks = [int(x) for x in cset[b:b + c]]
        lens.append(c)
        variants = [toks + [cert_ref.tok(cert_ref.BRANCH, 0, 2)]]
        if c > 0:
            variants.append(toks[:-1])
        for t in range(c):
            kind, a, x = cert_ref.untok(toks[t])
            # (a split at another position may be another valid proof: not here)
            for v in (cert_ref.tok(kind, a, x - 1), cert_ref.tok(kind, a, x + 1),
                      cert_ref.tok(cert_ref.FORCE, a, x)):
                variants.append(toks[:t] + [v] + toks[t + 1:])
        for v in variants:
            if len(v) > len(keys[i]) or v == toks:
                continue
            one = np.zeros(len(keys[i]), dtype=np.int32)
            one[:len(v)] = v
            st = oracle.check_certificate(np.array(keys[i], dtype=np.int64), np.array([0, len(keys[i])]),
                                          np.array([cert_ref.PROOF, -1, -1, len(v)], dtype=np.int32),
                                          one, _res(np.array([cuts[i]])))
            assert st[0] == oracle.CERT_BAD, (i, toks, v)
            n_checked += 1
    assert n_checked > 100 and max(lens) >= 1, (n_checked, lens)


def test_proof_search_budget_is_the_cap():
    """helpers.proof_cap_key: invalid, and refutable only by a case analysis
    of 2,047 splits.  At the finder's budget (2,048 nodes, the device's
    cert.hip kNodes) the PROOF search gives up — no certificate, never a
    wrong one — and with a larger budget the same finder's proof is accepted
    by the checker: what stops it is the node cap, not the token room (one
    token per record of the key)."""
    from helpers import proof_cap_key
    recs = proof_cap_key()
    ops, off = pack_keys([recs])
    _, j = oracle.check(ops, off, algo=oracle.JITC, n_threads=1, max_configs=1 << 22)
    assert j["verdict"][0] == 0 and j["fail_op"][0] == 34
    cut = int(j["fail_prefix_end"][0])
    assert cert_ref.find([tuple(r) for r in recs], cut)[0] == cert_ref.NONE
    kind, a, b, c, toks = cert_ref.find([tuple(r) for r in recs], cut, proof_budget=1 << 16)
    assert kind == cert_ref.PROOF and c == len(toks) == 2047 <= len(recs)
    cert = np.array([kind, a, b, c], dtype=np.int32)
    cset = np.zeros(len(recs), dtype=np.int32)
    cset[:c] = toks
    assert oracle.check_certificate(ops, off, cert, cset, _res(np.array([cut])))[0] == oracle.CERT_OK
