"""Shared test helpers: tiny random register histories, fixture loading."""
import json
import os
import random

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
INF = (1 << 63) - 1
R, W, C, N = 0, 1, 2, -1


def load_kats():
    with open(os.path.join(GOLDEN, "kat.json")) as fh:
        return json.load(fh)


def pack_keys(list_of_ops):
    """[[record...] per key] -> (ops (n,6) int64, key_off)."""
    key_off = np.zeros(len(list_of_ops) + 1, dtype=np.int64)
    rows = []
    for i, ops in enumerate(list_of_ops):
        key_off[i + 1] = key_off[i] + len(ops)
        rows.extend(ops)
    ops = np.array(rows, dtype=np.int64).reshape(-1, 6)
    return ops, key_off


def _step(state, f, value, expected, version):
    ver, val = state
    if f == W:
        return (ver + 1, value)
    if f == C:
        return (ver + 1, value) if val == expected else None
    return state


def random_tiny(rng, n_ops, p_info=0.2, p_perturb=0.35, n_values=3):
    """A small history: a random sequential execution whose ops get random
    overlapping intervals around their linearization points, then (with
    p_perturb) one field perturbed.  Mix of valid and invalid keys, nil
    versions/values, crashed ops (some never take effect)."""
    # linearization order = op order; intervals from random event positions
    state = (0, N)
    recs = []
    for _ in range(n_ops):
        f = rng.choice([R, R, W, C])
        info = f != R and rng.random() < p_info
        if f == R:
            ver, val = state
            rec = [R, val if ver > 0 else N, N, ver if ver > 0 else N]
            if rng.random() < 0.15:
                rec[1] = N  # version-only read
        elif f == W:
            v = rng.randrange(n_values)
            took = not info or rng.random() < 0.5
            if took:
                state = (state[0] + 1, v)
            rec = [W, v, N, N if info else state[0]]
        else:
            old = rng.choice([state[1], rng.randrange(n_values)])
            new = rng.randrange(n_values)
            ok = state[1] == old
            if not ok and not info:
                continue  # a failed CAS is dropped by history completion
            took = ok and (not info or rng.random() < 0.5)
            if took:
                state = (state[0] + 1, new)
            rec = [C, new, old, N if info else state[0]]
        recs.append((rec, info))
    n = len(recs)
    # lin point of op i at time 2i+1; call uniformly before, ret after
    ops = []
    times = []
    for i, (rec, info) in enumerate(recs):
        lin = 10 * i + 5
        call = lin - rng.randrange(1, 25)
        ret = INF if info else lin + rng.randrange(1, 25)
        times.append((call, ret))
        ops.append(rec)
    # rank event times into distinct indices (calls before rets at ties)
    ev = []
    for i, (c, r) in enumerate(times):
        ev.append((c, 0, i))
        if r != INF:
            ev.append((r, 1, i))
    ev.sort()
    cidx, ridx = {}, {}
    for k, (_, kind, i) in enumerate(ev):
        (ridx if kind else cidx)[i] = k
    out = []
    for i, rec in enumerate(ops):
        out.append(rec + [cidx[i], ridx.get(i, INF)])
    out.sort(key=lambda r: r[4])
    if out and rng.random() < p_perturb:
        j = rng.randrange(len(out))
        fld = rng.choice([1, 3])
        out[j][fld] = rng.choice([N, 0, 1, 2, 3])
        if out[j][0] != C and fld == 2:
            out[j][2] = N
    return out


def tiny_batch(seed, n_keys, max_ops=6):
    rng = random.Random(seed)
    return [random_tiny(rng, rng.randrange(0, max_ops + 1)) for _ in range(n_keys)]


# ---- other knossos models (history.py "Models"): record-level generators
FREE, HELD = 0, 1


def _intervals(rng, n, infos, spread=25):
    """Distinct call/ret indices around linearization points 10i+5."""
    times = []
    for i in range(n):
        lin = 10 * i + 5
        call = lin - rng.randrange(1, spread)
        ret = INF if infos[i] else lin + rng.randrange(1, spread)
        times.append((call, ret))
    ev = []
    for i, (c, r) in enumerate(times):
        ev.append((c, 0, i))
        if r != INF:
            ev.append((r, 1, i))
    ev.sort()
    cidx, ridx = {}, {}
    for k, (_, kind, i) in enumerate(ev):
        (ridx if kind else cidx)[i] = k
    return [(cidx[i], ridx.get(i, INF)) for i in range(n)]


def random_mutex(rng, n_ops, p_info=0.15, p_perturb=0.35):
    """A knossos mutex history as records (acquire = CAS FREE->HELD, release
    = CAS HELD->FREE, no versions, initial state FREE): a random sequential
    run of the lock (an acquire of a held lock or a release of a free one is
    :fail and dropped), crashed ops that take effect with p = 0.5, intervals
    around the linearization points, then (with p_perturb) one op flipped."""
    held = False
    recs, infos = [], []
    for _ in range(n_ops):
        acq = rng.random() < 0.5
        info = rng.random() < p_info
        legal = (not held) if acq else held
        if not legal and not info:
            continue  # :fail, dropped by completion
        if legal and (not info or rng.random() < 0.5):
            held = acq
        recs.append([C, HELD, FREE, N] if acq else [C, FREE, HELD, N])
        infos.append(info)
    out = [r + list(t) for r, t in zip(recs, _intervals(rng, len(recs), infos))]
    out.sort(key=lambda r: r[4])
    if out and rng.random() < p_perturb:
        j = rng.randrange(len(out))
        out[j][1], out[j][2] = out[j][2], out[j][1]  # acquire <-> release
    return out


def random_casreg(rng, n_ops, p_info=0.2, p_perturb=0.35, n_values=3):
    """knossos cas-register records: random_tiny with every version nil."""
    out = random_tiny(rng, n_ops, p_info, p_perturb, n_values)
    for r in out:
        r[3] = N
    return out


def dup_versions(keys, seed, frac=0.5):
    """Copies of keys with one :ok mutation's version given to another
    mutation (two mutations claiming one version: the lost-CAS shape)."""
    rng = random.Random(seed)
    out = []
    for recs in keys:
        muts = [i for i, r in enumerate(recs) if r[0] != 0 and r[3] != -1 and r[5] != INF]
        if len(muts) >= 2 and rng.random() < frac:
            recs = [list(r) for r in recs]
            a, b = rng.sample(muts, 2)
            recs[b][3] = recs[a][3]
        out.append(recs)
    return out


def proof_cap_key(k_free=10, conflict=3, pad=2100):
    """An invalid version-pinned key whose refutation needs a case analysis
    larger than the certificate finder's PROOF search budget (2,048 nodes,
    cert.hip / tests/cert_ref.py) but whose proof would fit the key's
    certificate set (one token per record): positions 0..k_free-1 each need
    a distinct value (a read of version p+1 claims it) and have two crashed
    writes of that value; the last `conflict` positions all need value 99
    and only conflict-1 crashed writes of 99 exist.  The search splits every
    free position before it reaches the conflict, so its tree has ~2^(k_free
    + 2) nodes and 2^(k_free + 1) - 1 case splits.  Reads [nil nil] after the
    failing return pad the key to `pad` records.  Fails at the read of
    version k_free + conflict (record index 3 k_free + 2 conflict + 1)."""
    recs, t = [], 0
    vals = list(range(k_free)) + [99] * conflict
    for p in range(k_free + conflict):
        if p < k_free:
            for _ in range(2):
                recs.append([W, p, N, N, t, INF])
                t += 1
        elif p == k_free:
            for _ in range(conflict - 1):
                recs.append([W, 99, N, N, t, INF])
                t += 1
        recs.append([R, vals[p], N, p + 1, t, t + 1])
        t += 2
    while len(recs) < pad:
        recs.append([R, N, N, N, t, t + 1])
        t += 2
    return recs
