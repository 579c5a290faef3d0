"""The CPU oracle against hand-derived known answers and against itself.

Three independent deciders: brute force (definitional), the JIT-linear
restatement of knossos.linear, the WGL restatement of knossos.wgl — plus the
JIT with the eager read closure, which must match plain JIT exactly."""
import numpy as np
import pytest

import oracle
from oracle import brute
from helpers import dup_versions, load_kats, pack_keys, tiny_batch, INF
from jepsen.etcd_amd import abi

KATS = load_kats()


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_brute_force_matches_hand_derived(kat):
    ops = [tuple(o) for o in kat["ops"]]
    assert brute.check(ops) == kat["valid"]
    assert brute.first_failure(ops) == kat["fail_op"]


@pytest.mark.parametrize("algo", [oracle.JIT, oracle.JITC, oracle.WGL], ids=["jit", "jitc", "wgl"])
def test_restatements_match_kats(algo):
    ops, off = pack_keys([k["ops"] for k in KATS])
    rc, r = oracle.check(ops, off, algo=algo)
    assert rc == 0
    for i, k in enumerate(KATS):
        assert r["verdict"][i] == (1 if k["valid"] else 0), k["name"]
        if algo != oracle.WGL:
            assert r["fail_op"][i] == k["fail_op"], k["name"]
            assert r["fail_prefix_end"][i] == k["fail_prefix_end"], k["name"]


def test_step_rules():
    """register.clj:60-96 case by case via the C step function's callers:
    single-op histories with every nil combination."""
    cases = [  # (record, valid from (0, nil))
        ([0, -1, -1, -1, 0, 1], True),    # read [nil nil]
        ([0, -1, -1, 0, 0, 1], True),     # read [0 nil]: version 0 matches
        ([0, 1, -1, -1, 0, 1], False),    # read [nil 1]: value nil != 1
        ([1, 3, -1, -1, 0, 1], True),     # write [nil 3]
        ([1, 3, -1, 1, 0, 1], True),      # write [1 3]
        ([1, 3, -1, 2, 0, 1], False),     # write [2 3]: version' = 1
        ([2, 3, -1, 1, 0, 1], True),      # cas nil->3 [1 ...]
        ([2, 3, 0, -1, 0, 1], False),     # cas 0->3 on nil
    ]
    ops, off = pack_keys([[c[0]] for c in cases])
    for algo in (oracle.JIT, oracle.JITC, oracle.WGL):
        _, r = oracle.check(ops, off, algo=algo)
        assert [bool(v) for v in r["verdict"]] == [c[1] for c in cases]


def test_tiny_random_three_way():
    keys = tiny_batch(12345, 600, max_ops=6)
    ops, off = pack_keys(keys)
    _, j = oracle.check(ops, off, algo=oracle.JIT)
    _, c = oracle.check(ops, off, algo=oracle.JITC)
    _, w = oracle.check(ops, off, algo=oracle.WGL)
    for k, recs in enumerate(keys):
        t = [tuple(x) for x in recs]
        b = brute.check(t)
        assert (j["verdict"][k] == 1) == b
        assert (w["verdict"][k] == 1) == b
        assert c["verdict"][k] == j["verdict"][k]
        assert j["fail_op"][k] == brute.first_failure(t) == c["fail_op"][k]


@pytest.mark.parametrize("name", ["c1", "c5", "info", "tiny"])
def test_golden_fixtures(name):
    import os
    from helpers import GOLDEN
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    for algo in (oracle.JIT, oracle.JITC, oracle.WGL):
        _, r = oracle.check(z["ops"], z["key_off"], algo=algo, n_threads=4)
        assert (r["verdict"] == z["verdict"]).all()
        if algo != oracle.WGL:
            assert (r["fail_op"] == z["fail_op"]).all()


@pytest.mark.parametrize("mode", ["READ_CLOSURE", "CRASH_SYMMETRY", "RETIRE", "DEADLINE_ORDER", "ALL"])
@pytest.mark.parametrize("p_info,seed", [(0.05, 99), (0.15, 7)])
def test_reductions_are_exact_on_synthetic(mode, p_info, seed):
    """Each exact reduction (oracle.c) agrees with the faithful knossos.linear
    search on every key both decide: verdict and canonical fail op."""
    flag = oracle.JITC if mode == "ALL" else oracle.JIT | getattr(oracle, mode)
    ops, off, _, _ = abi.synth(150, 100, concurrency=8, p_info=p_info, p_anomaly=0.2,
                               seed=seed)
    _, j = oracle.check(ops, off, algo=oracle.JIT, n_threads=4, max_configs=200000)
    _, c = oracle.check(ops, off, algo=flag, n_threads=4, max_configs=200000)
    known = (j["verdict"] != -1) & (c["verdict"] != -1)
    assert known.mean() > 0.8
    assert (j["verdict"][known] == c["verdict"][known]).all()
    assert (j["fail_op"][known] == c["fail_op"][known]).all()
    if mode == "ALL":  # the reductions never lose a decision the plain search makes
        assert ((j["verdict"] != -1) <= (c["verdict"] != -1)).all()


def test_crash_symmetry_kat():
    """Three identical crashed writes and a read needing two of them: the
    symmetric search considers prefixes only, with the same verdict."""
    recs = [[1, 4, -1, -1, 0, INF], [1, 4, -1, -1, 1, INF], [1, 4, -1, -1, 2, INF],
            [0, 4, -1, 2, 3, 4], [0, 4, -1, 4, 5, 6]]
    ops, off = pack_keys([recs, recs[:4]])
    _, j = oracle.check(ops, off, algo=oracle.JIT)
    _, c = oracle.check(ops, off, algo=oracle.JITC)
    assert list(j["verdict"]) == [0, 1] == list(c["verdict"])
    assert list(j["fail_op"]) == [4, -1] == list(c["fail_op"])
    assert brute.check([tuple(r) for r in recs]) is False


def test_malformed_and_unknown_f():
    bad_order = [[1, 1, -1, 1, 5, 6], [1, 2, -1, 2, 3, 4]]       # calls not increasing
    bad_ret = [[1, 1, -1, 1, 5, 5]]                               # ret <= call
    unknown_f = [[7, 1, -1, 1, 0, 1]]
    ops, off = pack_keys([bad_order, bad_ret, unknown_f, [[1, 1, -1, 1, 0, 1]]])
    rc, r = oracle.check(ops, off)
    assert rc != 0
    assert list(r["reason"]) == [4, 4, 5, 0]
    assert list(r["verdict"]) == [-1, -1, -1, 1]


def test_budget_gives_unknown():
    # many concurrent crashed writes: the faithful search must give up
    recs = [[1, v % 3, -1, -1, i, INF] for i, v in enumerate(range(20))]
    recs.append([0, 2, -1, 21, 30, 31])
    ops, off = pack_keys([recs])
    _, r = oracle.check(ops, off, algo=oracle.JIT, max_configs=1000)
    assert r["verdict"][0] == -1 and r["reason"][0] == 2


def test_version_order_decision_matches_search():
    """The GPU fast tier's decision procedure (restated in fastpath_ref.py)
    agrees with the searches on every key it decides."""
    import fastpath_ref
    keys = tiny_batch(4242, 3000, max_ops=8)
    sets = [keys]
    for (nk, n, conc, pi, pa, seed) in [(200, 200, 10, 0, 0.5, 1), (100, 300, 20, 0.02, 0.5, 2)]:
        ops, off, _, _ = abi.synth(nk, n, concurrency=conc, p_info=pi, p_anomaly=pa, seed=seed)
        sets.append([ops[off[k]:off[k + 1]].tolist() for k in range(nk)])
    decided = 0
    for ks in sets:
        ops, off = pack_keys(ks)
        _, j = oracle.check(ops, off, algo=oracle.JITC, n_threads=4)
        for i, recs in enumerate(ks):
            d = fastpath_ref.decide([tuple(r) for r in recs])
            if d is None:
                continue
            decided += 1
            assert d == j["verdict"][i], recs
    assert decided > 2000
    for k in KATS:
        d = fastpath_ref.decide([tuple(r) for r in k["ops"]])
        assert d is None or d == (1 if k["valid"] else 0), k["name"]


def test_first_failure_rule_matches_search():
    """The GPU's O(n) first-failure rule (restated in fastpath_ref.py) names
    the same fail op as knossos.linear's frontier on every invalid key it
    decides, and its prefix witness certifies; where two mutations claim one
    version it either decides exactly or declines.  Random tiny keys,
    synthetic keys with injected stale reads / lost CAS (C5's shapes) at
    several concurrencies, and the same keys with versions duplicated."""
    import fastpath_ref
    sets = [tiny_batch(777, 3000, max_ops=8)]
    for (nk, n, conc, pa, seed) in [(300, 120, 6, 1.0, 11), (300, 200, 10, 1.0, 12),
                                    (200, 300, 20, 1.0, 13), (200, 200, 10, 0.3, 14)]:
        ops, off, _, _ = abi.synth(nk, n, concurrency=conc, p_anomaly=pa, seed=seed)
        sets.append([ops[off[k]:off[k + 1]].tolist() for k in range(nk)])
    sets.append(dup_versions(sets[1], 21))
    sets.append(dup_versions(sets[2] + sets[3], 22, frac=1.0))
    decided = declined = 0
    for ks in sets:
        ops, off = pack_keys(ks)
        _, j = oracle.check(ops, off, algo=oracle.JITC, n_threads=4)
        wit = np.full(len(ops), -1, dtype=np.int32)
        kind = np.zeros(len(ks), dtype=np.int32)
        res = np.zeros(len(ks), dtype=oracle.RESULT_DTYPE)
        res["fail_prefix_end"] = 0
        for i, recs in enumerate(ks):
            t = [tuple(r) for r in recs]
            if fastpath_ref.decide(t) != 0:
                continue
            ff = fastpath_ref.first_failure(t)
            if ff is None:
                declined += 1
                continue
            decided += 1
            assert j["verdict"][i] == 0 and ff[0] == j["fail_op"][i], (recs, ff, j["fail_op"][i])
            wit[off[i]:off[i + 1]] = ff[1]
            kind[i] = 2
            res["fail_prefix_end"][i] = recs[ff[0]][5]
        st, _ = oracle.check_witness(ops, off, wit, kind, results=res)
        assert (st[kind == 2] == oracle.WIT_OK).all()
    assert decided > 1500 and declined < decided // 10, (decided, declined)


@pytest.mark.parametrize("conc,seed", [(6, 3), (10, 5), (14, 8)])
def test_deadline_order_exact_version_less(conc, seed):
    """DEADLINE_ORDER matters where equal writes/CAS are common: version-less
    keys (the cas-register model).  Verdict and canonical fail op equal the
    faithful search on every key both decide, with fewer configurations."""
    ops, off, _, _ = abi.synth(80, 120, concurrency=conc, p_info=0.03, p_anomaly=0.0, seed=seed)
    ops = ops.copy()
    ops[:, 3] = -1
    rng = np.random.default_rng(seed)  # a few reads of a value nothing wrote
    reads = np.nonzero((ops[:, 0] == 0) & (ops[:, 5] != INF))[0]
    ops[rng.choice(reads, 12, replace=False), 1] = 999
    _, j = oracle.check(ops, off, algo=oracle.JIT, n_threads=4, max_configs=400000)
    _, d = oracle.check(ops, off, algo=oracle.JIT | oracle.DEADLINE_ORDER, n_threads=4,
                        max_configs=400000)
    known = (j["verdict"] != -1) & (d["verdict"] != -1)
    assert known.mean() > 0.8 and (j["verdict"][known] == 0).any()
    assert (j["verdict"][known] == d["verdict"][known]).all()
    assert (j["fail_op"][known] == d["fail_op"][known]).all()
    assert d["configs_explored"][known].sum() < j["configs_explored"][known].sum()
