"""Other knossos models: cas-register, register and
mutex (the lock workload's model, lock.clj:243-244) as packings of the same
records (history.py "Models").  The oracle's three analyzers must agree on
them, the packers (Python and EDN) must agree with each other, and the GPU
must agree with the oracle."""
import random

import numpy as np
import pytest

import oracle
from helpers import FREE, HELD, INF, pack_keys, random_casreg, random_mutex
from jepsen.etcd_amd import abi, checker, edn, history as H
from jepsen.etcd_amd.history import Tuple
from oracle import brute


def ops_of(seq):
    """Sequential mini-histories: [(process, f, invoke value, completion type,
    completion value)] in order, each completion right after its invoke
    unless it is None (pending)."""
    h = []
    for p, f, v, t, cv in seq:
        h.append({"type": "invoke", "f": f, "process": p, "value": v})
        if t is not None:
            h.append({"type": t, "f": f, "process": p, "value": cv})
    return h


MUTEX_KATS = [
    ("acq-rel-acq", [(0, "acquire", None, "ok", None), (0, "release", None, "ok", None),
                     (1, "acquire", None, "ok", None)], True),
    ("double-acquire", [(0, "acquire", None, "ok", None), (1, "acquire", None, "ok", None)], False),
    ("release-free", [(0, "release", None, "ok", None)], False),
    ("crashed-acquire-may-not-happen", [(0, "acquire", None, "info", None),
                                       (1, "acquire", None, "ok", None)], True),
    ("crashed-acquire-then-release", [(0, "acquire", None, "info", None),
                                     (1, "release", None, "ok", None),
                                     (2, "acquire", None, "ok", None)], True),
    ("failed-acquire-ignored", [(0, "acquire", None, "ok", None), (1, "acquire", None, "fail", None),
                               (0, "release", None, "ok", None)], True),
]


@pytest.mark.parametrize("name,seq,valid", MUTEX_KATS)
def test_mutex_kats_oracle(name, seq, valid):
    keys, ops, off, _ = H.pack(ops_of(seq), model="mutex", independent=False)
    assert keys == [None]
    for algo in (oracle.JIT, oracle.WGL):
        _, r = oracle.check(ops, off, algo=algo, init_value=FREE)
        assert r["verdict"][0] == (1 if valid else 0), (name, algo)
    assert brute.check(ops.tolist(), init=(0, FREE)) == valid


def test_mutex_packing():
    h = ops_of([(0, "acquire", None, "ok", None), (0, "release", None, "ok", None),
                (1, "frob", None, "ok", None)])
    _, ops, _, _ = H.pack(h, model="mutex", independent=False)
    assert ops.tolist() == [[2, HELD, FREE, -1, 0, 1], [2, FREE, HELD, -1, 2, 3],
                            [3, -1, -1, -1, 4, 5]]


def test_cas_register_and_register_packing():
    h = ops_of([(0, "write", 1, "ok", 1), (1, "cas", [1, 2], "ok", [1, 2]),
                (2, "read", None, "ok", 2), (3, "read", None, "ok", None)])
    _, ops, _, _ = H.pack(h, model="cas-register", independent=False)
    assert ops.tolist() == [[1, 0, -1, -1, 0, 1], [2, 1, 0, -1, 2, 3], [0, 1, -1, -1, 4, 5],
                            [0, -1, -1, -1, 6, 7]]
    _, ops, _, _ = H.pack(h, model="register", independent=False)
    assert ops[1, 0] == H.F_UNKNOWN
    # a non-nil initial value is id 0 of every key
    _, ops, _, _ = H.pack(h, model="cas-register", independent=False, init_value=1)
    assert ops[0].tolist()[:2] == [1, 0]


@pytest.mark.parametrize("model,gen,init", [("mutex", random_mutex, FREE),
                                            ("cas-register", random_casreg, -1)])
def test_three_analyzers_agree(model, gen, init):
    rng = random.Random(11)
    keys = [gen(rng, rng.randrange(0, 8)) for _ in range(600)]
    ops, off = pack_keys(keys)
    _, a = oracle.check(ops, off, algo=oracle.JIT, init_value=init)
    _, b = oracle.check(ops, off, algo=oracle.WGL, init_value=init)
    assert (a["verdict"] == b["verdict"]).all()
    for k, recs in enumerate(keys):
        assert brute.check(recs, init=(0, init)) == (a["verdict"][k] == 1)
    assert 0.03 < (a["verdict"] == 0).mean() < 0.9  # both verdicts well represented


def _as_history(model, recs, key=None):
    """Records back to op dicts (for the packers' agreement test)."""
    ev = []
    for i, (f, v, e, ver, call, ret) in enumerate(recs):
        if model == "mutex":
            fk, iv = ("acquire" if v == HELD else "release"), None
        else:
            fk = {0: "read", 1: "write", 2: "cas"}[f]
            val = None if v == -1 else v
            iv = [None if e == -1 else e, val] if f == 2 else (None if f == 0 else val)
        wrap = (lambda x: Tuple(key, x)) if key is not None else (lambda x: x)
        ev.append((call, {"type": "invoke", "f": fk, "process": i, "value": wrap(iv)}))
        if ret != INF:
            ev.append((ret, {"type": "ok", "f": fk, "process": i, "value": wrap(iv)}))
    ev.sort(key=lambda t: t[0])
    return [op for _, op in ev]


@pytest.mark.parametrize("model", ["mutex", "cas-register", "register"])
def test_edn_reader_matches_pack_for_models(model):
    rng = random.Random(5)
    gen = random_mutex if model == "mutex" else random_casreg
    hist = []
    for k in range(20):
        hist += _as_history(model, gen(rng, 12), key=k)
    keys, ops, off, _ = H.pack(hist, model=model)
    h = edn.read(edn.to_edn(hist), model=model)
    assert (h.ops == ops).all() and (h.key_off == off).all()
    one = _as_history(model, gen(rng, 30))
    single = edn.read(edn.to_edn(one), independent=False, model=model)
    _, ops1, off1, _ = H.pack(one, model=model, independent=False)
    assert single.n_keys == 1 and (single.ops == ops1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("model,gen,init", [("mutex", random_mutex, FREE),
                                            ("cas-register", random_casreg, -1)])
def test_models_gpu_vs_oracle(ctx, model, gen, init):
    rng = random.Random(99)
    keys = [gen(rng, rng.randrange(0, 60)) for _ in range(3000)]
    ops, off = pack_keys(keys)
    o = abi.default_opts(init_value=init)
    _, g = ctx.check(ops, off, opts=o)
    _, r = oracle.check(ops, off, algo=oracle.JIT, init_value=init, max_configs=2_000_000)
    known = r["verdict"] != -1
    assert known.mean() > 0.99
    assert (g["verdict"][known] == r["verdict"][known]).all()
    assert (g["fail_op"][known] == r["fail_op"][known]).all()


@pytest.mark.gpu
def test_lock_workload_checker_gpu():
    """checker/linearizable {:model (model/mutex)} over one lock history
    (lock.clj:243-244), through the checker mirror."""
    for name, seq, valid in MUTEX_KATS:
        res = checker.linearizable(checker.Mutex(), device_mask=1).check({}, ops_of(seq))
        assert res["valid?"] is valid, name
