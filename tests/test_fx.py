"""Frontier exchange (include/lincheck_fx.h): one key's JIT search over the
whole GPU, partitioned over ranks by hash ownership.

The oracle's JITC mode (oracle.c check_key_jit with the GPU's exact
reductions) runs the same search serially, so every field of every decided
key must match it exactly: verdict, canonical fail op, configurations
explored and largest frontier.  Forcing the partitioned mode
(part_above=0) on small keys runs every level through the all-to-all-v
exchange; a middle threshold switches between the replicated and the
partitioned frontier back and forth.  The multi-process test drives the
engine through torch.distributed (gloo, two ranks sharing the card) — the
transport an 8-GPU node uses under RCCL."""
import os
import random
import socket

import numpy as np
import pytest

import oracle
from helpers import FREE, pack_keys, random_casreg, random_mutex, random_tiny
from jepsen.etcd_amd import abi

FIELDS = ("verdict", "reason", "fail_op", "fail_prefix_end", "configs_explored", "max_frontier")


def _keys(seed, n_each=60):
    """(records, init_value) per key: cas-register, mutex and register keys,
    tiny to mid-sized, crashes and anomalies included."""
    rng = random.Random(seed)
    keys = []
    for _ in range(n_each):
        keys.append((random_casreg(rng, rng.randrange(1, 60), p_info=0.1), -1))
        keys.append((random_mutex(rng, rng.randrange(1, 60), p_info=0.1), FREE))
        keys.append((random_tiny(rng, rng.randrange(1, 30)), -1))
    # synthetic version-less keys with real frontiers (concurrency 8-12)
    for i, conc in enumerate((8, 10, 12)):
        ops, off, _, _ = abi.synth(4, 300, concurrency=conc, p_info=0.01, p_anomaly=0.5,
                                   seed=seed * 7 + i)
        ops = ops.copy()
        ops[:, 3] = -1
        for k in range(4):
            keys.append((ops[off[k]:off[k + 1]].tolist(), -1))
    return keys


def _oracle(recs, init_value):
    ops, off = pack_keys([recs])
    _, r = oracle.check(ops, off, algo=oracle.JITC, init_value=init_value)
    return r[0]


def _compare(got, want, tag):
    if want["reason"] == abi.LC_REASON_CONFIG_BUDGET:
        return  # the oracle's own budget; not a parity case
    for f in FIELDS:
        assert int(got[f]) == int(want[f]), (tag, f, int(got[f]), int(want[f]))


@pytest.mark.gpu
@pytest.mark.parametrize("ranks,part_above", [(1, -1), (3, 0), (2, 6), (4, 0)])
def test_fx_matches_oracle_jitc(ranks, part_above):
    from jepsen.etcd_amd.fx import FrontierExchange
    keys = _keys(0xF00 + ranks * 10 + max(part_above, 0))
    with FrontierExchange(device=0, virtual_ranks=ranks, part_above=part_above,
                          table_log2=18) as fx:
        for i, (recs, init) in enumerate(keys):
            want = _oracle(recs, init)
            got = fx.check(np.array(recs, dtype=np.int64).reshape(-1, 6),
                           abi.default_opts(init_value=init))
            _compare(got, want, (ranks, part_above, i))
        st = fx.stats()
    if ranks > 1 and part_above == 0:
        assert st["part_returns"] > 0


@pytest.mark.gpu
def test_fx_incremental_retirement_and(monkeypatch, capfd):
    """The retirement AND is kept incrementally (each workgroup of the insert
    and of every level ANDs the masks it puts into R; no pass over R).  Under
    LC_FX_DEBUG the engine recomputes the AND of R whole after every
    replicated return and fails the check on any difference.  Version-less
    keys whose returns start in the one-workgroup small-return kernel and
    continue on the grid (kcur hand-off) across several batches, no counted
    classes: every return checked, every result field equal to the oracle's
    JITC."""
    from jepsen.etcd_amd.fx import FrontierExchange
    monkeypatch.setenv("LC_FX_DEBUG", "1")
    monkeypatch.setenv("LC_FX_CLASSES", "0")
    with FrontierExchange(device=0) as fx:
        for n, conc, seed in ((700, 40, 81), (900, 40, 83), (1200, 36, 84)):
            ops, off, _, _ = abi.synth(1, n, concurrency=conc, p_anomaly=0.0, seed=seed)
            ops = ops.copy()
            ops[:, 3] = -1
            got = fx.check(ops)
            _compare(got, _oracle(ops.tolist(), -1), (n, conc))
            assert int(got["max_frontier"]) > 1024  # levels beyond the small kernel's cutoff
    err = capfd.readouterr().err
    assert err.count("fx and-check ok") > 500 and "LC_FX_DEBUG: incremental" not in err


@pytest.mark.gpu
@pytest.mark.parametrize("transport", ["rccl", "hub"])
def test_fx_self_exchange_matches_oracle(transport):
    """The multi-rank protocol with one rank exchanging with itself
    (LC_FX_FLAG_EXCHANGE_SELF, every level partitioned): under "rccl" every
    configuration moves through the library's own RCCL transport — a
    one-device communicator from ncclCommInitAll, counts by ncclAllToAll on
    the device, payload by grouped ncclSend / ncclRecv — which is the path
    LC_FLAG_WHOLE_GPU takes over several GPUs (this pool has one GPU per box
    and RCCL refuses two ranks on one device).  Every field equals JITC's."""
    from jepsen.etcd_amd.fx import LC_FX_FLAG_EXCHANGE_SELF, FrontierExchange
    keys = _keys(0xF0E, n_each=25)
    kw = dict(rccl_devices=[0]) if transport == "rccl" else dict(virtual_ranks=1)
    sent = 0
    with FrontierExchange(device=0, part_above=0, table_log2=18,
                          flags=LC_FX_FLAG_EXCHANGE_SELF, **kw) as fx:
        for i, (recs, init) in enumerate(keys):
            got = fx.check(np.array(recs, dtype=np.int64).reshape(-1, 6),
                           abi.default_opts(init_value=init))
            _compare(got, _oracle(recs, init), (transport, i))
            st = fx.stats()
            sent += st["sent_configs"]
            if len(recs) > 20 and got["verdict"] != -1:
                assert st["part_returns"] > 0, (i, st)
    assert sent > 1000


@pytest.mark.gpu
def test_fx_rccl_one_rank_plain():
    """A one-device RCCL engine without self-exchange: the single-rank path
    (no collective runs), same results as the in-process engine."""
    from jepsen.etcd_amd.fx import FrontierExchange
    ops, off, _, _ = abi.synth(1, 600, concurrency=14, p_info=0.005, seed=0xFACE)
    ops = ops.copy()
    ops[:, 3] = -1
    with FrontierExchange(device=0, rccl_devices=[0]) as fx:
        got = fx.check(ops)
    _compare(got, _oracle(ops.tolist(), -1), "rccl one rank")


@pytest.mark.gpu
def test_fx_frontier_is_the_oracles_frontier():
    """knossos's :configs for keys only the frontier search decides: the
    frontier just before the failing return (lc_fx_frontier) is exactly the
    oracle's JITC frontier at that return — each configuration's state and
    pending ops, built there by replaying oracle_step — and a truncated copy
    (knossos keeps 10) is a subset of it."""
    from jepsen.etcd_amd.fx import FrontierExchange
    rng = random.Random(0xC0F)
    keys = [(random_casreg(rng, rng.randrange(4, 40), p_info=0.1), -1) for _ in range(150)]
    keys += [(random_mutex(rng, rng.randrange(4, 40), p_info=0.1), FREE) for _ in range(100)]
    ops, off, _, _ = abi.synth(12, 150, concurrency=8, p_info=0.01, p_anomaly=1.0, seed=0xC10)
    ops = ops.copy()
    ops[:, 3] = -1
    keys += [(ops[off[k]:off[k + 1]].tolist(), -1) for k in range(12)]
    n_inv = n_cfg = 0
    with FrontierExchange(device=0) as fx:
        for i, (recs, init) in enumerate(keys):
            a = np.array(recs, dtype=np.int64).reshape(-1, 6)
            o = abi.default_opts(init_value=init)
            r = fx.check(a, o)
            if r["verdict"] != 0:
                continue
            fo = int(r["fail_op"])
            want, n_want = oracle.frontier(a, fo, init_value=init)
            got = fx.frontier(a, fo, max_configs=1 << 16, opts=o)
            assert set(got) == want and len(got) == n_want, (i, len(got), n_want)
            top = fx.frontier(a, fo, max_configs=10, opts=o)
            assert len(top) == min(10, n_want) and set(top) <= want, i
            n_inv += 1
            n_cfg += len(got)
    assert n_inv >= 20 and n_cfg > n_inv


def _crash_heavy_mutex_keys(seed, n=24):
    """The lock workload's model (lock.clj:244) under a partition: long keys
    whose crashed acquires / releases pile up — 140 to 300 of them never
    complete, far more than LC_MAX_WINDOW open at once."""
    rng = random.Random(seed)
    return [random_mutex(rng, rng.randrange(200, 800), p_info=0.4, p_perturb=0.5)
            for _ in range(n)]


@pytest.mark.gpu
def test_fx_counted_classes_decide_crash_heavy_keys(monkeypatch):
    """Counted classes (fx.hip): a key's crashed writes/CAS of one class
    (f, value, expected, version) are a count in the configuration, not one
    window slot each.  Keys with 65-300 outstanding crashed ops, which one
    slot per op turns :unknown (LC_REASON_WINDOW_OVERFLOW), are decided and
    equal the oracle's JITC in every field (its window is unbounded) and
    WGL's verdicts.  (Every key with a crashed write/CAS takes the counted
    classes, so the oracle comparisons of test_fx_matches_oracle_jitc and
    test_fx_frontier_is_the_oracles_frontier, whose keys carry crashes and
    anomalies, cover their frontiers and counterexamples.)"""
    from jepsen.etcd_amd.fx import FrontierExchange
    keys = _crash_heavy_mutex_keys(0xC1A55)
    ops, off = pack_keys(keys)
    _, j = oracle.check(ops, off, algo=oracle.JITC, init_value=FREE, n_threads=8)
    _, g = oracle.check(ops, off, algo=oracle.WGL, init_value=FREE, n_threads=8)
    assert (j["verdict"] != -1).all() and (j["verdict"] == g["verdict"]).all()
    outstanding = [sum(1 for r in k if r[5] == abi.LC_INF) for k in keys]
    assert min(outstanding) > 64
    o = abi.default_opts(init_value=FREE)
    with FrontierExchange(device=0) as fx:
        for i, k in enumerate(keys):
            got = fx.check(np.array(k, dtype=np.int64), o)
            for f in FIELDS:
                assert int(got[f]) == int(j[f][i]), (i, f, int(got[f]), int(j[f][i]))
        # one slot per crashed op: the window overflows
        monkeypatch.setenv("LC_FX_CLASSES", "0")
        over = sum(int(fx.check(np.array(k, dtype=np.int64), o)["reason"] ==
                       abi.LC_REASON_WINDOW_OVERFLOW) for k in keys)
    assert over >= len(keys) // 2


@pytest.mark.gpu
@pytest.mark.parametrize("ranks,part_above", [(2, 0), (3, 0), (2, 1)])
def test_fx_counted_classes_over_ranks(ranks, part_above):
    """Counted classes on the multi-rank engine: a configuration's owner
    hashes each class by its absolute count (members retired + its field),
    which retirement leaves unchanged, and a class's retirement takes the
    smallest field over every rank's R.  Crash-heavy mutex keys (frontiers
    of a few configurations), every level partitioned (part_above=0) or
    only returns above one configuration: every field equals the oracle's
    JITC, with configurations exchanged when every level is partitioned."""
    from jepsen.etcd_amd.fx import FrontierExchange
    keys = _crash_heavy_mutex_keys(0xC1A57 + ranks, n=8)
    ops, off = pack_keys(keys)
    _, j = oracle.check(ops, off, algo=oracle.JITC, init_value=FREE, n_threads=8)
    assert (j["verdict"] != -1).all()
    o = abi.default_opts(init_value=FREE)
    sent = part = 0
    with FrontierExchange(device=0, virtual_ranks=ranks, part_above=part_above,
                          repl_below=part_above // 2, table_log2=18) as fx:
        for i, k in enumerate(keys):
            got = fx.check(np.array(k, dtype=np.int64), o)
            for f in FIELDS:
                assert int(got[f]) == int(j[f][i]), (ranks, part_above, i, f, int(got[f]), int(j[f][i]))
            st = fx.stats()
            sent += st["sent_configs"]
            part += st["part_returns"]
    if part_above == 0:
        assert part > 0 and sent > 0


@pytest.mark.gpu
def test_whole_gpu_spreads_window_overflow_keys(monkeypatch, capfd):
    """Fewer window-overflow keys than the context has devices: each one's
    re-search spans every device (two device contexts on this box's GPU,
    LC_VIRTUAL_DEVICES=2, run their two ranks in process; LC_FX_DEBUG names
    the rank of every return), counted classes included, and the results
    equal the oracle's JITC in every field."""
    monkeypatch.setenv("LC_VIRTUAL_DEVICES", "2")
    keys = _crash_heavy_mutex_keys(0xC1A58, n=6)
    ops, off = pack_keys(keys)
    with abi.Context(1) as ctx:
        _, plain = ctx.check(ops, off, abi.default_opts(init_value=FREE))
        over = np.flatnonzero(plain["reason"] == abi.LC_REASON_WINDOW_OVERFLOW)
        assert len(over) >= 1
        one = over[:1]  # one key: fewer than the two devices
        sops, soff = pack_keys([keys[int(one[0])]])
        monkeypatch.setenv("LC_FX_DEBUG", "1")
        _, whole = ctx.check(sops, soff, abi.default_opts(init_value=FREE,
                                                          flags=abi.LC_FLAG_WHOLE_GPU))
        assert ctx.stats()["n_devices"] == 2
    err = capfd.readouterr().err
    assert "fx r1 ret" in err and "fx r0 ret" in err
    _, j = oracle.check(sops, soff, algo=oracle.JITC, init_value=FREE)
    for f in FIELDS:
        assert (whole[f] == j[f]).all(), f
    assert whole["verdict"][0] != -1


@pytest.mark.gpu
def test_whole_gpu_decides_window_overflow_keys():
    """lc_check's search tiers keep one window slot per open op
    (LC_MAX_WINDOW = 64): crash-heavy version-less keys come back :unknown
    with reason window-overflow.  LC_FLAG_WHOLE_GPU searches them again on
    one-rank frontier-exchange engines, which count crashed ops per class:
    every key is decided, equal to the oracle's JITC."""
    keys = _crash_heavy_mutex_keys(0xC1A56, n=12)
    ops, off = pack_keys(keys)
    with abi.Context(1) as ctx:
        _, plain = ctx.check(ops, off, abi.default_opts(init_value=FREE))
        _, whole = ctx.check(ops, off, abi.default_opts(init_value=FREE,
                                                        flags=abi.LC_FLAG_WHOLE_GPU))
    assert (plain["reason"] == abi.LC_REASON_WINDOW_OVERFLOW).sum() >= 6
    _, j = oracle.check(ops, off, algo=oracle.JITC, init_value=FREE, n_threads=8)
    for f in FIELDS:
        assert (whole[f] == j[f]).all(), f


@pytest.mark.gpu
def test_fx_partition_switches_and_exchanges():
    """A key whose frontier crosses the thresholds both ways: replicated ->
    partitioned (filter by owner) -> replicated (gather), same result as one
    rank, with configurations actually sent between ranks."""
    from jepsen.etcd_amd.fx import FrontierExchange
    ops, off, _, _ = abi.synth(1, 600, concurrency=14, p_info=0.005, seed=0xFACE)
    ops = ops.copy()
    ops[:, 3] = -1
    with FrontierExchange(device=0, virtual_ranks=1) as fx:
        one = fx.check(ops)
    want = _oracle(ops.tolist(), -1)
    _compare(one, want, "one rank")
    assert one["max_frontier"] > 40
    with FrontierExchange(device=0, virtual_ranks=3, part_above=30, repl_below=10,
                          table_log2=18) as fx:
        got = fx.check(ops)
        st = fx.stats()
    _compare(got, want, "three ranks")
    assert st["part_returns"] > 0 and st["gathers"] > 0 and st["sent_configs"] > 0


@pytest.mark.gpu
def test_fx_full_size_ranks_and_tiers_agree():
    """Full-size keys the oracle takes seconds on: one rank, three in-process
    ranks partitioned above a few thousand configurations, and (where they decide)
    lc_check's tiers give the same verdict, configurations explored and
    largest frontier — an order-independent count of a 10^7-configuration
    search, so agreement pins the whole set semantics."""
    from jepsen.etcd_amd.fx import FrontierExchange
    for conc, info, n, pa in ((28, 0.002, 1000, 600), (40, 0.0, 2000, 4096)):
        ops, off, _, _ = abi.synth(1, n, concurrency=conc, p_info=info, seed=0x5EED0004)
        ops = ops.copy()
        ops[:, 3] = -1
        with FrontierExchange(device=0) as fx:
            one = fx.check(ops)
        with FrontierExchange(device=0, virtual_ranks=3, part_above=pa, repl_below=pa // 4) as fx:
            three = fx.check(ops)
            st = fx.stats()
        assert st["part_returns"] > 0 and st["gathers"] > 0
        for f in FIELDS:
            assert int(one[f]) == int(three[f]), (conc, f)
        assert one["verdict"] == 1
        with abi.Context(1) as ctx:
            _, t = ctx.check(ops, off)
        if t["verdict"][0] == 1:
            assert int(t["configs_explored"][0]) == int(one["configs_explored"])
            assert int(t["max_frontier"][0]) == int(one["max_frontier"])


@pytest.mark.gpu
@pytest.mark.parametrize("ranks", [1, 2])
def test_fx_wide_tables(ranks):
    """Keys with many distinct values still pack (mask, value id) into one
    word (fewer mask bits, more value bits); the 16-byte-key tables (epoch
    tags, fenced publication) serve what does not fit and, forced, every key:
    both give the oracle's results."""
    from jepsen.etcd_amd.fx import LC_FX_FLAG_WIDE_TABLES, FrontierExchange
    ops, off, _, _ = abi.synth(3, 300, concurrency=10, n_values=400, p_info=0.01,
                               p_anomaly=0.5, seed=0x71DE + ranks)
    ops = ops.copy()
    ops[:, 3] = -1
    keys = [ops[off[k]:off[k + 1]] for k in range(3)]
    small = abi.synth(1, 200, concurrency=8, seed=0x71DF)[0].copy()
    small[:, 3] = -1
    for flags in (0, LC_FX_FLAG_WIDE_TABLES):
        with FrontierExchange(device=0, virtual_ranks=ranks, part_above=0 if ranks > 1 else -1,
                              table_log2=18, flags=flags) as fx:
            for k in keys + [small, keys[0]]:
                got = fx.check(k)
                _compare(got, _oracle(k.tolist(), -1), ("wide", ranks, flags))
                wide = fx.stats()["wide_returns"]
                assert (wide > 0) if flags else (wide == 0), (flags, wide)


@pytest.mark.gpu
def test_fx_small_tables_redo_and_decide(monkeypatch):
    """Table prefixes sized to the expected work itself (LC_FX_TABLE_MUL=1,
    a dev knob; the default is 4x) and full tables only 4x the largest
    frontier: returns outgrow their prefix, are redone with a 4x larger one
    up to the full table, and the key is still decided — partitioned over
    two in-process ranks and replicated over two (where the ranks must agree
    on a redo, since probe-chain lengths follow the order of atomic inserts)
    — with the results of a default run."""
    from jepsen.etcd_amd.fx import FrontierExchange
    ops, off, _, _ = abi.synth(1, 2000, concurrency=40, seed=0x5EED0004)
    ops = ops.copy()
    ops[:, 3] = -1
    with FrontierExchange(device=0) as fx:
        want = fx.check(ops)
    assert want["verdict"] == 1
    full = 1
    while (1 << full) < 4 * int(want["max_frontier"]):
        full += 1
    monkeypatch.setenv("LC_FX_TABLE_MUL", "1")
    redos = 0
    for ranks, pa in ((2, 0), (2, 1 << 30), (1, -1)):
        for lg in (full, full + 1):
            with FrontierExchange(device=0, virtual_ranks=ranks, part_above=pa,
                                  table_log2=lg) as fx:
                got = fx.check(ops)
                redos += fx.stats()["redos"]
            for f in FIELDS:
                assert int(got[f]) == int(want[f]), (ranks, pa, lg, f)
    assert redos > 0


@pytest.mark.gpu
def test_fx_budget_window_and_errors():
    from jepsen.etcd_amd.fx import FrontierExchange
    ops, off, _, _ = abi.synth(1, 400, concurrency=16, p_info=0.02, seed=0xB0B)
    ops = ops.copy()
    ops[:, 3] = -1
    with FrontierExchange(device=0, virtual_ranks=2, part_above=0, table_log2=16) as fx:
        r = fx.check(ops, abi.default_opts(max_configs_per_key=50))
        assert r["verdict"] == -1 and r["reason"] == abi.LC_REASON_CONFIG_BUDGET
        # 70 writes open at once: more than LC_MAX_WINDOW slots
        recs = [[1, i % 3, -1, -1, i, 1000 + i] for i in range(70)]
        r = fx.check(np.array(recs, dtype=np.int64))
        assert r["verdict"] == -1 and r["reason"] == abi.LC_REASON_WINDOW_OVERFLOW
        bad = np.array([[1, 0, -1, -1, 5, 3]], dtype=np.int64)  # ret < call
        assert fx.check(bad)["reason"] == abi.LC_REASON_MALFORMED
        unk = np.array([[7, 0, -1, -1, 0, 1]], dtype=np.int64)
        assert fx.check(unk)["reason"] == abi.LC_REASON_UNKNOWN_F
        empty = fx.check(np.zeros((0, 6), dtype=np.int64))
        assert empty["verdict"] == 1
    # the time budget: every rank agrees the key is :unknown (reason 7)
    big, _, _, _ = abi.synth(1, 2000, concurrency=40, seed=0x5EED0004)
    big = big.copy()
    big[:, 3] = -1
    for ranks in (1, 2):
        with FrontierExchange(device=0, virtual_ranks=ranks, part_above=0 if ranks > 1 else -1) as fx:
            r = fx.check(big, abi.default_opts(time_budget_ms=5))
            assert r["verdict"] == -1 and r["reason"] == 7, (ranks, r)


@pytest.mark.gpu
def test_whole_gpu_flag_decides_budget_keys():
    """LC_FLAG_WHOLE_GPU: keys the tiers leave :unknown at the configuration
    budget (cumulative over one workgroup's search) are decided by the
    frontier exchange, whose budget bounds each return's sets as the
    oracle's does; keys the tiers decide are untouched."""
    ops, off, _, _ = abi.synth(3, 1000, concurrency=28, p_info=0.002, seed=0xB16)
    ops = ops.copy()
    ops[:, 3] = -1
    small, soff, _, _ = abi.synth(2, 200, concurrency=6, seed=0xB17)
    small = small.copy()
    small[:, 3] = -1
    allops = np.concatenate([ops, small])
    alloff = np.concatenate([off, soff[1:] + off[-1]])
    budget = 100000
    with abi.Context(1) as ctx:
        _, plain = ctx.check(allops, alloff, abi.default_opts(max_configs_per_key=budget))
        _, whole = ctx.check(allops, alloff, abi.default_opts(max_configs_per_key=budget,
                                                              flags=abi.LC_FLAG_WHOLE_GPU))
    assert (plain["reason"][:3] == abi.LC_REASON_CONFIG_BUDGET).all()
    _, ref = oracle.check(allops, alloff, algo=oracle.JITC, max_configs=budget)
    for k in range(len(alloff) - 1):
        for f in FIELDS:
            assert int(whole[f][k]) == int(ref[f][k]), (k, f)
    assert (whole["verdict"][:3] == 1).all()
    assert (whole[3:] == plain[3:]).all()
    # the device entry point: records, offsets and results in device memory
    # (a slice of the batch: d_ops starts at the record key_off[1] names)
    import torch
    dev = torch.device("cuda:0")
    d_ops = torch.from_numpy(allops[alloff[1]:]).to(dev)
    d_off = torch.from_numpy(alloff[1:].copy()).to(dev)
    n = len(alloff) - 2
    d_out = torch.zeros(n * abi.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    with abi.Context(1) as ctx:
        ctx.check_device(d_ops.data_ptr(), d_off.data_ptr(), n, d_out.data_ptr(),
                         opts=abi.default_opts(max_configs_per_key=budget,
                                               flags=abi.LC_FLAG_WHOLE_GPU))
    torch.cuda.synchronize()
    got = np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)
    for f in FIELDS:
        assert (got[f] == whole[f][1:]).all(), f


@pytest.mark.gpu
def test_whole_gpu_key_spans_every_device_of_the_context(monkeypatch):
    """LC_FLAG_WHOLE_GPU with fewer budget keys than the context has GPUs:
    each key's search spans all of them (one rank per GPU, the frontier
    partitioned by owner above part_above).  Two device contexts on this
    box's one GPU (LC_VIRTUAL_DEVICES) run their ranks in process; results
    equal the oracle's in every field, and keys the tiers decide keep
    their results."""
    monkeypatch.setenv("LC_VIRTUAL_DEVICES", "2")
    ops, off, _, _ = abi.synth(1, 1000, concurrency=28, p_info=0.002, seed=0xB16)
    ops = ops.copy()
    ops[:, 3] = -1
    small, soff, _, _ = abi.synth(3, 200, concurrency=6, seed=0xB17)
    small = small.copy()
    small[:, 3] = -1
    allops = np.concatenate([ops, small])
    alloff = np.concatenate([off, soff[1:] + off[-1]])
    budget = 100000
    with abi.Context(1) as ctx:
        _, plain = ctx.check(allops, alloff, abi.default_opts(max_configs_per_key=budget))
        _, whole = ctx.check(allops, alloff, abi.default_opts(max_configs_per_key=budget,
                                                              flags=abi.LC_FLAG_WHOLE_GPU))
        assert ctx.stats()["n_devices"] == 2
    assert plain["reason"][0] == abi.LC_REASON_CONFIG_BUDGET
    _, ref = oracle.check(allops, alloff, algo=oracle.JITC, max_configs=budget)
    for k in range(len(alloff) - 1):
        for f in FIELDS:
            assert int(whole[f][k]) == int(ref[f][k]), (k, f)
    assert whole["verdict"][0] == 1
    assert (whole[1:] == plain[1:]).all()


@pytest.mark.gpu
def test_whole_gpu_failed_research_keeps_key_unknown(monkeypatch):
    """A re-search that cannot run costs only its key: it stays :unknown at
    the budget, every other key is decided, the call returns 0 and
    lc_last_error says why.  LC_FX_FAIL_RESERVE=1 (a test hook) makes the
    engine's list allocation fail, as an over-large budget would."""
    monkeypatch.setenv("LC_FX_FAIL_RESERVE", "1")
    ops, off, _, _ = abi.synth(1, 1000, concurrency=28, p_info=0.002, seed=0xB16)
    ops = ops.copy()
    ops[:, 3] = -1
    small, soff, _, _ = abi.synth(2, 200, concurrency=6, seed=0xB17)
    allops = np.concatenate([ops, small])
    alloff = np.concatenate([off, soff[1:] + off[-1]])
    opts = abi.default_opts(max_configs_per_key=100000, flags=abi.LC_FLAG_WHOLE_GPU)
    with abi.Context(1) as ctx:
        _, r = ctx.check(allops, alloff, opts)
        err = ctx.last_error()
    assert r["verdict"][0] == -1 and r["reason"][0] == abi.LC_REASON_CONFIG_BUDGET
    assert (r["verdict"][1:] == 1).all()
    assert "kept :unknown" in err and "injected" in err, err


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, keys, q):
    import torch.distributed as dist
    from jepsen.etcd_amd.fx import FrontierExchange
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                            world_size=world)
    try:
        out = []
        fx = FrontierExchange(device=0, group=dist.group.WORLD, part_above=4, repl_below=2)
        for recs in keys:
            r = fx.check(np.array(recs, dtype=np.int64).reshape(-1, 6))
            out.append([int(r[f]) for f in FIELDS])
        st = fx.stats()
        fx.close()
        q.put((rank, out, st))
    except Exception as e:  # reported by the parent
        q.put((rank, repr(e), None))
    finally:
        dist.destroy_process_group()


def _nccl_main(port, q):
    import torch
    import torch.distributed as dist
    from jepsen.etcd_amd import fx as F
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0,
                            world_size=1)
    try:
        tr = F.TorchTransport(dist.group.WORLD, device=0)
        assert tr.on_device
        import ctypes
        send = (ctypes.c_int64 * 1)(7)
        recv = (ctypes.c_int64 * 1)(0)
        assert tr._counts(None, send, recv) == 0 and recv[0] == 7
        src = torch.arange(48, dtype=torch.uint8, device="cuda")
        dst = torch.zeros(48, dtype=torch.uint8, device="cuda")
        sc = (ctypes.c_int64 * 1)(3)
        rc = (ctypes.c_int64 * 1)(3)
        assert tr._a2av(None, src.data_ptr(), sc, dst.data_ptr(), rc, 16) == 0, tr.error
        vals = (ctypes.c_int64 * 2)(4, 9)
        assert tr._allred(None, vals, 2, F.LC_FX_SUM) == 0 and list(vals) == [4, 9]
        q.put(bool(torch.equal(src, dst)))
    except Exception as e:
        q.put(repr(e))
    finally:
        dist.destroy_process_group()


def _rccl_rank_main(port, keys, q):
    import torch.distributed as dist
    from jepsen.etcd_amd.fx import LC_FX_FLAG_EXCHANGE_SELF, FrontierExchange
    dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=0,
                            world_size=1)
    try:
        fx = FrontierExchange(device=0, rccl_group=dist.group.WORLD, part_above=0,
                              flags=LC_FX_FLAG_EXCHANGE_SELF)
        out = []
        for recs in keys:
            r = fx.check(np.array(recs, dtype=np.int64).reshape(-1, 6))
            out.append([int(r[f]) for f in FIELDS])
        st = fx.stats()
        fx.close()
        q.put((out, st))
    except Exception as e:
        q.put((repr(e), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_fx_rccl_multiprocess_entry_point():
    """lc_fx_open_rccl, the one-process-per-GPU form (torchrun): rank 0's
    ncclUniqueId travels over a torch.distributed group, then the library's
    own communicator carries the search (one rank here, exchanging with
    itself; RCCL refuses two ranks on one device)."""
    import torch.multiprocessing as mp
    rng = random.Random(0xD17)
    keys = [random_casreg(rng, rng.randrange(5, 50), p_info=0.1) for _ in range(8)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_rank_main, args=(_free_port(), keys, q))
    p.start()
    out, st = q.get(timeout=180)
    p.join(timeout=60)
    assert st is not None, out
    assert st["part_returns"] > 0
    for recs, got in zip(keys, out):
        _compare(dict(zip(FIELDS, got)), _oracle(recs, -1), "rccl process")


@pytest.mark.gpu
def test_torch_transport_rccl_device_buffers():
    """TorchTransport under "nccl" (RCCL): the engine's device buffers reach
    all_to_all_single through __cuda_array_interface__ with no copy.  One
    rank (this pool has one GPU per box; RCCL refuses two ranks on one
    device), so the collective is a self-exchange."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_main, args=(_free_port(), q))
    p.start()
    out = q.get(timeout=180)
    p.join(timeout=60)
    assert out is True, out


@pytest.mark.gpu
def test_fx_two_processes_over_torch_distributed():
    """Two ranks (processes) on one card, collectives over gloo through
    TorchTransport: equal results on both ranks, equal to the oracle."""
    import torch.multiprocessing as mp
    rng = random.Random(0xD15)
    keys = [random_casreg(rng, rng.randrange(5, 50), p_info=0.1) for _ in range(12)]
    ops, off, _, _ = abi.synth(2, 250, concurrency=10, p_info=0.01, p_anomaly=0.5, seed=0xD16)
    ops = ops.copy()
    ops[:, 3] = -1
    keys += [ops[off[k]:off[k + 1]].tolist() for k in range(2)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, keys, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, out, st = q.get(timeout=240)
        assert st is not None, out
        res[rank] = (out, st)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] == res[1][0]
    assert res[0][1]["part_returns"] > 0 and res[0][1]["sent_configs"] + res[1][1]["sent_configs"] > 0
    for recs, got in zip(keys, res[0][0]):
        want = _oracle(recs, -1)
        _compare(dict(zip(FIELDS, got)), want, "two processes")
