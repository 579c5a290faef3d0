"""GPU parity tests: the HIP path through the C ABI against the oracle and the
hand-derived known answers.  Integer work: bit-exact verdicts and fail ops."""
import os

import numpy as np
import pytest

import oracle
from helpers import GOLDEN, INF, load_kats, pack_keys, tiny_batch
from jepsen.etcd_amd import abi

pytestmark = pytest.mark.gpu

KATS = load_kats()


def test_kats(ctx):
    ops, off = pack_keys([k["ops"] for k in KATS])
    rc, r = ctx.check(ops, off)
    assert rc == 0
    for i, k in enumerate(KATS):
        assert r["verdict"][i] == (1 if k["valid"] else 0), k["name"]
        assert r["fail_op"][i] == k["fail_op"], k["name"]
        assert r["fail_prefix_end"][i] == k["fail_prefix_end"], k["name"]


@pytest.mark.parametrize("name", ["c1", "c5", "info", "tiny"])
def test_golden_fixtures(ctx, name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    _, r = ctx.check(z["ops"], z["key_off"])
    assert (r["verdict"] == z["verdict"]).all()
    assert (r["fail_op"] == z["fail_op"]).all()


@pytest.mark.parametrize("name", ["c1", "c5", "info", "tiny"])
def test_fast_tier_and_search_agree(ctx, name):
    """Version-order tier + JIT vs the JIT search alone: identical verdicts and
    fail ops (the fast tier hands invalid keys to the JIT for the fail op)."""
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    _, a = ctx.check(z["ops"], z["key_off"])
    fast_decided = len(a) - ctx.stats()["n_jit_keys"]
    _, b = ctx.check(z["ops"], z["key_off"], abi.default_opts(flags=abi.LC_FLAG_NO_FAST_PATH))
    assert ctx.stats()["n_jit_keys"] == len(b)
    assert (a["verdict"] == b["verdict"]).all() and (a["fail_op"] == b["fail_op"]).all()
    if name in ("c1", "c5"):
        assert fast_decided >= 0.85 * len(a)


def test_tiny_random_vs_oracle(ctx):
    ops, off = pack_keys(tiny_batch(777, 20000, max_ops=8))
    _, g = ctx.check(ops, off)
    _, j = oracle.check(ops, off, algo=oracle.JIT, n_threads=8)
    assert (g["verdict"] == j["verdict"]).all()
    assert (g["fail_op"] == j["fail_op"]).all()
    assert (g["fail_prefix_end"] == j["fail_prefix_end"]).all()


@pytest.mark.parametrize("conc,p_info,p_anom,seed", [
    (10, 0.0, 0.1, 0x5EED0005),   # C5-shaped
    (20, 0.0, 0.2, 11),
    (30, 0.02, 0.2, 12),
    (8, 0.1, 0.1, 13),
])
def test_synthetic_vs_oracle(ctx, conc, p_info, p_anom, seed):
    ops, off, lab, _ = abi.synth(400, 200, concurrency=conc, p_info=p_info,
                                 p_anomaly=p_anom, seed=seed)
    _, g = ctx.check(ops, off)
    _, j = oracle.check(ops, off, algo=oracle.JITC, n_threads=8, max_configs=1 << 21)
    known = j["verdict"] != -1
    assert known.mean() > 0.95
    assert (g["verdict"][known] == j["verdict"][known]).all()
    assert (g["fail_op"][known] == j["fail_op"][known]).all()
    assert (g["verdict"][lab == 1] == 0).all()   # stale reads are always visible


def _prefix(recs, end):
    """History truncated at index `end`: ops called after it dropped, ops
    still open at it made pending (completed fields kept)."""
    out = []
    for r in recs:
        if r[4] > end:
            continue
        r = list(r)
        if r[5] > end:
            r[5] = INF
        out.append(r)
    return out


def test_counterexamples_are_minimal_nonlinearizable_prefixes(ctx):
    ops, off, lab, _ = abi.synth(500, 200, concurrency=10, p_anomaly=0.5, seed=21)
    _, g = ctx.check(ops, off)
    bad = np.nonzero(g["verdict"] == 0)[0]
    assert len(bad) > 100
    pre, prev = [], []
    for k in bad:
        recs = ops[off[k]:off[k + 1]].tolist()
        end = int(g["fail_prefix_end"][k])
        assert recs[g["fail_op"][k]][5] == end
        pre.append(_prefix(recs, end))
        # the prefix ending just before the failing return is linearizable
        rets = sorted(r[5] for r in recs if r[5] < end)
        prev.append(_prefix(recs, rets[-1]) if rets else [])
    p_ops, p_off = pack_keys(pre)
    _, a = oracle.check(p_ops, p_off, algo=oracle.WGL, n_threads=8)
    assert (a["verdict"] == 0).all()
    q_ops, q_off = pack_keys(prev)
    _, b = oracle.check(q_ops, q_off, algo=oracle.WGL, n_threads=8)
    assert (b["verdict"] == 1).all()


@pytest.mark.parametrize("conc,seed,dup", [(10, 0x5EED0005, False), (6, 51, True),
                                           (20, 52, True), (10, 53, False)])
def test_first_failure_rule_vs_oracle(ctx, conc, seed, dup):
    """Invalid version-pinned keys get their fail op from the first-failure
    rule in the crash-light pass (check_kernel.hip, `first_failure`), not a
    bisection: verdict, fail op and prefix end equal knossos.linear's on
    every key, and every PREFIX witness the rule writes certifies
    (oracle/witness.c).  Keys with two mutations on one version (lost CAS;
    `dup`: one more such pair per key) are decided exactly or declined to the
    gap tier, which bisects — the same answers either way."""
    from helpers import dup_versions
    ops, off, _, _ = abi.synth(600, 200, concurrency=conc, p_anomaly=0.6, seed=seed)
    if dup:
        ops, off = pack_keys(dup_versions([ops[off[k]:off[k + 1]].tolist()
                                           for k in range(600)], seed, frac=0.7))
    _, g, wit, kind = ctx.check(ops, off, witness=True)
    _, j = oracle.check(ops, off, algo=oracle.JITC, n_threads=8)
    assert (g["verdict"] == 0).sum() > 200
    for f in ("verdict", "fail_op", "fail_prefix_end"):
        assert (g[f] == j[f]).all(), f
    st, _ = oracle.check_witness(ops, off, wit, kind, results=g)
    assert (kind[g["verdict"] == 0] == abi.LC_WITNESS_PREFIX).all()
    assert (st[kind != abi.LC_WITNESS_NONE] == oracle.WIT_OK).all()


def test_c2_full_size_properties(ctx):
    """BASELINE configs[1] at full size: 10k keys x 1k ops, concurrency 20.
    Valid by construction; a 300-key sample matches the oracle."""
    ops, off, _, _ = abi.synth(10000, 1000, concurrency=20, seed=0x5EED0002)
    _, g = ctx.check(ops, off)
    assert (g["verdict"] == 1).all()
    assert ctx.stats()["n_ops"] == 10_000_000
    _, j = oracle.check(ops[:off[300]], off[:301], algo=oracle.JITC, n_threads=8)
    assert (g["verdict"][:300] == j["verdict"]).all()


def test_long_key(ctx):
    ops, off, _, _ = abi.synth(2, 200_000, concurrency=40, p_anomaly=0.0, seed=3)
    _, g = ctx.check(ops, off)
    assert (g["verdict"] == 1).all()


def test_hbm_tier_resolves_lds_overflow(ctx, monkeypatch):
    """LDS tier first (LC_JIT_DIRECT=0): exactly the keys that outgrow it go
    on to the HBM tier; and by default (at most 1,024 frontier-search keys go
    straight to the cooperative tier) the same verdicts and fail ops."""
    z = np.load(os.path.join(GOLDEN, "info.npz"))
    nogap = abi.LC_FLAG_NO_GAP_TIER  # crash-heavy keys reach the JIT search
    o = abi.default_opts(flags=abi.LC_FLAG_NO_HBM_RETRY | nogap)
    _, lds_only = ctx.check(z["ops"], z["key_off"], o)
    spilled = lds_only["reason"] == 6
    assert spilled.any()
    monkeypatch.setenv("LC_JIT_DIRECT", "0")
    _, full = ctx.check(z["ops"], z["key_off"], abi.default_opts(flags=nogap))
    assert ctx.stats()["n_hbm_keys"] == spilled.sum()
    assert (full["verdict"] == z["verdict"]).all()
    assert (full["fail_op"] == z["fail_op"]).all()
    monkeypatch.delenv("LC_JIT_DIRECT")
    _, direct = ctx.check(z["ops"], z["key_off"], abi.default_opts(flags=nogap))
    assert ctx.stats()["n_hbm_keys"] == ctx.stats()["n_jit_keys"] > spilled.sum()
    for f in ("verdict", "fail_op", "fail_prefix_end", "max_frontier", "configs_explored"):
        assert (direct[f] == full[f]).all(), f


@pytest.mark.parametrize("mode", ["0", "4", "8", "16"])
def test_hbm_tier_cooperative_agrees(ctx, mode, monkeypatch):
    """The HBM tier with one wavefront per key (LC_HBM_COOP=0) and with a
    workgroup of 4 or 16 wavefronts per key reaches the same configuration sets: same
    verdicts, counterexamples and largest frontier as the golden vectors /
    each other (unversioned crash-heavy keys, gap tier off)."""
    z = np.load(os.path.join(GOLDEN, "info.npz"))
    o = abi.default_opts(flags=abi.LC_FLAG_NO_GAP_TIER)
    monkeypatch.setenv("LC_HBM_COOP", mode)
    _, r = ctx.check(z["ops"], z["key_off"], o)
    assert ctx.stats()["n_hbm_keys"] > 0
    assert (r["verdict"] == z["verdict"]).all()
    assert (r["fail_op"] == z["fail_op"]).all()
    # version-less keys (every key through the frontier search), valid and
    # with anomalies; the cooperative tier (LDS tables, work queue,
    # HBM tables for large returns) against the one-wave tier (HBM tables,
    # serial worklist): same verdicts, counterexamples, largest frontiers and
    # configurations explored (the expansion order differs, the sets do not)
    for seed, p_info, p_anom in ((99, 0.0, 0.0), (98, 0.0, 0.004)):
        ops, off, _, _ = abi.synth(64, 300, concurrency=20, p_info=p_info, seed=seed)
        ops[:, 3] = -1
        # version-less anomalies: a few :ok reads of a value nothing wrote
        rng = np.random.default_rng(seed)
        reads = np.nonzero((ops[:, 0] == abi.LC_F_READ) & (ops[:, 5] != abi.LC_INF))[0]
        ops[rng.choice(reads, int(len(reads) * p_anom), replace=False), 1] = 12345
        o = abi.default_opts(flags=abi.LC_FLAG_NO_GAP_TIER, time_budget_ms=5000)
        monkeypatch.setenv("LC_HBM_COOP", "0")
        _, a = ctx.check(ops, off, o)
        monkeypatch.setenv("LC_HBM_COOP", mode if mode != "0" else "1")
        _, b = ctx.check(ops, off, o)
        done = (a["verdict"] != -1) & (b["verdict"] != -1)
        # (the rest exceed the time budget: version-less concurrency-20 keys)
        assert done.sum() >= len(done) // 2, np.unique(a["reason"], return_counts=True)
        if p_anom:
            assert (a["verdict"][done] == 0).any()
        for f in ("verdict", "fail_op", "max_frontier", "configs_explored"):
            assert (a[f][done] == b[f][done]).all(), f


def test_edge_cases(ctx):
    W, R_ = 1, 0
    keys = [
        [],                                               # empty key
        [[R_, -1, -1, -1, 0, 1]],                         # lone [nil nil] read
        [[W, 1, -1, 1, 10, 11]],                          # one write
        [[R_, -1, -1, -1, i, 100 + i] for i in range(80)],  # 80 open trivial reads
        [],
    ]
    ops, off = pack_keys(keys)
    rc, r = ctx.check(ops, off)
    assert rc == 0 and (r["verdict"] == 1).all()
    rc, r = ctx.check(np.zeros((0, 6), np.int64), np.zeros(1, np.int64))
    assert rc == 0 and len(r) == 0


def test_window_overflow_is_unknown(ctx):
    recs = [[1, i % 4, -1, -1, i, INF] for i in range(65)]  # 65 crashed writes
    ops, off = pack_keys([recs, [[1, 1, -1, 1, 0, 1]]])
    _, r = ctx.check(ops, off, abi.default_opts(flags=abi.LC_FLAG_NO_GAP_TIER))
    assert r["verdict"][0] == -1 and r["reason"][0] == abi.LC_REASON_WINDOW_OVERFLOW
    assert r["verdict"][1] == 1
    # the gap tier decides it: no :ok op needs any crashed write
    _, r = ctx.check(ops, off)
    assert list(r["verdict"]) == [1, 1]


def test_budget_is_unknown(ctx):
    recs = [[1, i % 3, -1, -1, i, INF] for i in range(20)]
    recs.append([0, 2, -1, 21, 30, 31])
    ops, off = pack_keys([recs])
    o = abi.default_opts(max_configs_per_key=500, flags=abi.LC_FLAG_NO_GAP_TIER)
    _, r = ctx.check(ops, off, o)
    assert r["verdict"][0] == -1 and r["reason"][0] == abi.LC_REASON_CONFIG_BUDGET
    # the gap tier decides it: version 21 needs 21 mutations, 20 exist
    _, r = ctx.check(ops, off, abi.default_opts(max_configs_per_key=500))
    assert r["verdict"][0] == 0 and r["fail_op"][0] == 20


def _gm_recs(ops, off, k):
    return [tuple(r) for r in ops[off[k]:off[k + 1]].tolist()]


@pytest.mark.parametrize("opk,conc,seed", [(60, 10, 31), (120, 16, 32), (200, 20, 33)])
def test_gap_tier_vs_oracle(ctx, opk, conc, seed):
    """Crash-heavy keys (20 % :info, C4-shaped but small enough for the
    oracle's search): the gap tier decides them, bit-exact with the oracle
    wherever the oracle finishes, and the Python restatement everywhere."""
    import gapmatch_ref as gm
    ops, off, lab, _ = abi.synth(200, opk, concurrency=conc, p_info=0.2,
                                 p_anomaly=0.3, seed=seed)
    _, g = ctx.check(ops, off)
    st = ctx.stats()
    assert st["n_gap_keys"] > 0 and st["n_jit_keys"] == 0
    assert (g["verdict"] != -1).all()
    _, j = oracle.check(ops, off, algo=oracle.JITC, n_threads=8, max_configs=1 << 20)
    known = j["verdict"] != -1
    assert known.sum() >= 20
    assert (g["verdict"][known] == j["verdict"][known]).all()
    assert (g["fail_op"][known] == j["fail_op"][known]).all()
    assert (g["fail_prefix_end"][known] == j["fail_prefix_end"][known]).all()
    for k in range(0, 200, 7):
        recs = _gm_recs(ops, off, k)
        assert g["verdict"][k] == gm.decide(recs)
        if g["verdict"][k] == 0:
            assert (g["fail_op"][k], g["fail_prefix_end"][k]) == gm.first_failure(recs)


@pytest.mark.parametrize("budget", [1, 2, 3])
def test_gap_plain_order_rerun(ctx, monkeypatch, budget):
    """The gap tier's expected-value-first branching, cut off after `budget`
    matching passes, unwinds and reruns the plain ascending search
    (gapmatch.h): verdicts and counterexamples equal the full-budget run and
    the restated procedure, on crash-heavy keys that branch (C4-shaped, valid
    and invalid) and on a mixed batch."""
    import gapmatch_ref as gm
    cases = [abi.synth(1, 5000, concurrency=50, p_info=0.2, info_frac=0.2, p_anomaly=a, seed=s)[:2]
             for s, a in ((0x5EED0004, 0.0), (1007, 1.0))]
    cases.append(abi.synth(120, 200, concurrency=20, p_info=0.2, p_anomaly=0.3, seed=41)[:2])
    fields = ("verdict", "fail_op", "fail_prefix_end")
    for ops, off in cases:
        monkeypatch.delenv("LC_GAP_PREF_BUDGET", raising=False)
        _, full = ctx.check(ops, off)
        monkeypatch.setenv("LC_GAP_PREF_BUDGET", str(budget))
        _, cut = ctx.check(ops, off)
        for f in fields:
            assert (cut[f] == full[f]).all(), f
        assert (cut["verdict"] != -1).all()
        recs = _gm_recs(ops, off, 0)
        assert cut["verdict"][0] == gm.decide(recs)


@pytest.mark.parametrize("seed,anom", [(0x5EED0004, 0.0), (1007, 1.0), (1009, 1.0)])
def test_c4_hot_key(ctx, seed, anom):
    """BASELINE configs[3] at full size: one key, 5k ops, concurrency 50,
    20 % :info (exactly 1,000 crashed records, info_frac).  Every frontier
    search (knossos's, the oracle's, the JIT tier's) runs out of budget here;
    the gap tier decides it exactly.  No oracle search finishes, so the
    verdict is compared with the restated procedure here and certified by its
    witness in test_gpu_witness.py."""
    import gapmatch_ref as gm
    ops, off, lab, _ = abi.synth(1, 5000, concurrency=50, p_info=0.2, info_frac=0.2,
                                 p_anomaly=anom, seed=seed)
    assert int((ops[:, 5] == INF).sum()) == 1000
    _, g = ctx.check(ops, off)
    recs = _gm_recs(ops, off, 0)
    want = gm.decide(recs)
    assert want is not None and g["verdict"][0] == want
    if want == 0:
        assert (g["fail_op"][0], g["fail_prefix_end"][0]) == gm.first_failure(recs)
    if lab[0] == 1:
        assert want == 0  # an injected stale read is always visible
    assert want == (0 if anom else 1)


def test_gap_tier_c2_with_crashes(ctx):
    """C2-shaped keys (1,000 ops, concurrency 20) with 5 % crashed
    writes/CAS and injected anomalies: the shape of bench.py's crash_leg, with
    the skeleton in LDS.  Beyond the oracle's searches at this size (most keys
    exceed 4M configurations), so verdicts and counterexamples are checked
    against the restated procedure (tests/gapmatch_ref.py, itself checked
    against the oracle on smaller keys) and against the oracle's WGL wherever
    it decides."""
    import gapmatch_ref as gm
    ops, off, lab, _ = abi.synth(24, 1000, concurrency=20, p_info=0.05, p_anomaly=0.4,
                                 seed=0x5EED0013)
    _, g = ctx.check(ops, off)
    assert ctx.stats()["n_gap_keys"] == 24 and (g["verdict"] != -1).all()
    for k in range(24):
        recs = _gm_recs(ops, off, k)
        assert g["verdict"][k] == gm.decide(recs)
        if g["verdict"][k] == 0:
            assert (g["fail_op"][k], g["fail_prefix_end"][k]) == gm.first_failure(recs)
    assert (g["verdict"] == 0).sum() >= 3 and (g["verdict"] == 1).sum() >= 3
    _, w = oracle.check(ops, off, algo=oracle.WGL, n_threads=8, max_configs=1 << 18)
    known = w["verdict"] != -1
    assert (g["verdict"][known] == w["verdict"][known]).all()


def test_gap_tier_many_invalid_keys_bisect(ctx):
    """More invalid crash-heavy keys than half the gap tier's workgroups: the
    counterexamples are found by one bisecting workgroup per key instead of
    the multisection rounds; both agree with the oracle."""
    ops, off, lab, _ = abi.synth(1500, 50, concurrency=8, p_info=0.2,
                                 p_anomaly=0.9, seed=41)
    _, g = ctx.check(ops, off)
    assert (g["verdict"] == 0).sum() > 600  # > kGapMaxWG / 2: bisect mode
    _, j = oracle.check(ops, off, algo=oracle.JITC, n_threads=8, max_configs=1 << 20)
    known = j["verdict"] != -1
    assert known.sum() > 1000
    for f in ("verdict", "fail_op", "fail_prefix_end"):
        assert (g[f][known] == j[f][known]).all(), f


@pytest.mark.parametrize("seed,anom", [(0x5EED0004, 0.0), (1007, 1.0)])
def test_gap_tier_hbm_fallback_agrees(ctx, seed, anom, monkeypatch):
    """The matching arrays normally live in LDS; LC_GAP_LDS=0 keeps them in
    the HBM workspace.  Both placements give the same results (C4 hot key,
    valid and invalid, and a batch of small crash-heavy keys)."""
    cases = [abi.synth(1, 5000, concurrency=50, p_info=0.2, info_frac=0.2, p_anomaly=anom,
                       seed=seed),
             abi.synth(300, 80, concurrency=12, p_info=0.2, p_anomaly=0.4, seed=seed + 1)]
    for ops, off, _, _ in cases:
        _, a = ctx.check(ops, off)
        monkeypatch.setenv("LC_GAP_LDS", "0")
        _, b = ctx.check(ops, off)
        monkeypatch.delenv("LC_GAP_LDS")
        for f in ("verdict", "reason", "fail_op", "fail_prefix_end", "max_frontier"):
            assert (a[f] == b[f]).all(), f


def test_handoff_is_never_missed(ctx):
    """The version-order tier's handoff flag (host-coherent memory, read after
    an event sync recorded without a system fence; the kernel fences after its
    store) must be seen on every call: alternate a clean batch with a
    same-shaped crash-heavy one holding invalid keys, device-resident with one
    output buffer, so a missed handoff would leave the clean batch's verdicts
    in place for the crashed keys."""
    import torch
    dev = torch.device("cuda:0")
    clean = abi.synth(2000, 200, concurrency=10, seed=41)[:2]
    crash = abi.synth(2000, 200, concurrency=10, p_info=0.1, p_anomaly=0.3, seed=42)[:2]
    want = [ctx.check(o, f)[1] for o, f in (clean, crash)]
    assert (want[1]["verdict"] == 0).any() and (want[0]["verdict"] == 1).all()
    bufs = [(torch.from_numpy(o).to(dev), torch.from_numpy(f).to(dev)) for o, f in (clean, crash)]
    out = torch.zeros(2000 * abi.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    for i in range(40):
        k = i % 2
        d_ops, d_off = bufs[k]
        ctx.check_device(d_ops.data_ptr(), d_off.data_ptr(), 2000, out.data_ptr(),
                         stream=stream.cuda_stream)
        torch.cuda.synchronize()
        got = np.frombuffer(out.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)
        for f in ("verdict", "fail_op"):
            assert (got[f] == want[k][f]).all(), (i, f)


def test_gap_tier_repeatable(ctx):
    """Same batch, same answers, call after call: the gap tier's decisions
    within one workgroup follow each other without extra barriers, so a
    shared-word race would show as run-to-run differences here (C5 fixture:
    short invalid keys, bisected in place; a crash-heavy batch)."""
    z = np.load(os.path.join(GOLDEN, "c5.npz"))
    cases = [(z["ops"], z["key_off"]),
             abi.synth(400, 120, concurrency=12, p_info=0.2, p_anomaly=0.5, seed=77)[:2]]
    for ops, off in cases:
        _, first = ctx.check(ops, off)
        for _ in range(4):
            _, again = ctx.check(ops, off)
            for f in ("verdict", "fail_op", "fail_prefix_end", "max_frontier"):
                assert (again[f] == first[f]).all(), f
    _, r = ctx.check(z["ops"], z["key_off"])
    assert (r["verdict"] == z["verdict"]).all() and (r["fail_op"] == z["fail_op"]).all()


def test_gap_tier_and_search_agree(ctx):
    """Where the JIT search decides crash-heavy keys, the gap tier agrees."""
    z = np.load(os.path.join(GOLDEN, "info.npz"))
    _, a = ctx.check(z["ops"], z["key_off"])
    assert ctx.stats()["n_gap_keys"] > 0
    _, b = ctx.check(z["ops"], z["key_off"], abi.default_opts(flags=abi.LC_FLAG_NO_GAP_TIER))
    both = (a["verdict"] != -1) & (b["verdict"] != -1)
    assert (a["verdict"][both] == b["verdict"][both]).all()
    assert (a["fail_op"][both] == b["fail_op"][both]).all()
    assert ((a["verdict"] != -1) | (b["verdict"] == -1)).all()


def test_time_budget_is_unknown(ctx):
    """lc_opts.time_budget_ms bounds the frontier search per key: the C4 hot
    key with the gap tier off blows up every search (11.8 s to the
    configuration budget); with a 30 ms time budget it is :unknown
    (LC_REASON_TIME_BUDGET) in well under a second, while the clean keys of
    the same call are still decided."""
    import time
    hot, hoff, _, _ = abi.synth(1, 5000, concurrency=50, p_info=0.2, seed=0x5EED0004)
    ops, off, _, _ = abi.synth(20, 100, concurrency=5, seed=3)
    allops = np.concatenate([hot, ops])
    alloff = np.concatenate([hoff, off[1:] + hoff[-1]])
    t = time.perf_counter()
    _, r = ctx.check(allops, alloff, abi.default_opts(flags=abi.LC_FLAG_NO_GAP_TIER,
                                                      time_budget_ms=30))
    assert time.perf_counter() - t < 2.0
    assert r["verdict"][0] == -1 and r["reason"][0] == 7
    assert (r["verdict"][1:] == 1).all()


def test_malformed_and_unknown_f(ctx):
    bad_order = [[1, 1, -1, 1, 5, 6], [1, 2, -1, 2, 3, 4]]
    bad_ret = [[1, 1, -1, 1, 5, 5]]
    bad_range = [[1, 1 << 40, -1, 1, 0, 1]]
    unknown_f = [[7, 1, -1, 1, 0, 1]]
    good = [[1, 1, -1, 1, 0, 1]]
    ops, off = pack_keys([bad_order, bad_ret, bad_range, unknown_f, good])
    rc, r = ctx.check(ops, off, raise_on_error=False)
    assert rc == 0  # malformed keys are :unknown one by one, the call succeeds
    assert ctx.stats()["n_malformed"] == 3
    assert list(r["reason"]) == [4, 4, 4, 5, 0]
    assert list(r["verdict"]) == [-1, -1, -1, -1, 1]
    bad_off = np.array([0, 2, 1], dtype=np.int64)
    rc, _ = ctx.check(ops, bad_off, raise_on_error=False)
    assert rc == -22


def test_initial_state_option(ctx):
    # (->VersionedRegister 5 nil): the first write must report version 6
    ops, off = pack_keys([[[1, 1, -1, 6, 0, 1]], [[1, 1, -1, 1, 0, 1]]])
    _, r = ctx.check(ops, off, abi.default_opts(init_version=5))
    assert list(r["verdict"]) == [1, 0]


def test_check_device_path_with_torch(ctx):
    import torch
    z = np.load(os.path.join(GOLDEN, "c5.npz"))
    dev = torch.device("cuda", 0)
    # a slice of keys whose key_off does not start at 0
    a, b = 50, 250
    d_ops = torch.from_numpy(np.ascontiguousarray(z["ops"][z["key_off"][a]:])).to(dev)
    d_off = torch.from_numpy(np.ascontiguousarray(z["key_off"][a:b + 1])).to(dev)
    d_out = torch.zeros((b - a) * 40, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream(dev)
    ctx.check_device(d_ops.data_ptr(), d_off.data_ptr(), b - a, d_out.data_ptr(),
                     stream=s.cuda_stream)
    r = np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)
    bad = np.nonzero((r["verdict"] != z["verdict"][a:b]) | (r["fail_op"] != z["fail_op"][a:b]))[0]
    assert len(bad) == 0, [(a + int(k), r[k].tolist(), int(z["verdict"][a + k]),
                            int(z["fail_op"][a + k])) for k in bad[:5]] + [ctx.stats()]
    assert ctx.stats()["kernel_ms"] > 0
    # the pre-bound form bench.py times gives the same results and stats
    d_out.zero_()
    st = abi.LcStats()
    call = ctx.bind_check_device(d_ops.data_ptr(), d_off.data_ptr(), b - a, d_out.data_ptr(),
                                 stream=s.cuda_stream, stats=st)
    assert call() is st and st.n_keys == b - a and st.kernel_ms > 0
    r2 = np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)
    assert (r2 == r).all()


def _assert_configs_in_frontier(lin, kops, done, vals, k):
    """An invalid key's knossos :configs (at most 10) are configurations of
    the oracle's JITC frontier just before the failing return — state and
    pending ops — and its final paths end inconsistent."""
    fo = next(j for j, d in enumerate(done)
              if (d["completion"] or d["invoke"])["index"] == lin["op"]["index"])
    want, n_want = oracle.frontier(kops, fo)
    assert 1 <= len(lin["configs"]) <= min(10, n_want), k
    for cfg in lin["configs"]:
        val = cfg["model"]["value"]
        vid = -1 if val is None else vals.index(val)
        pend = tuple(sorted(next(j for j, d in enumerate(done)
                                 if d["invoke"]["index"] == inv["index"])
                            for inv in cfg["pending"]))
        assert (cfg["model"]["version"], vid, pend) in want, (k, cfg)
    assert all("inconsistent" in p[-1]["model"] for p in lin["final-paths"])


def test_register_checker_frontier_configs():
    """knossos's :configs for keys the frontier search decides: a history
    whose :ok completions carry no versions ([nil v], which the
    VersionedRegister checks only by value, register.clj:64,71,84) sends every
    key to the search tiers; each invalid key's "configs" (at most 10) are
    configurations of the oracle's JITC frontier just before the failing
    return — state and pending ops — and its final paths end inconsistent."""
    from jepsen.etcd_amd import checker as C, history as H, synth
    hist, _ = synth.jepsen_history(40, 80, concurrency=8, p_info=0.02,
                                        p_anomaly=0.5, seed=11)
    for op in hist:
        v = op.get("value")
        if op.get("type") == "ok" and isinstance(v, H.Tuple) and isinstance(v.value, (list, tuple)):
            op["value"] = H.Tuple(v.key, [None, v.value[1]])
    chk = C.register_checker(device_mask=1)
    res = chk.check({"name": "etcd register"}, hist, {})
    chk.close()
    vals = []
    keys, ops, off, done = H.pack(hist, values_out=vals)
    n_checked = 0
    for i, k in enumerate(keys):
        lin = res["results"][k]["linear"]
        if lin["valid?"] is not False:
            continue
        _assert_configs_in_frontier(lin, ops[off[i]:off[i + 1]], done[i], vals[i], k)
        n_checked += 1
    assert n_checked >= 5


def test_register_checker_end_to_end(tmp_path):
    from jepsen.etcd_amd import checker as C, synth
    hist, labels = synth.jepsen_history(60, 120, concurrency=10, p_info=0.03,
                                        p_anomaly=0.3, seed=5)
    chk = C.register_checker(device_mask=1, timeline_dir=str(tmp_path))
    res = chk.check({"name": "etcd register"}, hist, {})
    chk.close()
    from jepsen.etcd_amd import history as H
    vals = []
    _, ops, off, done = H.pack(hist, values_out=vals)
    _, ref = oracle.check(ops, off, algo=oracle.JITC)
    bad = sorted(int(k) for k in np.nonzero(ref["verdict"] == 0)[0])
    assert set(k for k, l in enumerate(labels) if l == 1) <= set(bad)
    assert res["valid?"] is False
    assert sorted(res["failures"]) == bad
    for k in bad:
        r = res["results"][k]
        assert r["valid?"] is False and r["linear"]["op"]["type"] == "ok"
        # knossos's diagnostics: :configs from the frontier re-search (keys
        # with at most FRONTIER_MAX_CRASHED crashed ops: every key here),
        # :last-op from the prefix witness (diagnostics.py)
        lin = r["linear"]
        assert lin["previous-ok"]["index"] < lin["fail-prefix-end"]
        assert "configs-error" not in lin and "last-op" in lin
        _assert_configs_in_frontier(lin, ops[off[k]:off[k + 1]], done[k], vals[k], k)
        page = open(r["timeline"]["file"]).read()  # independent/<k>/timeline.html
        assert 'cex"' in page and os.path.dirname(r["timeline"]["file"]).endswith("/%d" % k)
        svg = open(lin["linear-svg"]).read()  # independent/<k>/linear.svg
        assert 'class="fail"' in svg and os.path.dirname(lin["linear-svg"]) == \
            os.path.dirname(r["timeline"]["file"])
    assert res["results"][0]["timeline"]["valid?"] is True
    assert C.check_safe(chk, {}, [{"type": "invoke", "process": 0, "value": None}]) == \
        {"valid?": True, "results": {}, "failures": []}


def test_cooperative_pool_and_epoch_wrap_agree(ctx, monkeypatch):
    """The model leg's own keys (version-less, 1,000 ops, concurrency 20):
    hundreds of cooperative returns per key, so the 8-bit LDS epoch wraps
    (tables cleared), and the keys with the largest frontiers have returns
    past the LDS pool (nR + nW > 1,688: redone on HBM tables).  The six
    largest-frontier keys through the cooperative tier against the one-wave
    tier (HBM tables, serial worklist) — every result field."""
    ops, off, _, _ = abi.synth(1000, 1000, concurrency=20, seed=7)
    ops = ops.copy()
    ops[:, 3] = abi.LC_NIL
    _, full = ctx.check(ops, off)
    pick = np.argsort(full["max_frontier"])[-6:]
    keys = [ops[off[k]:off[k + 1]] for k in pick]
    sub = np.concatenate(keys)
    soff = np.concatenate([[0], np.cumsum([len(x) for x in keys])]).astype(np.int64)
    o = abi.default_opts(flags=abi.LC_FLAG_NO_GAP_TIER, time_budget_ms=60000)
    monkeypatch.setenv("LC_HBM_COOP", "0")
    _, a = ctx.check(sub, soff, o)
    monkeypatch.setenv("LC_HBM_COOP", "4")
    _, b = ctx.check(sub, soff, o)
    assert (a["verdict"] == 1).all() and (b["verdict"] == 1).all()
    assert int(b["max_frontier"].max()) > 1688  # returns past the pool
    for f in ("verdict", "reason", "fail_op", "fail_prefix_end", "configs_explored", "max_frontier"):
        assert (a[f] == b[f]).all(), f
        assert (b[f] == full[f][pick]).all(), f
