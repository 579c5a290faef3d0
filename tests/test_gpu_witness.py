"""GPU decisions certified by their witnesses (lc_aux), checked on the CPU by
oracle/witness.c — independent of the gap-matching procedure that produced
them, so this pins the full-size decisions no oracle search finishes:
BASELINE configs[3] (C4) at its stated 20 % crashed ops, and C2 with crashes.
Also the multi-device fan-out (LC_VIRTUAL_DEVICES) and per-key error model."""
import os

import numpy as np
import pytest

import gapmatch_ref as gm
import oracle
from helpers import GOLDEN, INF, pack_keys
from jepsen.etcd_amd import abi

pytestmark = pytest.mark.gpu


def certify(ops, off, r, wit, kind):
    st, ln = oracle.check_witness(ops, off, wit, kind, results=r, n_threads=16)
    bad = np.nonzero((kind != abi.LC_WITNESS_NONE) & (st != oracle.WIT_OK))[0]
    assert len(bad) == 0, [(int(k), int(kind[k]), oracle.WIT_CODES[int(st[k])]) for k in bad[:5]]
    # kinds match verdicts
    assert ((kind != abi.LC_WITNESS_FULL) | (r["verdict"] == 1)).all()
    assert ((kind != abi.LC_WITNESS_PREFIX) | (r["verdict"] == 0)).all()
    return st, ln


@pytest.mark.parametrize("name", ["c1", "c5", "info", "tiny"])
def test_witnesses_of_golden_fixtures(ctx, name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    _, r, wit, kind = ctx.check(z["ops"], z["key_off"], witness=True)
    assert (r["verdict"] == z["verdict"]).all() and (r["fail_op"] == z["fail_op"]).all()
    certify(z["ops"], z["key_off"], r, wit, kind)
    # the version-order and gap tiers witness every key they decide; only
    # keys a search tier decides (version-less ops, [nil x] reads) have none
    n_none = int((kind == abi.LC_WITNESS_NONE).sum())
    if name in ("c1", "c5"):
        assert n_none == 0
    # the witness outputs change nothing else
    _, r2 = ctx.check(z["ops"], z["key_off"])
    assert (r2 == r).all()


@pytest.mark.parametrize("seed,anom", [(0x5EED0004, 0.0), (1006, 0.0), (1010, 0.0),
                                       (1004, 1.0), (1007, 1.0), (1009, 1.0)])
def test_c4_at_20pct_crashed_certified(ctx, seed, anom):
    """BASELINE configs[3] as stated: one key, 5,000 ops, concurrency 50,
    1,000 (20 %) crashed writes/CAS.  Valid: the gap tier's linearization of
    the whole history passes the independent check.  With an injected
    anomaly: invalid, the counterexample agrees with the restated procedure,
    and the prefix just before the failing return is certified linearizable
    by its own witness (so the failing return is the first one that fails,
    given prefix-closure)."""
    ops, off, lab, _ = abi.synth(1, 5000, concurrency=50, p_info=0.2, info_frac=0.2,
                                 p_anomaly=anom, seed=seed)
    assert int((ops[:, 5] == INF).sum()) == 1000
    _, r, wit, kind = ctx.check(ops, off, witness=True)
    recs = [tuple(x) for x in ops.tolist()]
    want = gm.decide(recs)
    assert want is not None and r["verdict"][0] == want
    if want == 0:
        assert (r["fail_op"][0], r["fail_prefix_end"][0]) == gm.first_failure(recs)
        assert kind[0] == abi.LC_WITNESS_PREFIX
    else:
        assert kind[0] == abi.LC_WITNESS_FULL
    if lab[0] == 1:
        assert want == 0
    assert want == (0 if anom else 1)  # these seeds: three valid keys, three invalid
    st, ln = certify(ops, off, r, wit, kind)
    assert st[0] == oracle.WIT_OK and ln[0] > (3000 if want else 0)


def certify_invalid(ops, off, r, cert, cset, min_keys=1):
    """Every invalid key with a PREFIX witness carries an infeasibility
    certificate that oracle/cert.c accepts from the records alone (the
    witness shows the prefix before the failing return linearizable, the
    certificate the prefix at it not: the failing return is the first)."""
    st = oracle.check_certificate(ops, off, cert.reshape(-1), cset, r, n_threads=16)
    inv = np.nonzero(r["verdict"] == 0)[0]
    assert len(inv) >= min_keys
    assert not (st == oracle.CERT_BAD).any(), [(int(k), cert[k].tolist()) for k in
                                              np.nonzero(st == oracle.CERT_BAD)[0][:5]]
    return st


@pytest.mark.parametrize("seed", [1004, 1007, 1009])
def test_c4_invalid_certificates(ctx, seed):
    """BASELINE configs[3]'s invalid keys (20 % crashed, an injected anomaly):
    no oracle search finishes on them, so their counterexamples were certified
    on one side only (the witness of the prefix before the failing return).
    The certificate closes the other side: the prefix at the failing return
    has no linearization, by facts oracle/cert.c checks from the records."""
    ops, off, _, _ = abi.synth(1, 5000, concurrency=50, p_info=0.2, info_frac=0.2,
                               p_anomaly=1.0, seed=seed)
    _, r, wit, kind, cert, cset = ctx.check(ops, off, witness=True, certificate=True)
    assert r["verdict"][0] == 0 and kind[0] == abi.LC_WITNESS_PREFIX
    certify(ops, off, r, wit, kind)
    st = certify_invalid(ops, off, r, cert, cset)
    assert st[0] == oracle.CERT_OK, cert[0].tolist()


@pytest.mark.parametrize("case", ["c5", "c2_crashes", "mixed_crash", "dup"])
def test_invalid_keys_certified(ctx, case):
    """Every invalid key the version-pinned tiers decide — by the first-failure
    rule (C5 shapes, duplicated versions), the gap tier's bisection
    (crash-heavy keys) or its multisection — carries a certificate the
    checker accepts; valid keys carry none."""
    from helpers import dup_versions
    if case == "c5":
        z = np.load(os.path.join(GOLDEN, "c5.npz"))
        ops, off = z["ops"], z["key_off"]
    elif case == "c2_crashes":
        ops, off, _, _ = abi.synth(24, 1000, concurrency=20, p_info=0.05, p_anomaly=0.4,
                                   seed=0x5EED0013)
    elif case == "mixed_crash":
        ops, off, _, _ = abi.synth(2000, 120, concurrency=12, p_info=0.2, info_frac=0.15,
                                   p_anomaly=0.35, seed=51)
    else:
        ops, off, _, _ = abi.synth(600, 200, concurrency=10, p_anomaly=0.6, seed=52)
        ops, off = pack_keys(dup_versions([ops[off[k]:off[k + 1]].tolist() for k in range(600)],
                                          52, frac=0.7))
    _, r, wit, kind, cert, cset = ctx.check(ops, off, witness=True, certificate=True)
    certify(ops, off, r, wit, kind)
    st = certify_invalid(ops, off, r, cert, cset, min_keys=3)
    pinned = kind == abi.LC_WITNESS_PREFIX
    assert (st[pinned] == oracle.CERT_OK).all(), [
        (int(k), cert[k].tolist()) for k in np.nonzero(pinned & (st != oracle.CERT_OK))[0][:5]]
    assert (cert[r["verdict"] != 0][:, 0] == abi.LC_CERT_NONE).all()
    # the certificate outputs change nothing else
    _, r2 = ctx.check(ops, off)
    assert (r2 == r).all()


def test_branch_fixture_certified(ctx):
    """tests/golden/branch.npz: invalid keys whose failing prefix only a
    search over who holds the open positions refutes (no fixed certificate
    kind covers them).  The device's verdicts and fail ops are the
    fixture's, and its finder proves each one (LC_CERT_PROOF) by a proof
    oracle/cert.c checks step by step."""
    z = np.load(os.path.join(GOLDEN, "branch.npz"))
    ops, off = z["ops"], z["key_off"]
    _, r, wit, kind, cert, cset = ctx.check(ops, off, witness=True, certificate=True)
    assert (r["verdict"] == 0).all() and (r["fail_op"] == z["fail_op"]).all()
    assert (r["fail_prefix_end"] == z["fail_prefix_end"]).all()
    certify(ops, off, r, wit, kind)
    st = certify_invalid(ops, off, r, cert, cset, min_keys=100)
    assert (st == oracle.CERT_OK).all(), [(int(k), cert[k].tolist())
                                          for k in np.nonzero(st != oracle.CERT_OK)[0][:5]]
    assert (cert[:, 0] == abi.LC_CERT_PROOF).sum() >= 100


def test_crash_leg_every_key_certified(ctx):
    """bench.py's crash_leg workload at full size: C2 (10,000 keys x 1,000
    ops, concurrency 20) with 5 % of writes/CAS crashed.  Every key goes to
    the gap tier; every verdict is valid and every one is certified by its
    witness on the CPU."""
    ops, off, _, _ = abi.synth(10000, 1000, concurrency=20, p_info=0.05, seed=0x5EED0012)
    _, r, wit, kind = ctx.check(ops, off, witness=True)
    assert ctx.stats()["n_gap_keys"] == 10000
    assert (r["verdict"] == 1).all() and (kind == abi.LC_WITNESS_FULL).all()
    st, _ = certify(ops, off, r, wit, kind)
    assert (st == oracle.WIT_OK).all()


@pytest.mark.parametrize("case", ["crash_leg", "mixed", "clean"])
def test_fused_pass_equals_two_passes(ctx, monkeypatch, case):
    """Crash-heavy batches take one fused pass (version order + crash-light
    decision over every key) instead of the version-order tier followed by
    the crash-light pass over the keys it hands on (lincheck.cpp picks it
    from the previous call; LC_FUSED forces either).  Results and witnesses
    are identical, and the fused pass's decisions are certified."""
    if case == "crash_leg":
        ops, off, _, _ = abi.synth(2000, 1000, concurrency=20, p_info=0.05, seed=0x5EED0012)
    elif case == "mixed":
        ops, off, _, _ = abi.synth(2000, 120, concurrency=12, p_info=0.2, info_frac=0.15,
                                   p_anomaly=0.35, seed=52)
    else:
        ops, off, _, _ = abi.synth(1000, 300, concurrency=10, p_anomaly=0.1, seed=53)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("LC_FUSED", mode)
        _, r, wit, kind = ctx.check(ops, off, witness=True)
        out[mode] = (r, wit, kind)
    r0, w0, k0 = out["0"]
    r1, w1, k1 = out["1"]
    assert (r0 == r1).all() and (k0 == k1).all() and (w0 == w1).all()
    st, _ = certify(ops, off, r1, w1, k1)
    assert ((st == oracle.WIT_OK) | (k1 == abi.LC_WITNESS_NONE)).all()
    if case == "crash_leg":
        assert (r1["verdict"] == 1).all() and (k1 == abi.LC_WITNESS_FULL).all()


def test_mixed_crash_batch_witnesses(ctx):
    """Many short crash-heavy keys, a third of them invalid: one-wave gap
    workgroups, in-place bisection, prefix witnesses."""
    ops, off, _, _ = abi.synth(2000, 120, concurrency=12, p_info=0.2, info_frac=0.15,
                               p_anomaly=0.35, seed=51)
    _, r, wit, kind = ctx.check(ops, off, witness=True)
    st, _ = certify(ops, off, r, wit, kind)
    assert (kind == abi.LC_WITNESS_PREFIX).sum() > 300
    assert (kind == abi.LC_WITNESS_FULL).sum() > 1000
    _, j = oracle.check(ops, off, algo=oracle.JITC, n_threads=16, max_configs=1 << 20)
    known = j["verdict"] != -1
    for f in ("verdict", "fail_op", "fail_prefix_end"):
        assert (r[f][known] == j[f][known]).all(), f


def test_witness_device_path_matches_host_path(ctx):
    import torch
    ops, off, _, _ = abi.synth(300, 200, concurrency=10, p_info=0.2, p_anomaly=0.3, seed=61)
    _, r, wit, kind = ctx.check(ops, off, witness=True)
    dev = torch.device("cuda", 0)
    d_ops = torch.from_numpy(ops).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    d_out = torch.zeros(300 * 40, dtype=torch.uint8, device=dev)
    d_wit = torch.full((len(ops),), -7, dtype=torch.int32, device=dev)
    d_kind = torch.full((300,), -7, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream(dev)
    ctx.check_device(d_ops.data_ptr(), d_off.data_ptr(), 300, d_out.data_ptr(),
                     stream=s.cuda_stream, d_witness=d_wit.data_ptr(),
                     d_witness_kind=d_kind.data_ptr())
    r2 = np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)
    assert (r2 == r).all()
    assert (d_kind.cpu().numpy() == kind).all()
    w2 = d_wit.cpu().numpy()
    has = np.repeat(kind != 0, np.diff(off))
    assert (w2[has] == wit[has]).all()


def test_virtual_devices_fan_out_equals_one_device(ctx, monkeypatch):
    """lc_check's multi-device path (cost partition, one host thread and
    stream per device, results into one array) run as 3 contexts on one GPU
    (LC_VIRTUAL_DEVICES): identical results and witnesses to the
    single-device call, on a batch whose crash-heavy keys are clustered."""
    heavy, hoff, _, _ = abi.synth(300, 300, concurrency=16, p_info=0.2, p_anomaly=0.3, seed=71)
    light, loff, _, _ = abi.synth(2700, 300, concurrency=16, p_anomaly=0.05, seed=72)
    ops = np.concatenate([heavy, light])
    off = np.concatenate([hoff, loff[1:] + hoff[-1]])
    _, a, wa, ka = ctx.check(ops, off, witness=True)
    monkeypatch.setenv("LC_VIRTUAL_DEVICES", "3")
    with abi.Context(device_mask=1) as c3:
        _, b, wb, kb = c3.check(ops, off, witness=True)
        st = c3.stats()
    assert st["n_devices"] == 3
    assert (a == b).all() and (ka == kb).all() and (wa == wb).all()
    bounds = abi.plan_partition(off, 3, ops=ops)
    assert bounds[1] < 1000  # the clustered heavy keys are spread by cost


def test_c2_fan_out_over_8_devices(ctx, monkeypatch):
    """BASELINE configs[2] (C3) the way the drop-in runs it: one lc_ctx over
    8 devices (here 8 device contexts on one GPU, LC_VIRTUAL_DEVICES), the
    whole C2 batch (10k keys x 1k ops) from host buffers through lc_check's
    in-process fan-out.  Every result field equals the one-device call; the
    per-device stats cover the keys in 8 contiguous cost-balanced ranges;
    with the caller's buffer page-locked (lc_host_register) the results are
    the same and every device reports pinned copies."""
    ops, off, _, _ = abi.synth(10000, 1000, concurrency=20, seed=0x5EED0002)
    _, a = ctx.check(ops, off)
    monkeypatch.setenv("LC_VIRTUAL_DEVICES", "8")
    with abi.Context(device_mask=1) as c8:
        _, b = c8.check(ops, off)
        assert c8.stats()["n_devices"] == 8
        ds = c8.device_stats()
        c8.host_register(ops)
        try:
            _, c = c8.check(ops, off)
            dp = c8.device_stats()
        finally:
            c8.host_unregister(ops)
    assert (a == b).all() and (a == c).all() and (a["verdict"] == 1).all()
    bounds = abi.plan_partition(off, 8, ops=ops)
    assert [(d["key_begin"], d["key_end"]) for d in ds] == \
        [(int(bounds[i]), int(bounds[i + 1])) for i in range(8)]
    assert sum(d["h2d_bytes"] for d in ds) == ops.nbytes + 8 * 8 + 8 * 10000
    assert all(d["pinned"] == 0 for d in ds) and all(d["pinned"] == 1 for d in dp)
    assert all(d["h2d_ms"] > 0 and d["kernel_ms"] > 0 for d in ds + dp)


def test_malformed_key_is_unknown_alone(ctx):
    """One malformed key no longer fails the call: it is :unknown with reason
    malformed (jepsen.independent would lose only that key), and the other
    keys — an invalid one among them — keep their verdicts.  A version no
    state reaches (beyond int32, or below -1) is not malformed: knossos
    rejects the op at every step, so the key is invalid."""
    W, R = 1, 0
    bad_order = [[W, 1, -1, 1, 5, 6], [W, 2, -1, 2, 3, 4]]
    stale = [[W, 1, -1, 1, 0, 1], [W, 2, -1, 2, 2, 3], [R, 1, -1, 1, 4, 5]]
    huge_ver = [[W, 1, -1, 1, 0, 1], [R, 1, -1, 1 << 40, 2, 3]]
    neg_ver = [[W, 1, -1, -7, 0, 1]]
    huge_crashed = [[W, 1, -1, 1 << 40, 0, INF], [W, 2, -1, 1, 1, 2]]
    good = [[W, 1, -1, 1, 0, 1]]
    keys = [bad_order, stale, huge_ver, neg_ver, huge_crashed, good]
    ops, off = pack_keys(keys)
    rc, r = ctx.check(ops, off, raise_on_error=False)
    assert rc == 0
    assert list(r["verdict"]) == [-1, 0, 0, 0, 1, 1]
    assert r["reason"][0] == abi.LC_REASON_MALFORMED and ctx.stats()["n_malformed"] == 1
    _, o = oracle.check(ops[off[1]:], off[1:] - off[1], algo=oracle.JIT)
    assert (r["verdict"][1:] == o["verdict"]).all() and (r["fail_op"][1:] == o["fail_op"]).all()


@pytest.mark.parametrize("seed", [61, 62])
def test_gap_tier_early_launch_equal(ctx, monkeypatch, seed):
    """A few long keys: the gap tier proper is launched right behind the
    crash-light pass (sized from the host offsets, its task count read on the
    device) instead of after a host round trip for the status.  Same results
    and witnesses as the waiting launch, on valid and invalid long keys mixed
    with short ones the light pass decides alone."""
    lng, lo, _, _ = abi.synth(6, 2500, concurrency=30, p_info=0.2, info_frac=0.2,
                              p_anomaly=0.5, seed=seed)
    sht, so, _, _ = abi.synth(10, 60, concurrency=6, p_info=0.2, p_anomaly=0.3, seed=seed + 100)
    keys = [lng[lo[k]:lo[k + 1]].tolist() for k in range(6)]
    keys += [sht[so[k]:so[k + 1]].tolist() for k in range(10)]
    ops, off = pack_keys(keys)
    outs = []
    for early in ("0", "1"):
        monkeypatch.setenv("LC_GAP_EARLY", early)
        _, r, wit, kind = ctx.check(ops, off, witness=True)
        outs.append((r, wit, kind))
    (a, wa, ka), (b, wb, kb) = outs
    assert (a == b).all() and (ka == kb).all() and (wa == wb).all()
    certify(ops, off, b, wb, kb)
    assert (b["verdict"][:6] == 0).any() and (b["verdict"] == 1).any()


def test_proof_search_over_its_cap_leaves_no_certificate(ctx):
    """helpers.proof_cap_key: the device's PROOF search (cert.hip, 2,048
    nodes) runs out before it refutes the failing prefix.  The key stays
    invalid with the oracle's fail op and a checked PREFIX witness, and
    carries LC_CERT_NONE (certified on the witness side only) — next to a
    branch-fixture key the same call proves, so the cap is per key."""
    from helpers import proof_cap_key
    z = np.load(os.path.join(GOLDEN, "branch.npz"))
    k0 = [z["ops"][z["key_off"][0]:z["key_off"][1]].tolist()]
    ops, off = pack_keys([proof_cap_key()] + k0)
    _, r, wit, kind, cert, cset = ctx.check(ops, off, witness=True, certificate=True)
    assert list(r["verdict"]) == [0, 0] and r["fail_op"][0] == 34
    assert r["fail_op"][1] == z["fail_op"][0]
    assert list(kind) == [abi.LC_WITNESS_PREFIX, abi.LC_WITNESS_PREFIX]
    certify(ops, off, r, wit, kind)
    assert cert[0, 0] == abi.LC_CERT_NONE and cert[1, 0] == abi.LC_CERT_PROOF
    st = oracle.check_certificate(ops, off, cert.reshape(-1), cset, r)
    assert st[1] == oracle.CERT_OK
