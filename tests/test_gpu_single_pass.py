"""The version-order / fused / crash-light passes after round 4's single
record pass (check_kernel.hip, fast_key): value claims as LDS
compare-and-swaps, crashed ops stashed per wave in LDS, lane 0's order check
against the previous wave's last call through LDS, DPP wave scans.  Edge
cases of each, on both the fused pass and the two-pass path (LC_FUSED)."""
import numpy as np
import pytest

import oracle
from helpers import INF, dup_versions, pack_keys
from jepsen.etcd_amd import abi
from test_gpu_witness import certify

pytestmark = pytest.mark.gpu


def both_paths(ctx, monkeypatch, ops, off):
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("LC_FUSED", mode)
        _, r, wit, kind = ctx.check(ops, off, witness=True)
        out[mode] = (r, wit, kind)
    (r0, w0, k0), (r1, w1, k1) = out["0"], out["1"]
    assert (r0 == r1).all() and (k0 == k1).all() and (w0 == w1).all()
    return r1, w1, k1


@pytest.mark.parametrize("info", [0.0, 0.05])
def test_order_violation_at_every_boundary(ctx, monkeypatch, info):
    """A record whose call does not follow its predecessor's makes the key
    malformed wherever it sits: inside a wave (lane-1 by DPP), at a wave's
    first lane (the previous wave's last call, through LDS) and at a chunk's
    first record (the last wave of the chunk before)."""
    base, boff, _, _ = abi.synth(12, 1000, concurrency=20, p_info=info, seed=71)
    keys = [base[boff[k]:boff[k + 1]].tolist() for k in range(12)]
    spots = [1, 63, 64, 65, 128, 192, 256, 257, 512, 768, 960]
    bad = []
    for i, r in enumerate(spots):
        recs = [list(x) for x in keys[i]]
        recs[r][4] = recs[r - 1][4]  # same call as its predecessor (ret still after it)
        bad.append(recs)
    ops, off = pack_keys(bad + [keys[11]])
    r, _, _ = both_paths(ctx, monkeypatch, ops, off)
    assert (r["verdict"][:len(spots)] == -1).all(), r["verdict"].tolist()
    reason = r["reason"][:len(spots)]
    if info == 0:
        assert (reason == abi.LC_REASON_MALFORMED).all(), reason.tolist()
    else:
        # the key goes to the JIT search, which reports the record when it
        # reaches it; with crashed ops in the window it may run out of its
        # configuration budget first on a late one (:unknown either way)
        assert ((reason == abi.LC_REASON_MALFORMED) |
                (reason == abi.LC_REASON_CONFIG_BUDGET)).all(), reason.tolist()
        assert (reason[:4] == abi.LC_REASON_MALFORMED).all(), reason.tolist()
    assert r["verdict"][-1] == 1


def crash_in_wave0(recs, count, rng):
    """`count` :ok writes among wave 0's records (r % 256 < 64) made crashed
    writes without a version: the history stays valid (each still takes effect
    where it did), and pass 1 stashes them all in wave 0's LDS stash."""
    recs = [list(x) for x in recs]
    cand = [i for i, x in enumerate(recs) if i % 256 < 64 and x[0] == 1 and x[5] != INF and x[3] != -1]
    for i in rng.choice(cand, size=count, replace=False):
        recs[i][3] = -1
        recs[i][5] = INF
    return recs


def test_stash_overflow_goes_to_the_gap_tier(ctx, monkeypatch):
    """32 crashed writes in one wave fit its stash (decided in place); 40 do
    not (kSumOvf: handed to the gap tier).  Both valid, certified, and the
    same on both paths."""
    rng = np.random.default_rng(5)
    base, boff, _, _ = abi.synth(4, 1000, concurrency=20, seed=72)
    keys = [base[boff[k]:boff[k + 1]].tolist() for k in range(4)]
    mod = [crash_in_wave0(keys[0], 32, rng), crash_in_wave0(keys[1], 40, rng),
           crash_in_wave0(keys[2], 20, rng), keys[3]]
    ops, off = pack_keys(mod)
    r, wit, kind = both_paths(ctx, monkeypatch, ops, off)
    assert (r["verdict"] == 1).all(), r["verdict"].tolist()
    certify(ops, off, r, wit, kind)


@pytest.mark.parametrize("seed", [81, 82])
def test_crash_light_claims_vs_oracle(ctx, monkeypatch, seed):
    """Crash-light keys with two mutations on one version (the lost-CAS
    shape) and injected value anomalies: value claims on held and unheld
    positions, duplicates found by the hole count.  Verdicts and fail ops
    equal the oracle's; valid keys' witnesses certified."""
    base, boff, _, _ = abi.synth(400, 160, concurrency=8, p_info=0.08, p_anomaly=0.3, seed=seed)
    keys = dup_versions([base[boff[k]:boff[k + 1]].tolist() for k in range(400)], seed, frac=0.3)
    ops, off = pack_keys(keys)
    r, wit, kind = both_paths(ctx, monkeypatch, ops, off)
    _, o = oracle.check(ops, off, algo=oracle.JIT)
    done = o["verdict"] != -1
    assert done.sum() > 350
    assert (r["verdict"][done] == o["verdict"][done]).all()
    assert (r["fail_op"][done] == o["fail_op"][done]).all()
    assert (r["verdict"] == 0).any() and (r["verdict"] == 1).any()
    certify(ops, off, r, wit, kind)
