"""The 16-byte record path (round 6: lc_op16, lc_pack16, lc_check16,
include/lincheck.h): f plus 15-bit value and expected ids in one word, then
the version and the key-relative call and return.

CPU: lc_pack16's records, unpacked by the header's rule, are lc_pack32's
records for every record that is not malformed, and a malformed record stays
malformed (the device reads nothing else of a malformed key); a batch with
an id above LC_ID15_MAX is refused (it goes as lc_op32).

GPU: lc_check16(lc_pack16(x)) returns what lc_check(x) returns, field for
field, witnesses and certificates included, on the golden fixtures, batches
through every tier, the malformed-key batches, and the multi-device fan-out.
"""
import os

import numpy as np
import pytest

from helpers import GOLDEN, INF, pack_keys
from jepsen.etcd_amd import abi
from test_op32 import K_FIELD_MAX, decode, widen

MARK = 0x7FFF


def unpack16(q):
    """The lc_op32 an lc_op16 record stands for (include/lincheck.h)."""
    fve, ver, call, ret = (int(x) for x in q)
    v, x = (fve >> 15) & 0x7FFF, fve & 0x7FFF
    return [fve >> 30, -2 if v == MARK else v - 1, -2 if x == MARK else x - 1,
            int(np.int32(np.uint32(ver))), call, ret]


def same_as_pack32(ops, off):
    got = abi.pack16(ops, off)
    assert got is not None
    o16, base16 = got
    o32, base32 = abi.pack32(ops, off)
    assert (base16 == base32).all()
    o32u = o32.view(np.uint32)
    for k in range(len(off) - 1):
        a, b = int(off[k]), int(off[k + 1])
        for i in range(a, b):
            r16 = unpack16(o16[i])
            r32 = [int(np.int32(o32u[i][j])) for j in range(4)] + [int(o32u[i][4]), int(o32u[i][5])]
            if r32[1] == -2:  # malformed (value -2): stays malformed, whatever else it holds
                assert r16[1] == -2, (k, i)
                assert decode(widen(o32u[i], int(base32[k])), int(base32[k]))[0] == "bad"
                continue
            assert r16 == r32, (k, i, ops[i].tolist(), r16, r32)
    return o16, base16


@pytest.mark.parametrize("name", ["c1", "c5", "info", "tiny"])
def test_pack16_golden_fixtures(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    same_as_pack32(z["ops"], z["key_off"])


def test_pack16_out_of_range_fields():
    """Every field out of range (ids within 15 bits where the record is well
    formed): the same narrowing as lc_pack32, malformed stays malformed."""
    rng = np.random.default_rng(6)
    specials = [-(1 << 40), -3, -2, -1, 0, 1, 2, 3, 7, K_FIELD_MAX - 1, K_FIELD_MAX,
                K_FIELD_MAX + 1, 1 << 31, 1 << 32, (1 << 40), INF]
    keys = []
    for _ in range(400):
        n = int(rng.integers(1, 8))
        call = int(rng.choice([0, 5, 1 << 33]))
        recs = []
        for _ in range(n):
            call += int(rng.choice([1, 2, 1 << 32, -3])) if rng.random() < 0.2 else 1
            ret = call + int(rng.integers(1, 6))
            r = [int(rng.integers(0, 3)), int(rng.integers(-1, 4)), -1, int(rng.integers(-1, 5)),
                 call, INF if rng.random() < 0.2 else ret]
            if rng.random() < 0.5:
                j = int(rng.integers(0, 6))
                v = int(rng.choice(specials))
                # a well-formed id stays within 15 bits (larger ones: next test)
                if j in (1, 2) and 0x7FFD < v <= K_FIELD_MAX:
                    v = 0x7FFD
                r[j] = v
            recs.append(r)
        keys.append(recs)
    ops, off = pack_keys(keys)
    same_as_pack32(ops, off)


def test_pack16_refuses_wide_ids():
    W, C = 1, 2
    ok = [[W, 0x7FFD, -1, 1, 0, 1], [C, 3, 0x7FFD, 2, 2, 3]]
    assert abi.pack16(*pack_keys([ok])) is not None
    assert abi.pack16(*pack_keys([ok, [[W, 0x7FFE, -1, 1, 0, 1]]])) is None
    assert abi.pack16(*pack_keys([[[C, 1, 0x7FFE, 1, 0, 1]]])) is None
    # a malformed record may hold any id: it is marked, not narrowed
    got = abi.pack16(*pack_keys([[[W, 1 << 40, -1, 1, 0, 1]]]))
    assert got is not None and (got[0][0][0] >> 15) & 0x7FFF == MARK


# ---------------------------------------------------------------- GPU parity


@pytest.fixture(scope="module")
def ctx():
    c = abi.Context(device_mask=1)
    yield c
    c.close()


def _assert_same16(ctx, ops, off, what):
    o16, base = abi.pack16(ops, off)
    a = ctx.check(ops, off, raise_on_error=False, witness=True, certificate=True)
    b = ctx.check16(o16, off, base, raise_on_error=False, witness=True, certificate=True)
    assert a[0] == b[0], what
    bad = np.nonzero(a[1] != b[1])[0]
    assert len(bad) == 0, (what, [(int(k), a[1][k].tolist(), b[1][k].tolist()) for k in bad[:5]])
    for i, name in ((2, "witness"), (3, "kind"), (4, "certificate"), (5, "certificate_set")):
        x, y = np.asarray(a[i]), np.asarray(b[i])
        diff = np.nonzero((x != y).reshape(len(x), -1).any(axis=1))[0]
        assert len(diff) == 0, (what, name, diff[:5].tolist())
    # and without lc_aux outputs
    _, want = ctx.check(ops, off, raise_on_error=False)
    _, got = ctx.check16(o16, off, base, raise_on_error=False)
    assert (want == got).all(), what
    return b


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1", "c5", "info", "tiny"])
def test_check16_golden_fixtures(ctx, name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    b = _assert_same16(ctx, z["ops"], z["key_off"], name)
    assert (b[1]["verdict"] == z["verdict"]).all() and (b[1]["fail_op"] == z["fail_op"]).all()


@pytest.mark.gpu
def test_check16_batches(ctx):
    cases = [
        ("c5", abi.synth(1000, 200, concurrency=10, p_anomaly=0.1, seed=0x5EED0005)),
        ("crash", abi.synth(2000, 300, concurrency=20, p_info=0.05, seed=12)),
        ("crash-invalid", abi.synth(500, 300, concurrency=20, p_info=0.1, p_anomaly=0.5, seed=13)),
        ("c4", abi.synth(2, 5000, concurrency=50, p_info=0.2, info_frac=0.2, p_anomaly=1.0,
                         seed=1007)),
    ]
    for name, (ops, off, _, _) in cases:
        for _ in range(2):
            _assert_same16(ctx, ops, off, name)
    ops, off, _, _ = abi.synth(200, 150, concurrency=8, p_info=0.02, p_anomaly=0.3, seed=14)
    ops = ops.copy()
    ops[:, 3] = abi.LC_NIL
    _assert_same16(ctx, ops, off, "version-less")


@pytest.mark.gpu
def test_check16_malformed_keys(ctx):
    W, R = 1, 0
    keys = [
        [[W, 1, -1, 1, 5, 6], [W, 2, -1, 2, 3, 4]],
        [[1, 1, -1, 1, 5, 5]],
        [[1, 1 << 40, -1, 1, 0, 1]],
        [[7, 1, -1, 1, 0, 1]],
        [[W, 1, -1, 1, 0, 1], [W, 2, -1, 2, 2, 3], [R, 1, -1, 1, 4, 5]],
        [[W, 1, -1, 1, 0, 1], [R, 1, -1, 1 << 40, 2, 3]],
        [[W, 1, -1, -7, 0, 1]],
        [[W, 1, -1, 1 << 40, 0, INF], [W, 2, -1, 1, 1, 2]],
        [[W, 1, -1, 1, 0, 1], [W, 2, -1, 2, 1 << 33, (1 << 33) + 1]],
        [[W, 1, -1, 1, 0, 1]],
    ]
    ops, off = pack_keys(keys)
    _assert_same16(ctx, ops, off, "malformed")
    assert ctx.stats()["n_malformed"] >= 3


@pytest.mark.gpu
def test_check16_fan_out_over_devices(monkeypatch):
    ops, off, _, _ = abi.synth(3000, 1000, concurrency=20, p_info=0.01, p_anomaly=0.05, seed=31)
    o16, base = abi.pack16(ops, off)
    with abi.Context(device_mask=1) as c1:
        _, want = c1.check(ops, off)
    monkeypatch.setenv("LC_VIRTUAL_DEVICES", "3")
    with abi.Context(device_mask=1) as c3:
        _, got = c3.check16(o16, off, base)
        prof = c3.call_profile()
    assert (got == want).all()
    assert prof["n_devices"] == 3 and prof["n_chunks"] >= 3
