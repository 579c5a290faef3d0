"""The 24-byte record path (ABI 4: lc_op32, lc_pack32, lc_check32,
lc_check_device32, include/lincheck.h).

CPU: lc_pack32 narrows each record so that the lc_op it stands for decodes,
by the device's own rules (a restatement of csrc/records.h `decode` below),
to exactly what the 48-byte record decodes to — on every record of the
golden fixtures and on random records with every field out of range.

GPU: lc_check32(lc_pack32(x)) returns what lc_check(x) returns, field for
field, witnesses and certificates included: C1, C5, the crash-heavy and
tiny fixtures, C4-shaped keys, a batch with crashes, the malformed-key
batches of test_gpu.py / test_gpu_witness.py, random garbage keys, and the
device-resident form lc_check_device32.  (The widened records are the
originals for every well-formed record, so every tier sees the same input.)
"""
import os

import numpy as np
import pytest

from helpers import GOLDEN, INF, pack_keys
from jepsen.etcd_amd import abi

K_FIELD_MAX = 0x7FFFFFFE
K_NEVER = 0xFFFFFFFF


def decode(rec, base):
    """csrc/records.h decode() of one 48-byte record (key's first call =
    base): (padding, bad, f, val, exp, ver, call, ret) as the device holds
    them (call / ret key-relative uint32)."""
    f, value, expected, version, call, ret = (int(x) for x in rec)
    if call == -1 and ret == -1:
        return ("pad",)
    rc, rr = call - base, ret - base
    bad = (value < -1 or value > K_FIELD_MAX or expected < -1 or expected > K_FIELD_MAX
           or call < 0 or ret <= call or rc < 0 or rc >= K_NEVER
           or (ret != INF and rr >= K_NEVER))
    fm = f if 0 <= f <= 2 else 3
    ver = K_FIELD_MAX if (version < -1 or version > K_FIELD_MAX) else version
    c32 = rc & 0xFFFFFFFF
    r32 = K_NEVER if ret == INF else rr & 0xFFFFFFFF
    if bad:  # the device reads nothing else of a malformed record
        return ("bad", c32)
    return ("ok", fm, value, expected, ver, c32, r32)


def widen(r32, base):
    """The lc_op an lc_op32 record stands for (include/lincheck.h)."""
    f, value, expected, version = (int(np.int32(x)) for x in r32[:4])
    call, ret = int(np.uint32(r32[4])), int(np.uint32(r32[5]))
    return [f, value, expected, version, base + call, INF if ret == K_NEVER else base + ret]


def same_decoding(ops, off):
    o32, base = abi.pack32(ops, off)
    o32u = o32.view(np.uint32)
    for k in range(len(off) - 1):
        a, b = int(off[k]), int(off[k + 1])
        if a == b:
            continue
        b48 = int(ops[a][4])
        w = [widen(o32u[i], int(base[k])) for i in range(a, b)]
        b32 = w[0][4]
        for i in range(a, b):
            d48 = decode(ops[i], b48)
            d32 = decode(w[i - a], b32)
            if d48 == ("pad",):
                continue  # (documented: an index no history has; the device's padding marker)
            assert d48 == d32, (k, i, ops[i].tolist(), o32[i].tolist(), d48, d32)
    return o32, base


@pytest.mark.parametrize("name", ["c1", "c5", "info", "tiny"])
def test_pack32_golden_fixtures_widen_exactly(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    ops, off = z["ops"], z["key_off"]
    o32, base = same_decoding(ops, off)
    # well-formed records come back exactly
    o32u = o32.view(np.uint32)
    for k in range(0, len(off) - 1, max(1, (len(off) - 1) // 50)):
        for i in range(int(off[k]), int(off[k + 1])):
            assert widen(o32u[i], int(base[k])) == ops[i].tolist()


def test_pack32_out_of_range_fields():
    """Every field out of range, alone and together: the narrowed record
    decodes as the 48-byte one does (malformed stays malformed, unreachable
    versions stay unreachable, unknown :f stays unknown)."""
    rng = np.random.default_rng(5)
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
                r[j] = int(rng.choice(specials))
            recs.append(r)
        keys.append(recs)
    ops, off = pack_keys(keys)
    same_decoding(ops, off)


def test_pack32_rejects_bad_offsets():
    ops, off = pack_keys([[[1, 1, -1, 1, 0, 1]]])
    with pytest.raises(abi.LcError):
        abi.pack32(ops, np.array([0, 2, 1], dtype=np.int64))


# ---------------------------------------------------------------- GPU parity


def _both(ctx, ops, off, **kw):
    o32, base = abi.pack32(ops, off)
    a = ctx.check(ops, off, raise_on_error=False, witness=True, certificate=True, **kw)
    b = ctx.check32(o32, off, base, raise_on_error=False, witness=True, certificate=True, **kw)
    return a, b


def _assert_same(a, b, what):
    ra, rb = a[1], b[1]
    assert a[0] == b[0], what
    bad = np.nonzero(ra != rb)[0]
    assert len(bad) == 0, (what, [(int(k), ra[k].tolist(), rb[k].tolist()) for k in bad[:5]])
    for i, name in ((2, "witness"), (3, "kind"), (4, "certificate"), (5, "certificate_set")):
        x, y = np.asarray(a[i]), np.asarray(b[i])
        diff = np.nonzero((x != y).reshape(len(x), -1).any(axis=1))[0]
        assert len(diff) == 0, (what, name, diff[:5].tolist())


@pytest.fixture(scope="module")
def ctx():
    c = abi.Context(device_mask=1)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c1", "c5", "info", "tiny"])
def test_check32_golden_fixtures(ctx, name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    a, b = _both(ctx, z["ops"], z["key_off"])
    _assert_same(a, b, name)
    assert (b[1]["verdict"] == z["verdict"]).all() and (b[1]["fail_op"] == z["fail_op"]).all()


@pytest.mark.gpu
def test_check32_batches(ctx):
    """Synthetic batches through every tier: C5-shaped invalid keys, crash
    batches (the fused pass from the second call, the crash-light pass, the
    gap tier), C4-shaped long crash-heavy keys (multisection
    counterexamples), version-less keys (the frontier search)."""
    cases = [
        ("c5", abi.synth(1000, 200, concurrency=10, p_anomaly=0.1, seed=0x5EED0005)),
        ("crash", abi.synth(2000, 300, concurrency=20, p_info=0.05, seed=12)),
        ("crash-invalid", abi.synth(500, 300, concurrency=20, p_info=0.1, p_anomaly=0.5, seed=13)),
        ("c4", abi.synth(2, 5000, concurrency=50, p_info=0.2, info_frac=0.2, p_anomaly=1.0,
                         seed=1007)),
    ]
    for name, (ops, off, _, _) in cases:
        for _ in range(2):  # the second call of a crash batch takes the fused pass
            a, b = _both(ctx, ops, off)
            _assert_same(a, b, name)
    ops, off, _, _ = abi.synth(200, 150, concurrency=8, p_info=0.02, p_anomaly=0.3, seed=14)
    ops = ops.copy()
    ops[:, 3] = abi.LC_NIL
    a, b = _both(ctx, ops, off)
    _assert_same(a, b, "version-less")


@pytest.mark.gpu
def test_check32_malformed_keys(ctx):
    """The malformed-key batches of test_gpu.py / test_gpu_witness.py and
    random keys with out-of-range fields: the same verdicts, reasons and
    fail ops (and malformed counts) through both widths."""
    W, R = 1, 0
    keys = [
        [[W, 1, -1, 1, 5, 6], [W, 2, -1, 2, 3, 4]],            # calls out of order
        [[1, 1, -1, 1, 5, 5]],                                  # ret <= call
        [[1, 1 << 40, -1, 1, 0, 1]],                            # value beyond int32
        [[7, 1, -1, 1, 0, 1]],                                  # unknown :f
        [[W, 1, -1, 1, 0, 1], [W, 2, -1, 2, 2, 3], [R, 1, -1, 1, 4, 5]],   # stale read
        [[W, 1, -1, 1, 0, 1], [R, 1, -1, 1 << 40, 2, 3]],       # unreachable version
        [[W, 1, -1, -7, 0, 1]],
        [[W, 1, -1, 1 << 40, 0, INF], [W, 2, -1, 1, 1, 2]],
        [[W, 1, -1, 1, 0, 1], [W, 2, -1, 2, 1 << 33, (1 << 33) + 1]],   # span beyond 2^32
        [[W, 1, -1, 1, 0, 1]],
    ]
    ops, off = pack_keys(keys)
    a, b = _both(ctx, ops, off)
    _assert_same(a, b, "malformed")
    na = ctx.stats()["n_malformed"]
    assert na >= 3
    rng = np.random.default_rng(9)
    specials = [-(1 << 40), -3, -2, 3, 7, K_FIELD_MAX, K_FIELD_MAX + 1, 1 << 32, INF]
    keys = []
    for _ in range(600):
        n = int(rng.integers(1, 10))
        call, recs, ver = int(rng.integers(0, 3)), [], 0
        for _ in range(n):
            call += 1 if rng.random() < 0.9 else int(rng.choice([1 << 32, -2]))
            f = int(rng.integers(0, 3))
            if f != R:
                ver += 1
            r = [f, int(rng.integers(-1, 3)), int(rng.integers(-1, 3)) if f == 2 else -1,
                 ver if f != R else int(rng.integers(-1, ver + 1)), call,
                 INF if (f != R and rng.random() < 0.15) else call + int(rng.integers(1, 4))]
            if rng.random() < 0.1:
                r[int(rng.integers(0, 6))] = int(rng.choice(specials))
            recs.append(r)
        keys.append(recs)
    ops, off = pack_keys(keys)
    a, b = _both(ctx, ops, off)
    _assert_same(a, b, "random out-of-range keys")


@pytest.mark.gpu
def test_check_device32_equals_check_device(ctx):
    import torch
    dev = torch.device("cuda", 0)
    ops, off, _, _ = abi.synth(1000, 200, concurrency=10, p_anomaly=0.1, p_info=0.02,
                               seed=0x5EED0015)
    o32, base = abi.pack32(ops, off)
    s = torch.cuda.current_stream(dev)
    # a slice of keys whose key_off does not start at 0
    a, b = 100, 900
    d48 = torch.from_numpy(np.ascontiguousarray(ops[off[a]:off[b]])).to(dev)
    d32 = torch.from_numpy(np.ascontiguousarray(o32[off[a]:off[b]])).to(dev)
    d_off = torch.from_numpy(np.ascontiguousarray(off[a:b + 1])).to(dev)
    d_base = torch.from_numpy(np.ascontiguousarray(base[a:b])).to(dev)
    outs = []
    for fn in ("48", "32"):
        d_out = torch.zeros((b - a) * 40, dtype=torch.uint8, device=dev)
        if fn == "48":
            ctx.check_device(d48.data_ptr(), d_off.data_ptr(), b - a, d_out.data_ptr(),
                             stream=s.cuda_stream)
        else:
            ctx.check_device32(d32.data_ptr(), d_off.data_ptr(), d_base.data_ptr(), b - a,
                               d_out.data_ptr(), stream=s.cuda_stream)
        outs.append(np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE))
    assert (outs[0] == outs[1]).all()
    assert (outs[1]["verdict"] == 0).any()


@pytest.mark.gpu
def test_check32_fan_out_over_devices(monkeypatch):
    """The fan-out over several device contexts (LC_VIRTUAL_DEVICES) with
    24-byte records and chunked copies: equal to the one-device 48-byte call,
    chunks counted in the call profile."""
    ops, off, _, _ = abi.synth(3000, 1000, concurrency=20, p_info=0.01, p_anomaly=0.05, seed=31)
    o32, base = abi.pack32(ops, off)
    with abi.Context(device_mask=1) as c1:
        _, want = c1.check(ops, off)
    monkeypatch.setenv("LC_VIRTUAL_DEVICES", "3")
    with abi.Context(device_mask=1) as c3:
        _, got = c3.check32(o32, off, base)
        prof = c3.call_profile()
        _, got48 = c3.check(ops, off)
    assert (got == want).all() and (got48 == want).all()
    assert prof["n_devices"] == 3 and prof["n_chunks"] >= 3
    assert prof["last_end_ms"] <= prof["joined_ms"] <= prof["total_ms"]


@pytest.mark.gpu
def test_check32_native_pass_equals_check(ctx):
    """Without lc_aux outputs lc_check32 decides the 24-byte records as they
    are (fast_tier32_kernel / fused_tier32_kernel), widening them only when a
    key is handed over: every result field equals lc_check's on the golden
    fixtures, batches through every tier (clean, crash-light via both passes,
    invalid, C4-long, version-less) and the malformed keys."""
    batches = []
    for name in ("c1", "c5", "info", "tiny"):
        z = np.load(os.path.join(GOLDEN, name + ".npz"))
        batches.append((name, z["ops"], z["key_off"]))
    for name, kw in (("clean", dict(n_keys=2000, ops_per_key=400, concurrency=20, seed=21)),
                     ("c5", dict(n_keys=1000, ops_per_key=200, concurrency=10, p_anomaly=0.1,
                                 seed=0x5EED0005)),
                     ("crash", dict(n_keys=2000, ops_per_key=300, concurrency=20, p_info=0.05, seed=12)),
                     ("c4", dict(n_keys=2, ops_per_key=5000, concurrency=50, p_info=0.2,
                                 info_frac=0.2, p_anomaly=1.0, seed=1007))):
        kw = dict(kw)
        ops, off, _, _ = abi.synth(kw.pop("n_keys"), kw.pop("ops_per_key"), **kw)
        batches.append((name, ops, off))
    ops, off, _, _ = abi.synth(200, 150, concurrency=8, p_info=0.02, p_anomaly=0.3, seed=14)
    ops = ops.copy()
    ops[:, 3] = abi.LC_NIL
    batches.append(("version-less", ops, off))
    W, R = 1, 0
    ops, off = pack_keys([[[W, 1, -1, 1, 5, 6], [W, 2, -1, 2, 3, 4]], [[1, 1, -1, 1, 5, 5]],
                          [[1, 1 << 40, -1, 1, 0, 1]], [[7, 1, -1, 1, 0, 1]],
                          [[W, 1, -1, 1, 0, 1], [W, 2, -1, 2, 2, 3], [R, 1, -1, 1, 4, 5]],
                          [[W, 1, -1, 1, 0, 1], [R, 1, -1, 1 << 40, 2, 3]], [[W, 1, -1, -7, 0, 1]],
                          [[W, 1, -1, 1, 0, 1], [W, 2, -1, 2, 1 << 33, (1 << 33) + 1]],
                          [[W, 1, -1, 1, 0, 1]]])
    batches.append(("malformed", ops, off))
    for name, ops, off in batches:
        o32, base = abi.pack32(ops, off)
        for _ in range(2):  # a crash batch's second call takes the fused pass
            _, want = ctx.check(ops, off, raise_on_error=False)
            _, got = ctx.check32(o32, off, base, raise_on_error=False)
            bad = np.nonzero(want != got)[0]
            assert len(bad) == 0, (name, [(int(k), want[k].tolist(), got[k].tolist()) for k in bad[:5]])
