"""The resident version-order grid (kernels.h launch_fast_resident): every
lc_check_device call it serves must return exactly what a launched pass
returns — over repeated calls, after the records are rewritten in place
between calls while the grid stays resident (no stale cache lines), across
idle exits and relaunches, and for batches with keys the pass hands over
(C5's invalid keys: the grid is stopped, the later tiers decide them)."""
import os
import time

import numpy as np
import pytest

from helpers import GOLDEN
from jepsen.etcd_amd import abi

pytestmark = pytest.mark.gpu

FIELDS = ("verdict", "reason", "fail_op", "fail_prefix_end", "configs_explored", "max_frontier")


def _dev(arr):
    import torch
    return torch.from_numpy(np.ascontiguousarray(arr)).to(torch.device("cuda", 0))


def _run(ctx, d_ops, d_off, n, flags=0):
    import torch
    d_out = torch.zeros(max(n, 1) * 40, dtype=torch.uint8, device=d_ops.device)
    s = torch.cuda.current_stream(d_ops.device)
    ctx.check_device(d_ops.data_ptr(), d_off.data_ptr(), n, d_out.data_ptr(), stream=s.cuda_stream,
                     opts=abi.default_opts(flags=flags))
    return np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)[:n].copy()


def _launched(ctx, d_ops, d_off, n, monkeypatch):
    monkeypatch.setenv("LC_RESIDENT", "0")
    r = _run(ctx, d_ops, d_off, n)
    monkeypatch.delenv("LC_RESIDENT")
    return r


@pytest.mark.parametrize("name", ["c5", "c1", "tiny", "info"])
def test_resident_equals_launched(ctx, name, monkeypatch):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    n = min(len(z["key_off"]) - 1, 1200)
    d_ops, d_off = _dev(z["ops"][:z["key_off"][n]]), _dev(z["key_off"][:n + 1])
    want = _launched(ctx, d_ops, d_off, n, monkeypatch)
    assert (want["verdict"] == z["verdict"][:n]).all()
    monkeypatch.setenv("LC_RESIDENT_IDLE_US", "200000")
    for flags in (0, abi.LC_FLAG_NO_TIMING, 0, 0):
        got = _run(ctx, d_ops, d_off, n, flags)
        for f in FIELDS:
            assert (got[f] == want[f]).all(), (name, f, np.nonzero(got[f] != want[f])[0][:5])


def test_resident_sees_records_rewritten_in_place(ctx, monkeypatch):
    """Two batches of the same shape copied in turn into the SAME device
    buffers while the grid stays resident (a long idle bound): each call's
    results follow the records the buffer holds now.  Batch B is batch A
    with stale reads injected, so a grid reading cached lines of A would
    report B's invalid keys valid."""
    import torch
    a_ops, a_off, _, _ = abi.synth(1000, 200, concurrency=10, seed=0x5EED0101)
    b_ops, b_off, lab, _ = abi.synth(1000, 200, concurrency=10, p_anomaly=0.3, seed=0x5EED0101)
    if a_ops.shape != b_ops.shape or (a_off != b_off).any():
        pytest.skip("synth shapes differ")
    da, db = _dev(a_ops), _dev(b_ops)
    d_ops, d_off = torch.empty_like(da), _dev(a_off)
    want = {}
    for tag, src in (("a", da), ("b", db)):
        d_ops.copy_(src)
        want[tag] = _launched(ctx, d_ops, d_off, 1000, monkeypatch)
    assert (want["a"]["verdict"] == 1).all() and (want["b"]["verdict"] == 0).sum() > 50
    monkeypatch.setenv("LC_RESIDENT_IDLE_US", "2000000")
    for i in range(12):
        tag = "ab"[i % 2]
        d_ops.copy_(da if tag == "a" else db)
        got = _run(ctx, d_ops, d_off, 1000)
        for f in FIELDS:
            assert (got[f] == want[tag][f]).all(), (i, tag, f)


def test_resident_idle_exit_and_relaunch(ctx, monkeypatch):
    """A short idle bound: the grid leaves between calls spaced wider than it
    and is launched again; batches of growing key counts relaunch it larger.
    Every call equals the launched pass."""
    z = np.load(os.path.join(GOLDEN, "c1.npz"))
    n_all = len(z["key_off"]) - 1
    d_ops, d_off = _dev(z["ops"]), _dev(z["key_off"])
    want = _launched(ctx, d_ops, d_off, n_all, monkeypatch)
    monkeypatch.setenv("LC_RESIDENT_IDLE_US", "20")
    for i, n in enumerate((10, 10, 50, 100, 100, 30)):
        got = _run(ctx, d_ops, d_off, n)
        for f in FIELDS:
            assert (got[f] == want[f][:n]).all(), (i, n, f)
        time.sleep(0.002 if i % 2 else 0.0)


def test_resident_totals_count_every_call(ctx, monkeypatch):
    """lc_last_totals: a call the grid serves is timed by the device clock,
    untimed flag or not."""
    import torch
    z = np.load(os.path.join(GOLDEN, "c1.npz"))
    n = len(z["key_off"]) - 1
    d_ops, d_off = _dev(z["ops"]), _dev(z["key_off"])
    out = torch.zeros(n * 40, dtype=torch.uint8, device=d_ops.device)
    s = torch.cuda.current_stream(d_ops.device)
    monkeypatch.setenv("LC_RESIDENT_IDLE_US", "200000")
    call = ctx.bind_check_device(d_ops.data_ptr(), d_off.data_ptr(), n, out.data_ptr(),
                                 stream=s.cuda_stream,
                                 opts=abi.default_opts(flags=abi.LC_FLAG_NO_TIMING))
    call()
    ctx.totals(reset=True)
    for _ in range(20):
        call()
    t = ctx.totals(reset=True)
    assert t["calls"] == 20 and t["timed_calls"] == 20
    assert 0 < t["fast_kernel_ms"] / 20 < 1.0


@pytest.mark.parametrize("resident", ["0", "1"])
def test_contexts_reopened_signal_path(monkeypatch, resident):
    """Contexts opened and closed in turn, one signal-path call each (the
    follower kernel's completion word, or the resident grid's), alternating a
    clean batch with one whose invalid keys must be handed over: pinned words
    reused from a closed context (h_done, h_handoff) must not let a
    call return before its pass, nor hide a handoff."""
    clean = abi.synth(300, 100, concurrency=8, seed=61)[:2]
    bad = abi.synth(300, 100, concurrency=8, p_anomaly=0.4, seed=62)[:2]
    with abi.Context(device_mask=1) as c0:
        want = [c0.check(o, f)[1] for o, f in (clean, bad)]
    assert (want[1]["verdict"] == 0).any() and (want[0]["verdict"] == 1).all()
    devs = [(_dev(o), _dev(f)) for o, f in (clean, bad)]
    monkeypatch.setenv("LC_RESIDENT", resident)
    for i in range(12):
        k = i % 2
        with abi.Context(device_mask=1) as ctx:
            got = _run(ctx, devs[k][0], devs[k][1], 300)
        for f in ("verdict", "reason", "fail_op", "fail_prefix_end"):
            assert (got[f] == want[k][f]).all(), (i, f)
