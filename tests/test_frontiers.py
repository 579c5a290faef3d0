"""knossos's :configs for many invalid keys in one device call
(lc_check_frontiers, include/lincheck_fx.h, ABI 4), against the oracle's JITC
frontier just before each failing return (oracle.frontier, the restatement
of knossos.linear with the GPU's exact reductions) and against the frontier
exchange's one-key search (lc_fx_frontier)."""
import numpy as np
import pytest

import oracle
from helpers import pack_keys
from jepsen.etcd_amd import abi

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = abi.Context(device_mask=1)
    yield c
    c.close()


def _check(ctx, ops, off, max_per_key=10, min_ok=1):
    _, ref = oracle.check(ops, off, algo=oracle.JITC)
    inv = np.nonzero(ref["verdict"] == 0)[0]
    assert len(inv) >= min_ok
    parts = [ops[off[i]:off[i + 1]] for i in inv]
    sub = np.zeros(len(inv) + 1, dtype=np.int64)
    sub[1:] = np.cumsum([len(p) for p in parts])
    got = ctx.check_frontiers(np.concatenate(parts), sub, ref["fail_op"][inv], max_per_key)
    n_done = 0
    for j, i in enumerate(inv):
        if got[j] is None:
            # left to lc_fx_frontier only when the LDS tier cannot hold the
            # key's search: a frontier beyond its 128 configurations
            assert ref["max_frontier"][i] > 128, (int(i), int(ref["max_frontier"][i]))
            continue
        want, n_want = oracle.frontier(parts[j], int(ref["fail_op"][i]))
        assert len(got[j]) == min(max_per_key, n_want), (i, len(got[j]), n_want)
        for c in got[j]:
            assert c in want, (i, c)
        assert len(set(got[j])) == len(got[j])
        n_done += 1
    return n_done, len(inv)


def test_frontiers_c5(ctx):
    """C5: every invalid version-pinned key's frontier from the one call."""
    ops, off, _, _ = abi.synth(1000, 200, concurrency=10, p_anomaly=0.1, seed=0x5EED0005)
    n_done, n_inv = _check(ctx, ops, off, min_ok=50)
    assert n_done == n_inv


def test_frontiers_crashes_and_version_less(ctx):
    """Keys with crashed ops (frontiers of several configurations) and keys
    without versions (the cas-register model's shapes), max 1 and 10."""
    ops, off, _, _ = abi.synth(300, 150, concurrency=10, p_info=0.1, p_anomaly=0.5, seed=41)
    n_done, n_inv = _check(ctx, ops, off, min_ok=30)
    assert n_done >= n_inv * 0.7
    ops2 = ops.copy()
    ops2[:, 3] = abi.LC_NIL
    for mx in (1, 10):
        n_done, n_inv = _check(ctx, ops2, off, max_per_key=mx, min_ok=10)
        assert n_done >= n_inv * 0.3


def test_frontiers_equal_frontier_exchange(ctx):
    """The same number of configurations as lc_fx_frontier, each in the
    oracle's frontier; a stop op whose return is a no-op gives 0, a bad stop
    op -1 (None)."""
    from jepsen.etcd_amd.fx import FrontierExchange
    ops, off, _, _ = abi.synth(100, 120, concurrency=8, p_info=0.05, p_anomaly=1.0, seed=43)
    _, ref = oracle.check(ops, off, algo=oracle.JITC)
    inv = [int(i) for i in np.nonzero(ref["verdict"] == 0)[0]][:40]
    parts = [ops[off[i]:off[i + 1]] for i in inv]
    sub = np.zeros(len(inv) + 1, dtype=np.int64)
    sub[1:] = np.cumsum([len(p) for p in parts])
    got = ctx.check_frontiers(np.concatenate(parts), sub, ref["fail_op"][inv], 10)
    with FrontierExchange(device=0) as fx:
        for j, i in enumerate(inv):
            want = fx.frontier(parts[j], int(ref["fail_op"][i]), 10)
            if got[j] is not None:
                assert len(got[j]) == len(want), i
    # a read that returns with nothing pending (retired) and a bad stop op
    W, R = 1, 0
    keys = [[[W, 1, -1, 1, 0, 1], [R, 1, -1, 1, 2, 3]], [[W, 1, -1, 1, 0, 1]]]
    o, f = pack_keys(keys)
    got = ctx.check_frontiers(o, f, np.array([1, 5]), 10)
    assert got[1] is None and got[0] is not None and len(got[0]) <= 1
