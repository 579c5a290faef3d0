"""Host logic without a GPU: generator, Jepsen history preprocessing,
partitioning, and the C ABI's exported symbols."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle
from helpers import load_kats, pack_keys
from jepsen.etcd_amd import abi, history as H, synth
from jepsen.etcd_amd.history import Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(abi.LIB_PATH)
    names = []
    for h in ("lincheck.h", "lincheck_synth.h", "lincheck_edn.h", "lincheck_fx.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        names += re.findall(r"^\s*(?:const\s+)?\w+\s+\**(lc_\w+)\s*\(", src, re.M)
    assert set(names) == {
        "lc_open", "lc_check", "lc_check_device", "lc_last_stats", "lc_last_error",
        "lc_pack32", "lc_check32", "lc_check_device32", "lc_last_call_profile",
        "lc_check_frontiers", "lc_edn_ops32", "lc_edn_key_base", "lc_last_totals", "lc_quiesce",
        "lc_pack16", "lc_check16", "lc_edn_ops16",
        "lc_last_device_stats", "lc_host_register", "lc_host_unregister",
        "lc_close", "lc_default_opts", "lc_plan_partition", "lc_abi_version",
        "lc_check_ex", "lc_check_device_ex", "lc_key_cost", "lc_build_id",
        "lc_synth_register", "lc_synth_key", "lc_edn_parse", "lc_edn_n_keys", "lc_edn_n_ops",
        "lc_edn_n_events", "lc_edn_ops", "lc_edn_key_off", "lc_edn_key", "lc_edn_op_text",
        "lc_edn_value", "lc_edn_free", "lc_fx_open", "lc_fx_check", "lc_fx_last_stats",
        "lc_fx_last_error", "lc_fx_close", "lc_fx_open_devices", "lc_fx_rccl_unique_id",
        "lc_fx_open_rccl", "lc_fx_abort", "lc_fx_frontier"}
    for n in names:
        assert hasattr(lib, n), n
    assert abi.lib().lc_abi_version() == 5


def test_struct_sizes():
    assert abi.RESULT_DTYPE.itemsize == 40
    assert ctypes.sizeof(abi.LcOpts) == 40
    assert ctypes.sizeof(abi.LcSynthParams) == 56
    assert ctypes.sizeof(abi.LcStats) == 104
    assert ctypes.sizeof(abi.LcAux) == 32
    assert ctypes.sizeof(abi.LcDeviceStats) == 56
    assert ctypes.sizeof(abi.LcCallProfile) == 88
    assert ctypes.sizeof(abi.LcTotals) == 32
    from jepsen.etcd_amd import fx
    assert ctypes.sizeof(fx.LcFxParams) == 40
    assert ctypes.sizeof(fx.LcFxTransport) == 40
    assert ctypes.sizeof(fx.LcFxStats) == 80


def test_library_built_from_this_tree():
    """lc_build_id() names the sources the loaded library was built from;
    abi.lib() refuses a library whose id differs from this tree's (tests,
    smoke() and bench.py can never run a stale binary)."""
    built = abi.lib().lc_build_id().decode()
    assert built == abi.source_build_id() and len(built) == 16


def test_open_without_gpu_fails_loudly():
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("GPU present")
    with pytest.raises(abi.LcError):
        abi.Context(0)
    from jepsen.etcd_amd import fx
    with pytest.raises(abi.LcError):
        fx.FrontierExchange(device=0)


def test_synth_deterministic_and_exact():
    a = abi.synth(50, 300, concurrency=20, seed=42, n_threads=1)
    b = abi.synth(50, 300, concurrency=20, seed=42, n_threads=8)
    assert (a[0] == b[0]).all() and (a[1] == b[1]).all()
    ops, off = a[0], a[1]
    assert off[-1] == 50 * 300 and (np.diff(off) == 300).all()
    # per key: calls strictly increasing, ret > call, fields in range
    for k in range(50):
        r = ops[off[k]:off[k + 1]]
        assert (np.diff(r[:, 4]) > 0).all() and (r[:, 5] > r[:, 4]).all()
        assert set(np.unique(r[:, 0])) <= {0, 1, 2}
    c = abi.synth(50, 300, concurrency=20, seed=43)
    assert not (a[0] == c[0]).all()


def test_synth_clean_keys_valid_anomalies_invalid():
    ops, off, lab, ninv = abi.synth(300, 200, concurrency=10, p_anomaly=0.3, seed=5)
    assert ninv > len(ops)  # failed CAS invocations were dropped
    _, r = oracle.check(ops, off, algo=oracle.JITC, n_threads=4)
    assert (r["verdict"][lab == 0] == 1).all()
    assert (r["verdict"][lab == 1] == 0).all()          # stale read: always visible
    assert (r["verdict"][lab == 2] == 0).mean() > 0.8   # lost CAS: unless nothing follows it
    assert (lab > 0).sum() > 30


def test_history_pairing_kat8_fail_dropped():
    # KAT8 as a Jepsen history: a :fail CAS between the write and the read.
    h = [
        {"type": "invoke", "f": "write", "process": 0, "value": Tuple("k", [None, 1])},
        {"type": "ok", "f": "write", "process": 0, "value": Tuple("k", [1, 1])},
        {"type": "invoke", "f": "cas", "process": 1, "value": Tuple("k", [None, [3, 4]])},
        {"type": "fail", "f": "cas", "process": 1, "value": Tuple("k", [None, [3, 4]])},
        {"type": "invoke", "f": "read", "process": 0, "value": Tuple("k", [None, None])},
        {"type": "ok", "f": "read", "process": 0, "value": Tuple("k", [1, 1])},
    ]
    keys, ops, off, done = H.pack(h)
    assert keys == ["k"] and len(ops) == 2
    assert ops[0].tolist() == [1, 0, -1, 1, 0, 1]       # value 1 interned as id 0
    assert ops[1].tolist() == [0, 0, -1, 1, 4, 5]


def test_history_info_nemesis_and_nontuple():
    h = [
        {"type": "invoke", "f": "write", "process": 0, "value": Tuple(1, [None, 7])},
        {"type": "info", "f": "start", "process": "nemesis", "value": None},
        {"type": "info", "f": "write", "process": 0, "value": Tuple(1, [None, 7])},
        {"type": "invoke", "f": "cas", "process": 5, "value": Tuple(2, [None, [None, 3]])},
        {"type": "ok", "f": "cas", "process": 5, "value": Tuple(2, [1, [None, 3]])},
        {"type": "invoke", "f": "read", "process": 6, "value": Tuple(1, [None, None])},
    ]
    keys, ops, off, done = H.pack(h)
    assert keys == [1, 2]
    k1 = ops[off[0]:off[1]].tolist()
    assert k1[0] == [1, 0, -1, -1, 0, abi.LC_INF]       # crashed write
    assert k1[1] == [0, -1, -1, -1, 5, abi.LC_INF]      # unterminated read
    k2 = ops[off[1]:off[2]].tolist()
    assert k2 == [[2, 0, -1, 1, 3, 4]]                  # cas nil->3, version 1


def test_history_unknown_f_and_bad_value():
    h = [
        {"type": "invoke", "f": "frob", "process": 0, "value": Tuple("a", [None, 1])},
        {"type": "ok", "f": "frob", "process": 0, "value": Tuple("a", [1, 1])},
        {"type": "invoke", "f": "cas", "process": 1, "value": Tuple("b", [None, 3])},
        {"type": "ok", "f": "cas", "process": 1, "value": Tuple("b", [1, 3])},
    ]
    _, ops, off, _ = H.pack(h)
    assert ops[0, 0] == H.F_UNKNOWN and ops[1, 0] == H.F_UNKNOWN


def test_interning_distinguishes_types():
    it = H.Interner()
    assert it(1) == it(1) and it(1) != it(1.0) and it(True) != it(1)
    assert it(None) == abi.LC_NIL


def test_jepsen_history_roundtrip_matches_packed_generator():
    """Rendering generator keys as one Jepsen history (fails, nemesis ops,
    interleaving) and re-packing gives the same verdicts as the packed
    generator output."""
    hist, labels = synth.jepsen_history(40, 150, concurrency=10, p_info=0.05,
                                        p_anomaly=0.3, seed=77)
    keys, ops, off, done = H.pack(hist)
    assert keys == list(range(40))
    ref_ops = []
    for k in range(40):
        o, p, st, _ = abi.synth_key(k, 150, 10, 5, 0.05, 0.3, 77)
        ref_ops.append(o[st != 0])
    ref, ref_off = pack_keys([r.tolist() for r in ref_ops])
    _, a = oracle.check(ops, off, algo=oracle.JITC)
    _, b = oracle.check(ref, ref_off, algo=oracle.JITC)
    assert (a["verdict"] == b["verdict"]).all() and (a["fail_op"] == b["fail_op"]).all()
    assert (a["verdict"][np.array(labels) == 0] == 1).all()
    assert (a["verdict"][np.array(labels) == 1] == 0).all()


def test_plan_partition_balanced_and_contiguous():
    off = np.concatenate([[0], np.cumsum(np.random.RandomState(0).randint(0, 500, 1000))])
    for parts in (1, 2, 3, 8):
        b = abi.plan_partition(off, parts)
        assert b[0] == 0 and b[-1] == 1000 and (np.diff(b) >= 0).all()
        cost = [(off[b[i + 1]] - off[b[i]]) + 64 * (b[i + 1] - b[i]) for i in range(parts)]
        assert max(cost) - min(cost) <= 2 * (500 + 64)  # one key per boundary


def test_key_cost_follows_the_tier():
    """lc_key_cost prices a key by the tier that will decide it: version-
    pinned clean keys by their records, crash-heavy keys (gap tier) several
    times more, version-less keys (frontier search) far more."""
    clean, off, _, _ = abi.synth(4, 200, concurrency=10, seed=1)
    crash, _, _, _ = abi.synth(4, 200, concurrency=10, p_info=0.2, seed=1)
    nover = clean.copy()
    nover[:, 3] = -1
    c = [abi.key_cost(x, off) for x in (clean, crash, nover)]
    assert np.allclose(c[0], 200 + 64)
    assert (c[1] > 4 * c[0]).all() and (c[2] > 20 * c[1]).all()


def test_plan_partition_is_crash_aware():
    """A batch whose crash-heavy keys are clustered at the front: splitting by
    records would give the first device all of them; the cost-aware split
    gives it fewer keys, and every part's cost is within one key of equal."""
    heavy, hoff, _, _ = abi.synth(250, 400, concurrency=20, p_info=0.2, seed=2)
    light, loff, _, _ = abi.synth(750, 400, concurrency=20, seed=3)
    ops = np.concatenate([heavy, light])
    off = np.concatenate([hoff, loff[1:] + hoff[-1]])
    cost = abi.key_cost(ops, off)
    for parts in (2, 4, 8):
        b = abi.plan_partition(off, parts, ops=ops)
        assert b[0] == 0 and b[-1] == 1000 and (np.diff(b) >= 0).all()
        per = [cost[b[i]:b[i + 1]].sum() for i in range(parts)]
        assert max(per) - min(per) <= 2 * cost.max()
        naive = abi.plan_partition(off, parts)
        assert b[1] < naive[1]  # fewer of the clustered heavy keys on device 0
    assert abi.plan_partition(off, 2, ops=ops)[1] < 250


def test_kat_file_consistent():
    for k in load_kats():
        assert k["fail_prefix_end"] == (k["ops"][k["fail_op"]][5] if k["fail_op"] >= 0 else -1)


def test_timeline_render():
    """The :timeline half of register.clj:112 (host-side renderer): one box
    per client op, spanning invoke..completion, classed by completion type;
    the counterexample op outlined, later ops dimmed; text escaped."""
    from jepsen.etcd_amd import timeline as TL
    T = H.tuple_
    hist = [
        {"type": "invoke", "process": 0, "f": "write", "value": T(1, [None, 1])},
        {"type": "ok", "process": 0, "f": "write", "value": T(1, [1, 1])},
        {"type": "invoke", "process": 1, "f": "read", "value": T(1, [None, None])},
        {"type": "invoke", "process": "nemesis", "f": "kill", "value": None},
        {"type": "ok", "process": 1, "f": "read", "value": T(1, [1, "<b>"])},
        {"type": "invoke", "process": 2, "f": "cas", "value": T(1, [None, [1, 2]])},
        {"type": "info", "process": 2, "f": "cas", "value": T(1, [None, [1, 2]])},
        {"type": "invoke", "process": 0, "f": "read", "value": T(1, [None, None])},
    ]
    sub = H.split_by_key(H.index_history(hist))[1]
    ps = TL.pairs(sub)
    assert [(i["index"], c["index"] if c else None) for i, c in ps] == \
        [(0, 1), (2, 4), (5, 6), (7, None)]
    page = TL.render(sub, title="key 1", cex_index=4)
    assert page.count('class="op ') == 4
    assert 'class="op ok cex"' in page and 'class="op info after"' in page
    assert 'class="op invoke after"' in page
    assert "&lt;b&gt;" in page and "<b>" not in page.split("<body>")[1]
    assert ">0<" in page and ">2<" in page and "nemesis" not in page
