"""history.edn ingestion (include/lincheck_edn.h): the native reader must
build exactly the records history.py builds from the same ops (per-key split
of register.clj:108, knossos completion, interning), whatever the EDN
surface form.  Host code: CPU tests, plus one end-to-end GPU check."""
import os

import numpy as np
import pytest

import oracle
from jepsen.etcd_amd import abi, edn, history as H, synth
from jepsen.etcd_amd.history import Tuple
from helpers import GOLDEN


def same_as_pack(hist, text=None, **kw):
    text = edn.to_edn(hist) if text is None else text
    h = edn.read(text, **kw)
    keys, ops, off, _ = H.pack(hist)
    assert h.keys == [edn._edn(k) for k in keys]
    assert h.ops.shape == ops.shape
    assert (h.ops == ops).all()
    assert (h.key_off == off).all()
    return h


def test_generated_history_matches_pack():
    hist, _ = synth.jepsen_history(40, 150, concurrency=10, p_info=0.05, p_anomaly=0.3, seed=77)
    h = same_as_pack(hist)
    assert h.n_events == len(hist)


def test_ops32_are_lc_pack32_of_the_records():
    """lc_edn_ops32 / lc_edn_key_base (ABI 4): the 24-byte records lc_check32
    takes are lc_pack32's narrowing of the parsed 48-byte ones."""
    hist, _ = synth.jepsen_history(30, 60, concurrency=6, p_info=0.05, p_anomaly=0.3, seed=17)
    h = edn.read(edn.to_edn(hist))
    o32, base = h.ops32()
    want, wbase = abi.pack32(h.ops, h.key_off)
    assert (o32 == want).all() and (base == wbase).all() and len(base) == h.n_keys


def test_ops16_are_lc_pack16_of_the_records():
    """lc_edn_ops16 (round 6): the 16-byte records lc_check16 takes are
    lc_pack16's of the parsed 48-byte ones, with lc_edn_key_base's bases."""
    hist, _ = synth.jepsen_history(30, 60, concurrency=6, p_info=0.05, p_anomaly=0.3, seed=17)
    h = edn.read(edn.to_edn(hist))
    o16, base = h.ops16()
    want, wbase = abi.pack16(h.ops, h.key_off)
    assert (o16 == want).all() and (base == wbase).all() and len(base) == h.n_keys


def test_threads_do_not_change_the_result():
    hist, _ = synth.jepsen_history(60, 400, concurrency=20, p_info=0.02, seed=3)
    text = edn.to_edn(hist).encode()
    a = edn.read(text, n_threads=1)
    b = edn.read(text, n_threads=8)
    assert len(hist) > 8 * 4096  # enough forms for 8 parse threads
    assert (a.ops == b.ops).all() and (a.key_off == b.key_off).all() and a.keys == b.keys


def test_kat8_and_nemesis_nontuple_histories():
    h8 = [
        {"type": "invoke", "f": "write", "process": 0, "value": Tuple("k", [None, 1])},
        {"type": "ok", "f": "write", "process": 0, "value": Tuple("k", [1, 1])},
        {"type": "invoke", "f": "cas", "process": 1, "value": Tuple("k", [None, [3, 4]])},
        {"type": "fail", "f": "cas", "process": 1, "value": Tuple("k", [None, [3, 4]])},
        {"type": "invoke", "f": "read", "process": 0, "value": Tuple("k", [None, None])},
        {"type": "ok", "f": "read", "process": 0, "value": Tuple("k", [1, 1])},
    ]
    same_as_pack(h8)
    hn = [
        {"type": "invoke", "f": "write", "process": 0, "value": Tuple(1, [None, 7])},
        {"type": "info", "f": "start", "process": "nemesis", "value": None},
        {"type": "info", "f": "write", "process": 0, "value": Tuple(1, [None, 7])},
        {"type": "invoke", "f": "cas", "process": 5, "value": Tuple(2, [None, [None, 3]])},
        {"type": "ok", "f": "cas", "process": 5, "value": Tuple(2, [1, [None, 3]])},
        {"type": "invoke", "f": "read", "process": 6, "value": Tuple(1, [None, None])},
        # a client op whose value is not a tuple goes to every key
        {"type": "invoke", "f": "read", "process": 9, "value": None},
        {"type": "ok", "f": "read", "process": 9, "value": None},
    ]
    same_as_pack(hn)


def test_unknown_f_bad_shapes_and_interning():
    h = [
        {"type": "invoke", "f": "frob", "process": 0, "value": Tuple("a", [None, 1])},
        {"type": "ok", "f": "frob", "process": 0, "value": Tuple("a", [1, 1])},
        {"type": "invoke", "f": "cas", "process": 1, "value": Tuple("b", [None, 3])},
        {"type": "ok", "f": "cas", "process": 1, "value": Tuple("b", [1, 3])},
        {"type": "invoke", "f": "write", "process": 2, "value": Tuple("c", [None, 1.0])},
        {"type": "ok", "f": "write", "process": 2, "value": Tuple("c", [1, 1.0])},
        {"type": "invoke", "f": "write", "process": 2, "value": Tuple("c", [None, 1])},
        {"type": "ok", "f": "write", "process": 2, "value": Tuple("c", [2, 1])},
        {"type": "invoke", "f": "write", "process": 2, "value": Tuple("c", [None, "x"])},
        {"type": "ok", "f": "write", "process": 2, "value": Tuple("c", [3, "x"])},
        {"type": "invoke", "f": "cas", "process": 3, "value": Tuple("c", [None, ["x", 1]])},
        {"type": "ok", "f": "cas", "process": 3, "value": Tuple("c", [4, ["x", 1]])},
        {"type": "invoke", "f": "read", "process": 4, "value": Tuple("c", [None, None])},
        {"type": "ok", "f": "read", "process": 4, "value": Tuple("c", [4.5, 1])},  # float version
        {"type": "invoke", "f": "read", "process": 4, "value": Tuple("c", [None, None])},
        {"type": "ok", "f": "read", "process": 4, "value": Tuple("c", [True, 1])},   # bool version
    ]
    hh = same_as_pack(h)
    c = hh.ops[hh.key_off[2]:hh.key_off[3]]
    assert c[0, 1] != c[1, 1]          # 1.0 and 1 are different values
    assert c[3].tolist()[:4] == [2, c[1, 1], c[2, 1], 4]   # cas "x" -> 1
    assert c[4, 0] == 3 and c[5, 0] == 3


def test_explicit_index_and_out_of_order_processes():
    h = [
        {"type": "invoke", "f": "write", "process": 0, "value": Tuple(7, [None, 1]), "index": 10},
        {"type": "invoke", "f": "read", "process": 1, "value": Tuple(7, [None, None]), "index": 11},
        {"type": "ok", "f": "read", "process": 1, "value": Tuple(7, [1, 1]), "index": 12},
        {"type": "ok", "f": "write", "process": 0, "value": Tuple(7, [1, 1]), "index": 13},
        {"type": "ok", "f": "read", "process": 3, "value": Tuple(7, [1, 1]), "index": 14},  # no invoke
        {"type": "invoke", "f": "read", "process": 1, "value": Tuple(7, [None, None]), "index": 15},
        {"type": "invoke", "f": "read", "process": 1, "value": Tuple(7, [None, None]), "index": 16},
    ]
    hh = same_as_pack(h)
    assert hh.ops[:, 4].tolist() == [10, 11, 15, 16]


SURFACE = """; a comment line
[#jepsen.history.Op{:index 0, :time 1, :type :invoke, :process 0, :f :write, :value [5 [nil 2]]}
 #jepsen.history.Op{:index 1, :time 2, :type :info, :process :nemesis, :f :start,
                    :value {"n1" [:isolated "n2"], :msg "a ] tricky \\" string (with) {brackets}"}}
 {:index 2 :time 3 :type :ok :process 0 :f :write :value [5 [1 2]] :extra #{1 2 3}}
 #_ {:index 99 :type :invoke :process 0 :f :read :value [5 [nil nil]]}
 {:index 3, :type :invoke, :process 1, :f :read, :value [5 [nil nil]], :c \\( }
 {:index 4, :type :ok, :process 1, :f :read, :value [5 [1 2]], :t #inst "2025-01-01T00:00:00Z", :n 10N, :r 1/2}
]
"""


def test_edn_surface_forms():
    h = edn.read(SURFACE)
    assert h.keys == ["5"] and h.n_events == 5
    assert h.ops.tolist() == [[1, 0, -1, 1, 0, 2], [0, 0, -1, 1, 3, 4]]
    assert h.value(0, 0) == "2"
    assert h.op_text(1, 1).startswith("{:index 4, :type :ok")
    assert h.op_text(0, 0).startswith("#jepsen.history.Op{:index 0")


def test_single_key_mode():
    text = ("{:type :invoke, :f :write, :process 0, :value [nil 1]}\n"
            "{:type :ok, :f :write, :process 0, :value [1 1]}\n"
            "{:type :invoke, :f :cas, :process 1, :value [nil [1 2]]}\n"
            "{:type :ok, :f :cas, :process 1, :value [2 [1 2]]}\n")
    h = edn.read(text, independent=False)
    assert h.n_keys == 1 and h.ops.tolist() == [[1, 0, -1, 1, 0, 1], [2, 1, 0, 2, 2, 3]]


@pytest.mark.parametrize("bad", ["{:type :invoke", "[{:a 1}", "{:a 1 :b}", '{:a "x}', "{:a 1]}"])
def test_syntax_errors_are_reported(bad):
    with pytest.raises(abi.LcError) as e:
        edn.read(bad)
    assert "byte" in str(e.value)


def test_empty_and_file_input(tmp_path):
    assert edn.read("").n_keys == 0
    hist, _ = synth.jepsen_history(5, 50, seed=9)
    p = tmp_path / "history.edn"
    p.write_text(edn.to_edn(hist))
    h = edn.read(str(p))
    keys, ops, off, _ = H.pack(hist)
    assert (h.ops == ops).all() and (h.key_off == off).all()
    e = tmp_path / "empty.edn"
    e.write_text("")
    assert edn.read(str(e)).n_keys == 0


def test_records_decide_like_the_generator():
    """The EDN round trip of a generated history decides (oracle) exactly as
    the generator's own packed records."""
    hist, labels = synth.jepsen_history(30, 120, concurrency=10, p_info=0.05,
                                        p_anomaly=0.3, seed=21)
    h = edn.read(edn.to_edn(hist))
    _, a = oracle.check(h.ops, h.key_off, algo=oracle.JITC)
    assert (a["verdict"][np.array(labels) == 0] == 1).all()
    assert (a["verdict"][np.array(labels) == 1] == 0).all()


@pytest.mark.gpu
def test_check_edn_end_to_end_gpu(tmp_path):
    hist, labels = synth.jepsen_history(50, 200, concurrency=10, p_info=0.05,
                                        p_anomaly=0.3, seed=0x5EED0005)
    p = tmp_path / "history.edn"
    p.write_text(edn.to_edn(hist))
    result, h = edn.check(str(p), device_mask=1)
    _, ref = oracle.check(h.ops, h.key_off, algo=oracle.JIT)
    want = {h.keys[k] for k in range(h.n_keys) if ref["verdict"][k] == 0}
    assert set(result["failures"]) == want and len(want) > 0
    assert result["valid?"] is False
    for k in want:
        r = result["results"][k]
        kk = h.keys.index(k)
        rec = h.key_off[kk] + ref["fail_op"][kk]
        assert r["op"] == (h.op_text(rec, 1) or h.op_text(rec, 0))
    assert edn.render(result).startswith("{:valid? false")


def _expected(path):
    """{key: (valid, op_index or None)} from a make_edn.py expected file."""
    import re
    out = {}
    for m in re.finditer(r"(\d+) \{:valid\? (\w+)(?: :op-index (\d+))?\}", open(path).read()):
        out[int(m.group(1))] = (m.group(2) == "true", int(m.group(3)) if m.group(3) else None)
    return out


@pytest.mark.parametrize("name", ["kat", "c1", "tiny", "info", "c5"])
def test_jvm_parity_kit_histories(name):
    """The JVM parity kit (tests/golden/edn, tools/jvm_parity/parity.clj):
    each exported Jepsen history, read back by this build's EDN reader,
    splits into keys whose oracle verdicts and failing completions equal the
    kit's expected file — so a JVM box running the reference's own checker
    over the same file compares against the decisions the fixtures pin."""
    import gzip
    base = os.path.join(GOLDEN, "edn", name)
    h = edn.read(gzip.open(base + ".edn.gz").read())
    exp = _expected(base + ".expected.edn")
    assert len(h.keys) == len(exp)
    _, r = oracle.check(h.ops, h.key_off, algo=oracle.JITC, n_threads=8, max_configs=1 << 22)
    for i, ktext in enumerate(h.keys):
        valid, op_index = exp[int(ktext)]
        if r["verdict"][i] == -1:
            continue  # beyond the oracle's budget (info fixture)
        assert r["verdict"][i] == (1 if valid else 0), ktext
        if not valid:
            assert r["fail_prefix_end"][i] == op_index, ktext
    assert (r["verdict"] != -1).mean() > 0.9


def _awkward(hist):
    """to_edn with forms, strings and comments that span lines and hold brackets."""
    out = []
    for i, line in enumerate(edn.to_edn(hist).splitlines()):
        if i % 7 == 3:
            line = line.replace(", ", ",\n  ")  # one op map over several lines
        if i % 11 == 5:
            out.append('{:type :info, :f :log, :process :nemesis, :value "a\n] } ) [\n \\"{"}')
        if i % 13 == 2:
            out.append("; ] a comment [ {")
        if i % 17 == 9:
            out.append("#_ {:type :invoke,\n :process 0}")
        out.append(line)
    return "\n".join(out) + "\n"


@pytest.mark.parametrize("wrapped", [False, True])
def test_parallel_scan_equals_the_serial_scan(monkeypatch, wrapped):
    """The scan cuts the file at newlines and stitches the pieces (edn.cpp
    scan_forms); with pieces of a few hundred bytes nearly every cut falls
    inside a multi-line form or string, and the result must still be the
    serial scan's: same records, spans and event count."""
    hist, _ = synth.jepsen_history(30, 200, concurrency=10, p_info=0.05, p_anomaly=0.2, seed=31)
    text = _awkward(hist)
    if wrapped:
        text = "[" + text + "]\n"
    a = edn.read(text, n_threads=1)
    monkeypatch.setenv("LC_EDN_MIN_PIECE", "300")
    for t in (2, 8, 64):
        b = edn.read(text, n_threads=t)
        assert b.n_events == a.n_events and b.keys == a.keys
        assert (b.ops == a.ops).all() and (b.key_off == a.key_off).all()
        for rec in range(0, len(a.ops), 97):
            assert b.op_text(rec, 0) == a.op_text(rec, 0) and b.op_text(rec, 1) == a.op_text(rec, 1)
    assert a.n_events == len(hist) + len(range(5, len(hist), 11))  # + the :log ops


def test_parallel_scan_reports_the_first_error(monkeypatch):
    hist, _ = synth.jepsen_history(10, 200, seed=32)
    lines = _awkward(hist).splitlines()
    lines[len(lines) // 3] += ")"
    lines[2 * len(lines) // 3] = '{:a "unterminated'
    text = "\n".join(lines)
    with pytest.raises(abi.LcError) as e1:
        edn.read(text, n_threads=1)
    monkeypatch.setenv("LC_EDN_MIN_PIECE", "300")
    for t in (2, 8, 64):
        with pytest.raises(abi.LcError) as e2:
            edn.read(text, n_threads=t)
        assert str(e2.value) == str(e1.value)
