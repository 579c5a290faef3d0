"""knossos's invalid-analysis keys (jepsen/etcd_amd/diagnostics.py) built
from a prefix witness: previous-ok, configs, last-op, final-paths.  On CPU
the witness comes from the restated gap procedure (tests/gapmatch_ref.py);
the GPU path is covered by test_gpu.py::test_register_checker_end_to_end."""
import numpy as np

import gapmatch_ref as gm
from jepsen.etcd_amd import diagnostics as D, history as H, synth
from jepsen.etcd_amd.history import Tuple


def test_step_messages_follow_register_clj():
    w = {"f": "write", "value": [3, 7]}
    assert D.step((1, 5), w) == (None, "can't go from version 1 to 3")
    assert D.step((2, 5), w) == ((3, 7), None)
    c = {"f": "cas", "value": [None, [4, 9]]}
    assert D.step((2, 5), c) == (None, "can't CAS 5 from 4 to 9")
    # Clojure `str` prints nil as "" (register.clj:78), so does the model's message
    assert D.step((0, None), {"f": "cas", "value": [1, [0, 1]]}) == \
        (None, "can't CAS  from 0 to 1")
    assert D.step((1, None), {"f": "read", "value": [1, 3]}) == \
        (None, "can't read 3 from register ")
    r = {"f": "read", "value": [2, 1]}
    assert D.step((3, 1), r) == (None, "can't read version 2 from version 3")
    assert D.step((2, 4), r) == (None, "can't read 1 from register 4")
    assert D.step((2, 1), r) == ((2, 1), None)
    assert D.step((5, 1), {"f": "read", "value": [None, None]}) == ((5, 1), None)


def test_stale_read_analysis():
    """KAT2: w1 ok [1 1], w2 ok [2 2], then a read ok [1 1] invoked after
    both: the read fails; previous-ok is w2's completion; the one
    configuration is (v2, 2) after w2, and the read cannot step from it."""
    T = Tuple
    h = [
        {"type": "invoke", "f": "write", "process": 0, "value": T("k", [None, 1])},
        {"type": "ok", "f": "write", "process": 0, "value": T("k", [1, 1])},
        {"type": "invoke", "f": "write", "process": 1, "value": T("k", [None, 2])},
        {"type": "ok", "f": "write", "process": 1, "value": T("k", [2, 2])},
        {"type": "invoke", "f": "read", "process": 2, "value": T("k", [None, None])},
        {"type": "ok", "f": "read", "process": 2, "value": T("k", [1, 1])},
    ]
    keys, ops, off, done = H.pack(h)
    recs = [tuple(r) for r in ops.tolist()]
    fo, at = gm.first_failure(recs)
    assert (fo, at) == (2, 5)
    v, w = gm.decide(recs, cutoff=at - 1, witness=True)
    assert v == 1
    a = D.invalid_analysis(done[0], fo, at, np.array(w))
    assert a["previous-ok"]["index"] == 3
    cfg = a["configs"][0]
    assert cfg["model"] == {"version": 2, "value": 2} and cfg["last-op"]["index"] == 3
    assert [p["index"] for p in cfg["pending"]] == [4]
    assert a["final-paths"] == [[{"op": cfg["last-op"], "model": {"version": 2, "value": 2}},
                                 {"op": {"type": "ok", "f": "read", "process": 2,
                                         "value": [1, 1], "index": 5},
                                  "model": {"inconsistent":
                                                        "can't read version 1 from version 2"}}]]


def test_analysis_on_synthetic_anomalies():
    """Injected stale reads / lost CAS with crashes: every invalid key gets
    previous-ok before the failing completion, one configuration whose model
    the witness reaches, pending ops called before the cut, and final paths
    that all end inconsistent."""
    hist, labels = synth.jepsen_history(40, 150, concurrency=10, p_info=0.1,
                                        p_anomaly=0.6, seed=17)
    keys, ops, off, done = H.pack(hist)
    n_inv = 0
    for k in range(len(keys)):
        recs = [tuple(r) for r in ops[off[k]:off[k + 1]].tolist()]
        if gm.decide(recs) != 0:
            continue
        fo, at = gm.first_failure(recs)
        v, w = gm.decide(recs, cutoff=at - 1, witness=True)
        assert v == 1
        a = D.invalid_analysis(done[k], fo, at, np.array(w))
        n_inv += 1
        assert a["previous-ok"] is None or a["previous-ok"]["index"] < at
        cfg = a["configs"][0]
        assert all(p["index"] < at for p in cfg["pending"])
        assert 1 <= len(a["final-paths"]) <= D.MAX_ENTRIES
        for path in a["final-paths"]:
            assert "inconsistent" in path[-1]["model"]
            assert all("inconsistent" not in s["model"] for s in path[:-1])
    assert n_inv >= 10


def test_linear_svg_draws_the_failure(tmp_path):
    """linear.svg (jepsen/etcd_amd/linear_svg.py, the restated knossos
    render-analysis! figure): one bar per op the analysis names, the failing
    op drawn as the failure, every final path ending in a red inconsistent
    step labelled with the model's message; valid XML."""
    import xml.etree.ElementTree as ET
    from jepsen.etcd_amd import linear_svg as LS
    hist, labels = synth.jepsen_history(20, 120, concurrency=8, p_info=0.1,
                                        p_anomaly=0.8, seed=23)
    keys, ops, off, done = H.pack(hist)
    drawn = 0
    for k in range(len(keys)):
        recs = [tuple(r) for r in ops[off[k]:off[k + 1]].tolist()]
        if gm.decide(recs) != 0:
            continue
        fo, at = gm.first_failure(recs)
        v, w = gm.decide(recs, cutoff=at - 1, witness=True)
        a = D.invalid_analysis(done[k], fo, at, np.array(w))
        d = done[k][fo]
        a["op"] = d["completion"] or d["invoke"]
        path = LS.write(str(tmp_path / ("k%d" % k) / "linear.svg"), done[k], a, title="key %d" % k)
        root = ET.parse(path).getroot()
        ns = "{http://www.w3.org/2000/svg}"
        rects = root.findall(ns + "rect")
        rec = {id(r[f]): i for i, r in enumerate(done[k]) for f in ("invoke", "completion")
               if r.get(f) is not None}
        want = {rec[id(x)] for x in [a["previous-ok"], a["op"]] + a["configs"][0]["pending"]
                + [s["op"] for p in a["final-paths"] for s in p] if x is not None}
        assert len(rects) == len(want)
        assert [r.get("class") for r in rects].count("fail") == 1
        bad = [t.text for t in root.findall(ns + "text") if t.get("class") == "badmodel"]
        ends = [p[-1]["model"]["inconsistent"] for p in a["final-paths"]
                if "inconsistent" in p[-1]["model"]]
        assert sorted(bad) == sorted(ends) and ends
        drawn += 1
    assert drawn >= 3
