"""Export the golden fixtures as Jepsen histories for a JVM parity run.

For each fixture (tests/golden/{c1,c5,info,tiny}.npz and the hand-derived
KATs in kat.json) this writes tests/golden/edn/<name>.edn.gz — one Jepsen op
map per line, the history the reference's checker consumes — and
<name>.expected.edn — the verdict every key must get, with the history index
of the failing completion for invalid keys.  tools/jvm_parity/parity.clj
runs the reference's own (independent/checker (checker/linearizable {:model
(->VersionedRegister 0 nil)})) (register.clj:108-111) over each history on a
box that has a JVM and the reference's dependencies, and diffs its verdicts
against the expected file; the same histories are checked here by
test_edn.py against the packed fixtures (so the two files describe the same
decisions the GPU tests pin).

History construction from packed records (key k, record r): a fresh process
per op (k * 1e6 + r); the invoke at the record's call index with
[nil nil] / [nil v] / [nil [old new]] (register.clj:98-100); an :ok
completion at its ret index with [version value] / [version [old new]]
(register.clj:27-43); a crashed op gets an :info completion after the
last event.  Values are tuples [k value] (jepsen.independent).

    python tests/golden/make_edn.py
"""
import gzip
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from jepsen.etcd_amd.edn import op_edn  # noqa: E402
from jepsen.etcd_amd.history import Tuple  # noqa: E402

INF = (1 << 63) - 1
FN = {0: "read", 1: "write", 2: "cas"}


def nil(x):
    return None if x == -1 else int(x)


def history(ops, key_off):
    ev = []
    last = 0
    for k in range(len(key_off) - 1):
        for r in range(int(key_off[k]), int(key_off[k + 1])):
            f, value, expected, version, call, ret = (int(x) for x in ops[r])
            fk = FN[f]
            proc = k * 1000000 + (r - int(key_off[k]))
            inv = [None, None] if fk == "read" else \
                [None, nil(value)] if fk == "write" else [None, [nil(expected), nil(value)]]
            ev.append((call, 0, {"type": "invoke", "f": fk, "process": proc,
                                 "value": Tuple(k, inv)}))
            last = max(last, call)
            if ret != INF:
                ok = [nil(version), [nil(expected), nil(value)] if fk == "cas" else nil(value)]
                ev.append((ret, 1, {"type": "ok", "f": fk, "process": proc,
                                    "value": Tuple(k, ok)}))
                last = max(last, ret)
    # crashed ops: :info completions after everything
    extra = []
    for (_, _, op) in ev:
        if op["type"] == "invoke":
            extra.append(op)
    done = {op["process"] for (_, _, op) in ev if op["type"] == "ok"}
    ev.sort(key=lambda e: (e[0], e[1]))
    out = [op for (_, _, op) in ev]
    for op in extra:
        if op["process"] not in done:
            out.append({"type": "info", "f": op["f"], "process": op["process"],
                        "value": op["value"], "error": "timeout"})
    for i, op in enumerate(out):
        op["index"] = i
    return out


def write(name, ops, key_off, verdict, fail_op):
    hist = history(ops, key_off)
    # the failing completion's history index, per key (the re-indexed ret)
    ret_index = {}
    for op in hist:
        if op["type"] == "ok":
            ret_index[op["process"]] = op["index"]
    with gzip.open(os.path.join(HERE, "edn", name + ".edn.gz"), "wt") as fh:
        for op in hist:
            fh.write(op_edn(op) + "\n")
    lines = []
    for k in range(len(key_off) - 1):
        if key_off[k + 1] == key_off[k]:
            continue  # no ops: jepsen.independent never sees the key
        v = {1: "true", 0: "false"}.get(int(verdict[k]), ":unknown")
        fo = int(fail_op[k])
        extra = ""
        if fo >= 0:
            extra = " :op-index %d" % ret_index[k * 1000000 + fo]
        lines.append("%d {:valid? %s%s}" % (k, v, extra))
    with open(os.path.join(HERE, "edn", name + ".expected.edn"), "w") as fh:
        fh.write("{" + "\n ".join(lines) + "}\n")
    return len(hist)


def as_jepsen(ops, key_off, verdict, fail_op):
    """The records a Jepsen history can express: a crashed op's value is its
    invoke's [nil ...], so a version on one (some tiny random fixtures carry
    it) is dropped.  Keys whose records change are re-decided by the
    oracle's JIT restatement (test infrastructure) for the expected file."""
    ops = np.array(ops, dtype=np.int64)
    changed = (ops[:, 5] == INF) & (ops[:, 3] != -1)
    verdict = np.array(verdict).copy()
    fail_op = np.array(fail_op).copy()
    if changed.any():
        sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
        import oracle
        ops[changed, 3] = -1
        _, r = oracle.check(ops, key_off, algo=oracle.JIT)
        keys = np.unique(np.searchsorted(key_off, np.nonzero(changed)[0], side="right") - 1)
        verdict[keys] = r["verdict"][keys]
        fail_op[keys] = r["fail_op"][keys]
    return ops, verdict, fail_op


def main():
    for name in ("c1", "c5", "info", "tiny"):
        z = np.load(os.path.join(HERE, name + ".npz"))
        ops, verdict, fail_op = as_jepsen(z["ops"], z["key_off"], z["verdict"], z["fail_op"])
        n = write(name, ops, z["key_off"], verdict, fail_op)
        print(name, n, "events")
    kats = json.load(open(os.path.join(HERE, "kat.json")))
    rows, off = [], [0]
    for k in kats:
        rows.extend(k["ops"])
        off.append(len(rows))
    ops = np.array(rows, dtype=np.int64).reshape(-1, 6)
    n = write("kat", ops, np.array(off), [1 if k["valid"] else 0 for k in kats],
              [k["fail_op"] for k in kats])
    print("kat", n, "events")


if __name__ == "__main__":
    main()
