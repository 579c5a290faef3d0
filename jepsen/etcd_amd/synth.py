"""Jepsen-shaped synthetic histories (op maps) from the seeded generator.

lc_synth_key (include/lincheck_synth.h) simulates one key of the register
workload (register.clj:113-119) including :fail CAS ops and crashed (:info)
ops with process replacement.  This module renders several keys as ONE
Jepsen history — invoke/completion maps with independent tuples as values
(register.clj:28,34,43), processes per key as jepsen.independent's
concurrent-generator assigns them, plus interleaved nemesis ops — the input
the reference's checker receives.
"""
from . import abi
from .history import Tuple

_F = {0: "read", 1: "write", 2: "cas"}


def _nil(x):
    return None if x == abi.LC_NIL else int(x)


def key_events(k, ops, proc, status, proc_base):
    """(local_index, order, op-map) events for one key."""
    ev = []
    last = 0
    for r, p, st in zip(ops, proc, status):
        f, value, expected, version, call, ret = (int(x) for x in r)
        fk = _F[f]
        if fk == "read":
            inv_v = [None, None]
        elif fk == "write":
            inv_v = [None, _nil(value)]
        else:
            inv_v = [None, [_nil(expected), _nil(value)]]
        pid = proc_base + int(p)
        ev.append((call, 0, {"type": "invoke", "f": fk, "process": pid,
                             "value": Tuple(k, inv_v)}))
        last = max(last, call)
        if st == 1:  # ok
            if fk == "read":
                ok_v = [_nil(version), _nil(value)]
            elif fk == "write":
                ok_v = [_nil(version), _nil(value)]
            else:
                ok_v = [_nil(version), [_nil(expected), _nil(value)]]
            ev.append((ret, 1, {"type": "ok", "f": fk, "process": pid,
                                "value": Tuple(k, ok_v)}))
            last = max(last, ret)
        elif st == 0:  # fail (a CAS that did not succeed, register.clj:44)
            ev.append((ret, 1, {"type": "fail", "f": fk, "process": pid,
                                "value": Tuple(k, inv_v), "error": "did-not-succeed"}))
            last = max(last, ret)
    # crashed ops: the :info completion is logged late; knossos keeps the op
    # pending forever wherever the completion appears.
    for r, p, st in zip(ops, proc, status):
        if st == 2:
            f = _F[int(r[0])]
            last += 1
            ev.append((last, 1, {"type": "info", "f": f, "process": proc_base + int(p),
                                 "value": None, "error": "timeout"}))
    return ev


def jepsen_history(n_keys, ops_per_key, concurrency=10, n_values=5, p_info=0.0,
                   p_anomaly=0.0, seed=0x5EED0000, nemesis_every=97):
    """One interleaved Jepsen history over n_keys keys; returns (history, labels)."""
    events = []
    labels = []
    for k in range(n_keys):
        ops, proc, status, lab = abi.synth_key(k, ops_per_key, concurrency, n_values,
                                               p_info, p_anomaly, seed)
        labels.append(lab)
        for (li, order, op) in key_events(k, ops, proc, status, k * 100000):
            events.append((li, k, order, op))
    events.sort(key=lambda e: (e[0], e[1], e[2]))
    hist = []
    for n, (_, _, _, op) in enumerate(events):
        if nemesis_every and n % nemesis_every == nemesis_every - 1:
            hist.append({"type": "info", "f": "start-partition", "process": "nemesis",
                         "value": None})
        hist.append(op)
    # :info completions carry no tuple value: fix them to the key's tuple so
    # jepsen.independent routes them (Jepsen keeps the invoke's value).
    pending = {}
    for op in hist:
        if op["type"] == "invoke":
            pending[op["process"]] = op
        elif op["type"] == "info" and op["process"] != "nemesis" and op["value"] is None:
            op["value"] = pending[op["process"]]["value"]
    return hist, labels
