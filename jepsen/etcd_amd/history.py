"""Host-side history preprocessing: Jepsen op maps -> packed lc_op records.

Mirrors, on the host, what happens between jepsen.core's analysis call and the
model's step function for the register workload:

* client ops only (an integer :process) — nemesis ops have no model step
  (register.clj:63, condp without a default clause);
* jepsen.independent's per-key split (register.clj:108): ops whose value is
  an independent tuple [k v] (register.clj:28,34,43) belong to key k, with the
  value unwrapped; ops with a non-tuple value belong to every key;
* knossos history completion: an invoke is paired with the next completion of
  the same process; :ok copies the completion value into the op, :fail drops
  the pair, :info (or no completion) leaves the invoke value and makes the op
  pending forever (ret = LC_INF);
* values are interned per key to dense ids by equality (nil -> LC_NIL), and
  each op becomes one 48-byte record (include/lincheck.h):
  (f, value, expected, version, call, ret), sorted by call.

Histories are sequences of dicts {"type", "f", "process", "value"[, "index"]}
with string keywords ("invoke", "ok", "fail", "info"; "read", "write", "cas").
"""
from collections import namedtuple

import numpy as np

from .abi import LC_F_CAS, LC_F_READ, LC_F_WRITE, LC_INF, LC_NIL

F_CODES = {"read": LC_F_READ, "write": LC_F_WRITE, "cas": LC_F_CAS}
F_UNKNOWN = 3  # the device reports :unknown for it, as the model would throw


class Tuple(namedtuple("Tuple", ["key", "value"])):
    """jepsen.independent/tuple: a [k v] pair marking a per-key value."""


def tuple_(k, v):
    return Tuple(k, v)


def _kw(x):
    if isinstance(x, str) and x.startswith(":"):
        return x[1:]
    return x


def is_client(op):
    p = op.get("process")
    return isinstance(p, int) and not isinstance(p, bool)


def history_keys(history):
    """Distinct independent keys in order of first appearance."""
    seen, out = set(), []
    for op in history:
        v = op.get("value")
        if isinstance(v, Tuple) and v.key not in seen:
            seen.add(v.key)
            out.append(v.key)
    return out


def index_history(history):
    """Attach :index (position) where missing; returns a list of dicts."""
    out = []
    for i, op in enumerate(history):
        if "index" not in op:
            op = dict(op)
            op["index"] = i
        out.append(op)
    return out


def split_by_key(history):
    """{k: [op...]} — jepsen.independent/subhistory for every key, client ops
    only, tuple values unwrapped.  Non-tuple client ops go to every key."""
    keys = history_keys(history)
    subs = {k: [] for k in keys}
    for op in history:
        if not is_client(op):
            continue
        v = op.get("value")
        if isinstance(v, Tuple):
            o = dict(op)
            o["value"] = v.value
            subs[v.key].append(o)
        else:
            for k in keys:
                subs[k].append(op)
    return subs


class Interner:
    """Dense ids for values by equality; None is LC_NIL."""

    def __init__(self):
        self.ids = {}
        self.values = []

    def __call__(self, v):
        if v is None:
            return LC_NIL
        key = (type(v).__name__, v) if not isinstance(v, (list, dict)) else repr(v)
        i = self.ids.get(key)
        if i is None:
            i = len(self.values)
            self.ids[key] = i
            self.values.append(v)
        return i


def _fields(f, value, intern):
    """(value, expected, version) for a [version value] op value, or None if
    the value does not have the register workload's shape."""
    if not isinstance(value, (list, tuple)) or len(value) != 2:
        return None
    version, v = value
    if version is not None and (not isinstance(version, int) or isinstance(version, bool)):
        return None
    ver = LC_NIL if version is None else int(version)
    if f == LC_F_CAS:
        if not isinstance(v, (list, tuple)) or len(v) != 2:
            return None
        return intern(v[1]), intern(v[0]), ver
    return intern(v), LC_NIL, ver


def complete(subhistory):
    """knossos history completion for one key: list of dicts
    {"f", "value", "call", "ret", "invoke", "completion"} in invoke order."""
    pending = {}
    ops = []
    for op in subhistory:
        t = _kw(op.get("type"))
        p = op.get("process")
        if t == "invoke":
            rec = {"f": _kw(op.get("f")), "value": op.get("value"),
                   "call": op["index"], "ret": LC_INF, "invoke": op,
                   "completion": None, "type": "info"}
            pending[p] = rec
            ops.append(rec)
        elif t in ("ok", "fail", "info"):
            rec = pending.pop(p, None)
            if rec is None:
                continue  # completion without invoke: ignored
            rec["completion"] = op
            rec["type"] = t
            if t == "ok":
                rec["value"] = op.get("value")
                rec["ret"] = op["index"]
    return [r for r in ops if r["type"] != "fail"]


def pack_key(subhistory, intern=None):
    """One key's subhistory -> (records (n,6) int64, completed ops list)."""
    intern = intern or Interner()
    done = complete(subhistory)
    recs = np.zeros((len(done), 6), dtype=np.int64)
    for i, r in enumerate(done):
        f = F_CODES.get(r["f"], F_UNKNOWN)
        flds = _fields(f, r["value"], intern) if f != F_UNKNOWN else None
        if flds is None:
            f, flds = F_UNKNOWN, (LC_NIL, LC_NIL, LC_NIL)
        recs[i] = (f, flds[0], flds[1], flds[2], r["call"], r["ret"])
    return recs, done


def pack(history):
    """Whole history -> (keys, ops (n,6), key_off, per-key completed ops)."""
    hist = index_history(history)
    subs = split_by_key(hist)
    keys = list(subs.keys())
    parts, done = [], []
    for k in keys:
        recs, d = pack_key(subs[k])
        parts.append(recs)
        done.append(d)
    key_off = np.zeros(len(keys) + 1, dtype=np.int64)
    for i, p in enumerate(parts):
        key_off[i + 1] = key_off[i] + len(p)
    ops = np.concatenate(parts) if parts else np.zeros((0, 6), dtype=np.int64)
    return keys, ops, key_off, done
