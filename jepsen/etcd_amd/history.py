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

Models: the record format is the device's model.
A register op's precondition is a (version, value) match and its effect a
version bump plus a new value, so knossos's other register-like models are
packings, not new kernels:

* "versioned-register" — register.clj:55-96: values [version x];
* "cas-register" — knossos.model/cas-register: values are x itself, no
  versions (a nil version is never checked, register.clj:64-92); read nil
  matches any state;
* "register" — knossos.model/register: as cas-register, and a :cas has no
  step (knossos's condp throws), so it packs as an unknown f;
* "mutex" — knossos.model/mutex, the lock workload's model (lock.clj:244):
  the state is held / free; :acquire is a CAS free -> held, :release a CAS
  held -> free, with the fixed value ids FREE = 0 and HELD = 1 and the
  initial state free.
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


def _fields_plain(f, value, intern):
    """knossos cas-register: read/write x, cas [old new]; no versions."""
    if f == LC_F_CAS:
        if not isinstance(value, (list, tuple)) or len(value) != 2:
            return None
        return intern(value[1]), intern(value[0]), LC_NIL
    return intern(value), LC_NIL, LC_NIL


MUTEX_FREE, MUTEX_HELD = 0, 1


def _record(model, fk, value, intern):
    """(f, value, expected, version) of one completed op under `model`."""
    if model == "mutex":
        if fk == "acquire":
            return LC_F_CAS, MUTEX_HELD, MUTEX_FREE, LC_NIL
        if fk == "release":
            return LC_F_CAS, MUTEX_FREE, MUTEX_HELD, LC_NIL
        return F_UNKNOWN, LC_NIL, LC_NIL, LC_NIL
    f = F_CODES.get(fk, F_UNKNOWN)
    if model == "register" and f == LC_F_CAS:
        f = F_UNKNOWN
    flds = None
    if f != F_UNKNOWN:
        flds = (_fields if model == "versioned-register" else _fields_plain)(f, value, intern)
    if flds is None:
        return F_UNKNOWN, LC_NIL, LC_NIL, LC_NIL
    return (f,) + tuple(flds)


MODELS = ("versioned-register", "cas-register", "register", "mutex")


def pack_key(subhistory, intern=None, model="versioned-register"):
    """One key's subhistory -> (records (n,6) int64, completed ops list)."""
    if model not in MODELS:
        raise ValueError("unknown model %r (one of %s)" % (model, ", ".join(MODELS)))
    intern = intern or Interner()
    done = complete(subhistory)
    recs = np.zeros((len(done), 6), dtype=np.int64)
    for i, r in enumerate(done):
        f, v, e, ver = _record(model, r["f"], r["value"], intern)
        recs[i] = (f, v, e, ver, r["call"], r["ret"])
    return recs, done


def pack(history, model="versioned-register", independent=True, init_value=None,
         values_out=None):
    """Whole history -> (keys, ops (n,6), key_off, per-key completed ops).

    independent=False checks the history as one key (checker/linearizable
    without jepsen.independent, as lock.clj:243-244 does); its key is None.
    A non-nil init_value is interned first in every key, so it is id 0 there
    (pass 0 as lc_opts.init_value).  values_out (a list), if given, receives
    each key's value table (id -> value)."""
    hist = index_history(history)
    if independent:
        subs = split_by_key(hist)
    else:
        subs = {None: [op for op in hist if is_client(op)]}
    keys = list(subs.keys())
    parts, done = [], []
    for k in keys:
        it = Interner()
        if init_value is not None and model != "mutex":
            it(init_value)
        recs, d = pack_key(subs[k], it, model)
        if values_out is not None:
            values_out.append(it.values)
        parts.append(recs)
        done.append(d)
    key_off = np.zeros(len(keys) + 1, dtype=np.int64)
    for i, p in enumerate(parts):
        key_off[i + 1] = key_off[i] + len(p)
    ops = np.concatenate(parts) if parts else np.zeros((0, 6), dtype=np.int64)
    return keys, ops, key_off, done
