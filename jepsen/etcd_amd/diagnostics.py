"""knossos's invalid-analysis keys for a GPU counterexample.

For an invalid key, knossos's linearizable checker (called at
register.clj:110-111) reports, beside :op (the op whose completion empties
the search frontier), the diagnostics users read first [ext: knossos 0.3.x
knossos.linear / knossos.wgl, not in this container — restated, parity
unpinned]:

* :previous-ok  the last :ok completion before :op in history order;
* :configs      configurations of the search just before :op completes —
                each {:model, :last-op (the last op it linearized),
                :pending (ops called and not yet linearized)};
* :last-op      the last op linearized, as in those configurations;
* :final-paths  from a configuration, paths of [{:op, :model}] steps that
                try to linearize :op and end in an inconsistent model.

Two sources, by the tier that decided the key:

* keys the frontier search decided (no witness): the search's own frontier
  just before :op's completion (include/lincheck_fx.h lc_fx_frontier — the
  oracle's JITC frontier at that return, configuration for configuration, in
  tests/test_fx.py), up to 10 configurations as knossos keeps;
* keys the version-order / gap tiers decided: the witness of the history
  prefix just before :op's completion (lc_aux, LC_WITNESS_PREFIX: a
  linearization, certified independently by the tests), which is one
  configuration of that frontier.

:final-paths are built from those configurations by stepping the
VersionedRegister model (register.clj:60-96) — with the model's own messages
— through :op alone and through each pending op followed by :op.  The
search does not record which op each configuration linearized last, so
frontier configurations carry no :last-op.
"""
from .abi import LC_INF

MAX_ENTRIES = 10  # knossos truncates :configs / :final-paths to 10


def step(state, op):
    """VersionedRegister.step (register.clj:60-96) over a completed op map:
    returns (next_state, None) or (None, inconsistency message)."""
    version, value = state
    try:
        op_version, op_value = op["value"]
    except (TypeError, ValueError):
        return None, "can't step %r" % (op.get("value"),)
    version1 = version + 1
    f = op.get("f")
    if f == "write":
        if op_version is not None and version1 != op_version:
            return None, "can't go from version %s to %s" % (version, op_version)
        return (version1, op_value), None
    if f == "cas":
        v, v1 = op_value
        if op_version is not None and version1 != op_version:
            return None, "can't go from version %s to %s" % (version, op_version)
        if value != v:
            return None, "can't CAS %s from %s to %s" % (_s(value), _s(v), _s(v1))
        return (version1, v1), None
    if f == "read":
        if op_version is not None and version != op_version:
            return None, "can't read version %s from version %s" % (op_version, version)
        if op_value is not None and value != op_value:
            return None, "can't read %s from register %s" % (_s(op_value), _s(value))
        return state, None
    return None, "no step for %r" % (f,)


def _s(x):
    """Clojure `str`, which the model's messages use (register.clj:78,93):
    nil prints as the empty string."""
    return "" if x is None else str(x)


def _model(state):
    return {"version": state[0], "value": state[1]}


def _op_map(rec):
    return rec["completion"] if rec.get("completion") is not None and rec["ret"] != LC_INF \
        else rec["invoke"]


def previous_ok(done, fail_ret):
    """The last :ok completion before history index fail_ret."""
    best = None
    for r in done:
        if r["type"] == "ok" and r["ret"] < fail_ret and (best is None or r["ret"] > best["ret"]):
            best = r
    return best["completion"] if best is not None else None


def _final_paths(done, fail_op, states_pending, stepper=None):
    """knossos's :final-paths: from each configuration (state, pending op
    indices), the paths that try to linearize the failing op — directly, or
    after one pending op — and end inconsistent; at most MAX_ENTRIES."""
    stepper = stepper or step
    paths = []

    def try_op(st, i):
        nxt, err = stepper(st, done[i])
        return (nxt, {"op": _op_map(done[i]), "model": _model(nxt)}) if err is None else \
            (None, {"op": _op_map(done[i]), "model": {"inconsistent": err}})

    for state, last, pending in states_pending:
        head = {"op": _op_map(done[last]) if last is not None else None, "model": _model(state)}
        _, end = try_op(state, fail_op)
        if "inconsistent" in end["model"] and len(paths) < MAX_ENTRIES:
            paths.append([head, end])
        for i in pending:
            if i == fail_op or len(paths) >= MAX_ENTRIES:
                continue
            st2, mid = try_op(state, i)
            path = [head, mid]
            if st2 is not None:
                _, end = try_op(st2, fail_op)
                if "inconsistent" not in end["model"]:
                    continue  # linearizes the op: not a final path
                path.append(end)
            paths.append(path)
    return paths


def frontier_analysis(done, fail_op, fail_ret, configs, values, versioned=True):
    """knossos-shaped keys from the search's frontier before the failing
    return.  configs: [(version, value id, pending record indices)] from
    lc_fx_frontier; values: the key's value table (id -> value)."""
    out = {"previous-ok": previous_ok(done, fail_ret)}

    def val(i):
        return None if i < 0 else values[i] if i < len(values) else i

    cfgs, sp = [], []
    for ver, vid, pending in configs[:MAX_ENTRIES]:
        state = (ver, val(vid))
        cfgs.append({"model": _model(state) if versioned else {"value": state[1]},
                     "pending": [done[i]["invoke"] for i in pending]})
        sp.append((state, None, list(pending)))
    out["configs"] = cfgs
    if versioned:
        out["final-paths"] = _final_paths(done, fail_op, sp)
    return out


def invalid_analysis(done, fail_op, fail_ret, witness=None, init=(0, None)):
    """knossos-shaped keys for an invalid key.  done: the key's completed
    ops (history.complete order = record order); fail_op: index of the
    failing record; witness: the key's lc_aux witness (mutation position per
    record) for the prefix ending at fail_ret - 1, or None."""
    out = {"previous-ok": previous_ok(done, fail_ret)}
    if witness is None:
        return out
    cut = fail_ret - 1
    muts = sorted((int(p), i) for i, p in enumerate(witness) if p >= 0)
    state = init
    last = None
    for _, i in muts:
        nxt, err = step(state, done[i])
        if err is not None:  # not a linearization: report no configuration
            return out
        state, last = nxt, i
    # the reads of the final version come after the last mutation (by return)
    final_reads = [i for i, r in enumerate(done)
                   if r["f"] == "read" and r["ret"] <= cut and isinstance(r["value"], (list, tuple))
                   and len(r["value"]) == 2 and r["value"][0] == state[0]]
    if final_reads:
        last = max(final_reads, key=lambda i: done[i]["ret"])
    linearized = {i for _, i in muts}
    pending = [i for i, r in enumerate(done)
               if r["call"] <= cut and i not in linearized and (r["ret"] > cut)]
    last_op = _op_map(done[last]) if last is not None else None
    cfg = {"model": _model(state), "last-op": last_op,
           "pending": [done[i]["invoke"] for i in pending]}
    paths = _final_paths(done, fail_op, [(state, last, pending)])
    out.update({"configs": [cfg], "last-op": last_op, "final-paths": paths})
    return out
