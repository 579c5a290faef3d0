"""Checker mirror of the reference's plugin boundary for the register workload.

The reference builds, at /root/reference/src/jepsen/etcd/register.clj:108-112,

    (independent/checker
      (checker/compose {:linear   (checker/linearizable {:model (->VersionedRegister 0 nil)})
                        :timeline (timeline/html)}))

and jepsen calls it through the jepsen.checker/Checker protocol,
(check [this test history opts]) -> {:valid? ...}.  `register_checker()` is
the drop-in for that whole expression: one object whose check() splits the
history by key, completes and packs it on the host, and decides every key in
one batched GPU call (include/lincheck.h).  The result has
jepsen.independent/checker's shape:

    {"valid?": merged, "results": {k: {...}}, "failures": [k ...]}

with merged = false > "unknown" > true, and "failures" the keys whose
:valid? is false (jepsen.independent keeps :unknown keys out of :failures,
since :unknown is truthy in Clojure).  Each key's map has checker/compose's
shape, {"valid?", "linear": <the GPU verdict>, "timeline": ...}; with
timeline_dir set, the timeline half renders <dir>/independent/<k>/
timeline.html on the host (timeline.py), as jepsen's timeline/html would.
An invalid key's map also carries knossos's diagnostics (diagnostics.py):
"previous-ok", "configs" and "final-paths" — from the search's own frontier
just before the failing return (up to 10 configurations: one batched device
search over every invalid key, lc_check_frontiers, and lc_fx_frontier for a
key whose frontier outgrows it), and "last-op" from the witness of the prefix
before the failing return (lc_aux) for keys the version-order and gap tiers
decided.

Errors: a key with malformed records is "unknown" alone (cause
"malformed"), as jepsen.independent would lose only that key; unusable
arguments raise LcError, and jepsen's check-safe turns an exception into
{:valid? :unknown :error ...}, which `check_safe` reproduces.
"""
import os

from . import abi, diagnostics as D, history as H, linear_svg as LS, timeline as TL

UNKNOWN = "unknown"
# an invalid key the batched device search (lc_check_frontiers) could not
# take, and which the version-order / gap tiers decided, is re-searched alone
# (lc_fx_frontier) for knossos's :configs only when it has at most this many
# crashed ops (the frontier of a version-pinned key grows with its crashed ops
# only)
FRONTIER_MAX_CRASHED = 16
CERT_KINDS = {0: "none", 1: "dup", 2: "unreach", 3: "claims", 4: "pair", 5: "order", 6: "hall",
              7: "proof"}


class VersionedRegister:
    """The model of register.clj:55-96 as data: its initial state.  The step
    function itself runs on the GPU (check_kernel.hip, `legal`)."""

    def __init__(self, version=0, value=None):
        self.version = version
        self.value = value

    name = "versioned-register"

    def __repr__(self):  # register.clj:57
        return "v%s: %s" % (self.version, self.value)


class CASRegister:
    """knossos.model/cas-register: a value, read/write/cas, no versions."""
    name = "cas-register"
    version = 0

    def __init__(self, value=None):
        self.value = value


class Register(CASRegister):
    """knossos.model/register: read/write only (a :cas is :unknown)."""
    name = "register"


class Mutex:
    """knossos.model/mutex, the lock workload's model (lock.clj:244):
    :acquire / :release of one lock, initially free."""
    name = "mutex"
    version = 0
    value = None


def _merge_valid(vs):
    vs = list(vs)
    if any(v is False for v in vs):
        return False
    if any(v == UNKNOWN for v in vs):
        return UNKNOWN
    return True


class RegisterChecker:
    """Drop-in for independent/checker + checker/linearizable(VersionedRegister)
    (register.clj:108-112).  With independent=False it is a plain
    checker/linearizable over the whole history, e.g. the lock workload's
    (checker/linearizable {:model (model/mutex)}) at lock.clj:243-244; the
    result is then one key's map (no :results)."""

    def __init__(self, model=None, device_mask=0, max_configs_per_key=0, independent=True,
                 timeline_dir=None, time_budget_ms=0, whole_gpu=True, frontier_max_keys=1000):
        self.model = model or VersionedRegister(0, None)
        # cap on the frontier re-searches one check() runs for diagnostics of
        # witnessed invalid keys (each is one key's search up to its failing
        # return, bounded by max_configs_per_key / time_budget_ms); 0: none
        self.frontier_max_keys = frontier_max_keys
        self.device_mask = device_mask
        self.max_configs_per_key = max_configs_per_key
        self.independent = independent
        self.timeline_dir = timeline_dir
        self.time_budget_ms = time_budget_ms
        # a key one workgroup's search leaves :unknown at the configuration
        # budget is searched again over the whole GPU (LC_FLAG_WHOLE_GPU):
        # knossos keeps searching until it runs out of memory or time, so the
        # drop-in does too by default (time_budget_ms bounds it)
        self.whole_gpu = whole_gpu
        self._ctx = None
        self._fx = None

    def _context(self):
        if self._ctx is None:
            self._ctx = abi.Context(self.device_mask)
        return self._ctx

    def _frontier(self):
        if self._fx is None:
            from .fx import FrontierExchange
            dev = 0
            while self.device_mask and not (self.device_mask >> dev) & 1:
                dev += 1
            self._fx = FrontierExchange(device=dev)
        return self._fx

    def check(self, test, history, opts=None):
        m = self.model
        values = []
        keys, ops, key_off, done = H.pack(history, model=m.name, independent=self.independent,
                                          init_value=m.value, values_out=values)
        if not keys:
            return {"valid?": True, "results": {}, "failures": []}
        # the initial value is interned first in every key (id 0); the mutex
        # starts free (id MUTEX_FREE)
        init = H.MUTEX_FREE if m.name == "mutex" else (0 if m.value is not None else H.LC_NIL)
        o = abi.default_opts(self.max_configs_per_key, m.version, init,
                             flags=abi.LC_FLAG_WHOLE_GPU if self.whole_gpu else 0,
                             time_budget_ms=self.time_budget_ms)
        # the drop-in's call (ABI 5): 16-byte records when every value id
        # fits 15 bits, else 24-byte ones — what crosses PCIe (the JVM shim
        # packs them directly; here lc_pack16 / lc_pack32 narrow the 48-byte
        # pack by the same rules)
        p16 = abi.pack16(ops, key_off)
        if p16 is not None:
            ops16, key_base = p16
            _, res, wit, kind, cert, cset = self._context().check16(
                ops16, key_off, key_base, o, witness=True, certificate=True)
        else:
            ops32, key_base = abi.pack32(ops, key_off)
            _, res, wit, kind, cert, cset = self._context().check32(
                ops32, key_off, key_base, o, witness=True, certificate=True)
        cfgs_of = self._configs(ops, key_off, res, o)
        results = {}
        n_fallback = 0  # one-key frontier re-searches run for diagnostics in this call
        for i, k in enumerate(keys):
            r = res[i]
            v = {1: True, 0: False}.get(int(r["verdict"]), UNKNOWN)
            out = {"valid?": v, "analyzer": "mi355x",
                   "configs-explored": int(r["configs_explored"]),
                   "max-frontier": int(r["max_frontier"])}
            if v is False:
                d = done[i][int(r["fail_op"])]
                out["op"] = d["completion"] or d["invoke"]
                out["fail-prefix-end"] = int(r["fail_prefix_end"])
                # why the prefix at the failing return has no linearization
                # (include/lincheck.h LC_CERT_*; checkable from the records)
                ck = CERT_KINDS.get(int(cert[i][0]), "none")
                out["certificate"] = {"kind": ck}
                if ck in ("dup", "unreach", "claims", "pair", "order"):
                    out["certificate"]["ops"] = [done[i][int(x)]["completion"] or done[i][int(x)]["invoke"]
                                                 for x in cert[i][1:3] if x >= 0]
                elif ck == "hall":
                    out["certificate"]["positions"] = [
                        int(x) for x in cset[key_off[i]:key_off[i] + int(cert[i][3])]]
                elif ck == "proof":  # the case splits: (position, cases) in preorder
                    out["certificate"]["splits"] = [
                        ((int(x) & 0xFFFFFFFF) >> 15 & 0x7FFF, int(x) & 0x7FFF)
                        for x in cset[key_off[i]:key_off[i] + int(cert[i][3])]]
                recs = ops[key_off[i]:key_off[i + 1]]
                witnessed = m.name == "versioned-register" and kind[i] == abi.LC_WITNESS_PREFIX
                # knossos's :configs are its search's frontier just before the
                # failing return: every invalid key's came from one batched
                # device search (lc_check_frontiers, _configs); a key that
                # search could not take (its frontier outgrew the LDS tier) is
                # re-searched alone by the frontier exchange (lc_fx_frontier)
                # — any key the search decided, and witnessed keys with at
                # most FRONTIER_MAX_CRASHED crashed ops — at most
                # frontier_max_keys such re-searches per call (the Clojure
                # shim counts the same way); beyond that, or if the re-search
                # fails, the witness's one configuration (with
                # "configs-error" saying why)
                cfgs, err = cfgs_of.get(i), None
                if cfgs is None and n_fallback < self.frontier_max_keys and (
                        not witnessed or
                        int((recs[:, 5] == abi.LC_INF).sum()) <= FRONTIER_MAX_CRASHED):
                    n_fallback += 1
                    try:
                        cfgs = self._frontier().frontier(recs, int(r["fail_op"]), D.MAX_ENTRIES, o)
                    except Exception as e:  # noqa: BLE001 — diagnostics only; the verdict stands
                        err = repr(e)
                wa = D.invalid_analysis(done[i], int(r["fail_op"]), int(r["fail_prefix_end"]),
                                        wit[key_off[i]:key_off[i + 1]],
                                        init=(m.version, m.value)) if witnessed else None
                if cfgs is not None:
                    out.update(D.frontier_analysis(
                        done[i], int(r["fail_op"]), int(r["fail_prefix_end"]), cfgs, values[i],
                        versioned=m.name == "versioned-register"))
                    if wa is not None and "last-op" in wa:
                        out["last-op"] = wa["last-op"]  # the witness's last linearized op
                elif wa is not None:
                    out.update(wa)
                else:
                    out["previous-ok"] = D.previous_ok(done[i], int(r["fail_prefix_end"]))
                if err is not None:
                    out["configs-error"] = err
            elif v == UNKNOWN:
                # the Clojure shim's keys (mi355x.clj): :cause and :error
                cause = abi.REASONS.get(int(r["reason"]), int(r["reason"]))
                out["cause"] = cause
                out["error"] = ["lincheck-reason", cause]
            results[k] = out
        if not self.independent:
            return results[None]
        subs = H.split_by_key(H.index_history(history)) if self.timeline_dir else None
        for i, (k, lin) in enumerate(results.items()):
            if self.timeline_dir and lin["valid?"] is False and "final-paths" in lin:
                # jepsen's checker/linearizable renders a failed analysis
                # into the key's directory as linear.svg
                lin["linear-svg"] = LS.write(
                    os.path.join(self.timeline_dir, "independent", str(k), "linear.svg"),
                    done[i], lin, title="key %s" % (k,))
            results[k] = self._composed(k, lin, subs)
        return {"valid?": _merge_valid(r["valid?"] for r in results.values()),
                "results": results,
                "failures": [k for k, r in results.items() if r["valid?"] is False]}

    def _configs(self, ops, key_off, res, opts):
        """knossos's :configs of every invalid key in one device call
        (lc_check_frontiers): {key index: [(version, value id, pending)]},
        the keys the device search could not take left out."""
        import numpy as np
        inv = np.nonzero(res["verdict"] == abi.LC_INVALID)[0]
        if self.frontier_max_keys <= 0 or len(inv) == 0:
            return {}
        parts = [ops[key_off[i]:key_off[i + 1]] for i in inv]
        sub_off = np.zeros(len(inv) + 1, dtype=np.int64)
        sub_off[1:] = np.cumsum([len(x) for x in parts])
        try:
            got = self._context().check_frontiers(np.concatenate(parts), sub_off,
                                                  res["fail_op"][inv], D.MAX_ENTRIES, opts)
        except Exception:  # noqa: BLE001 — diagnostics only; the verdicts stand
            # (as mi355x.clj batched-configs): every key falls back to the
            # one-key re-search or its witness
            return {}
        return {int(i): c for i, c in zip(inv, got) if c is not None}

    def _composed(self, k, linear, subs):
        """checker/compose's per-key map (register.clj:109-112)."""
        if subs is None:
            return {"valid?": linear["valid?"], "linear": linear}
        path = os.path.join(self.timeline_dir, "independent", str(k), "timeline.html")
        tl = TL.write(path, subs[k], title="key %s" % (k,),
                      cex_index=linear.get("fail-prefix-end"))
        return {"valid?": _merge_valid([linear["valid?"], tl["valid?"]]),
                "linear": linear, "timeline": tl}

    def close(self):
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None
        if self._fx is not None:
            self._fx.close()
            self._fx = None


def register_checker(**kw):
    return RegisterChecker(**kw)


def linearizable(model, **kw):
    """checker/linearizable {:model model} over the whole history (no
    independent split)."""
    return RegisterChecker(model=model, independent=False, **kw)


def check_safe(checker, test, history, opts=None):
    """jepsen.checker/check-safe: exceptions become {:valid? :unknown :error}."""
    try:
        return checker.check(test, history, opts)
    except Exception as e:  # noqa: BLE001 — mirrors check-safe's catch-all
        return {"valid?": UNKNOWN, "error": repr(e)}
