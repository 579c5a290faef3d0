"""Brute-force linearizability check for tiny register histories.

TEST INFRASTRUCTURE ONLY (tests/ may import it; the product path never does).
PARITY UNPINNED against outputs of the reference itself (no JVM here, and the
reference holds no fixtures for this path): this is the *definitional* checker
that the two C restatements (oracle.c: JIT-linear and WGL) are cross-checked
against.

Definition ("parity-critical definition"): a key is valid iff
some total order of {every :ok op} ∪ {any subset of the :info ops}
  * respects real time: ret(a) < call(b)  =>  a before b, and
  * steps VersionedRegister (register.clj:59-96) from (0, nil) without
    becoming inconsistent.
Enumerates subsets and permutations outright: only for <= ~8 ops.
"""
from itertools import combinations, permutations

READ, WRITE, CAS = 0, 1, 2
NIL = -1
INF = (1 << 63) - 1


def step(state, op):
    """VersionedRegister.step, register.clj:60-96. op = (f, value, expected,
    version, call, ret). Returns the next state or None if inconsistent."""
    ver, val = state
    f, value, expected, opver = op[0], op[1], op[2], op[3]
    if f == WRITE:                                   # :64-68
        if opver != NIL and opver != ver + 1:
            return None
        return (ver + 1, value)
    if f == CAS:                                     # :70-82
        if opver != NIL and opver != ver + 1:
            return None
        if val != expected:
            return None
        return (ver + 1, value)
    if f == READ:                                    # :84-96
        if opver != NIL and opver != ver:
            return None
        if value != NIL and value != val:
            return None
        return state
    raise ValueError("unknown f %r (register.clj:63 has no default)" % (f,))


def _order_ok(order, ops):
    # real-time: for i before j in order, must not have ret(j) < call(i)
    for a in range(len(order)):
        for b in range(a + 1, len(order)):
            if ops[order[b]][5] < ops[order[a]][4]:
                return False
    return True


def check(ops, init=(0, NIL)):
    """ops: list of 6-tuples. Returns True/False."""
    ok_ops = [i for i, o in enumerate(ops) if o[5] != INF]
    info_ops = [i for i, o in enumerate(ops) if o[5] == INF]
    for k in range(len(info_ops) + 1):
        for sub in combinations(info_ops, k):
            chosen = ok_ops + list(sub)
            for order in permutations(chosen):
                if not _order_ok(order, ops):
                    continue
                s = init
                good = True
                for i in order:
                    s = step(s, ops[i])
                    if s is None:
                        good = False
                        break
                if good:
                    return True
    return False


def first_failure(ops, init=(0, NIL)):
    """Canonical counterexample: the :ok op x with the smallest ret such that
    the prefix history truncated at ret(x) is not linearizable (ops returning
    after ret(x) become pending/optional; ops called after it are dropped).
    Returns the op index or -1 if the whole history is valid."""
    rets = sorted((o[5], i) for i, o in enumerate(ops) if o[5] != INF)
    for r, i in rets:
        prefix = []
        for o in ops:
            if o[4] > r:
                continue
            if o[5] > r:
                # still open at ret(x): optional, with its completed fields
                # (knossos completes invoke values before either analyzer runs)
                o = (o[0], o[1], o[2], o[3], o[4], INF)
            prefix.append(o)
        if not check(prefix, init):
            return i
    return -1
