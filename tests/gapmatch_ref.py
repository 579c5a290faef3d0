"""Python restatement of the gap-matching decision procedure (test
infrastructure): decides keys whose :ok ops are version-pinned but which
also hold crashed (:info) writes/CAS — the SURVEY §7 ":info blow-up" case,
BASELINE configs[3] — without a frontier search.

Model (register.clj:59-96).  In any linearization, the k-th mutation (write
or successful CAS) takes the register from version V0+k-1 to V0+k.  So an
:ok mutation claiming version v is pinned to position p = v-V0-1, a read
claiming version v sits between positions v-V0-1 and v-V0, and the only
freedom left is which optional ops (crashed mutations; in a prefix, also
pending :ok mutations, pinned to their own position) fill the positions no
required mutation holds — the *gaps*.  Positions beyond the last one any
required op needs are never filled (an optional op may always be left out).

With linearization points t_0 < t_1 < ... (one per position) the history is
linearizable iff a filling exists with
    L_k < t_k < U_k,   L_k = max(call(m_k), calls of reads of version V0+k)
                       U_k = min(ret(m_k),  rets of reads of version V0+k+1)
and the values chain (register.clj:77 CAS expectations, read claims).  Points
exist iff max(L_0..L_k) < U_k for all k, i.e. iff L_j < min(U_j, U_{j+1}, ...)
= Uh_j for every j: the time constraint splits into one deadline per gap,
    call(op filling gap j) < Uh_j,
plus fixed checks on the pinned positions.  What remains is a bipartite
matching of gaps to optional ops (eligibility = deadline + value class),
coupled only where a gap's value is free and the next gap may take a CAS
(whose expectation then fixes it): those couplings are resolved by
branching on the free value, with the matching as a bound.

decide() returns 1 / 0, or None when the procedure does not apply (an :ok
mutation without a version, a read [nil x], an unknown :f, or the branch
budget ran out).  first_failure() returns the canonical counterexample
(index of the :ok op whose return first makes the prefix non-linearizable),
found by bisection over prefixes (linearizability is prefix-closed).
decide(..., witness=True) returns (verdict, positions): for a valid key the
mutation position of every record in the linearization the matching found
(-1 for records not linearized as mutations) — the lc_aux witness format, so
oracle.check_witness can certify this restatement's answers too.
"""
INF = (1 << 63) - 1
ANY = None  # a gap whose value nothing constrains


class _NA(Exception):
    pass


def _matching(n_gaps, elig, n_ops):
    """Maximum bipartite matching (augmenting paths).  elig[g] = op list."""
    match_op = [-1] * n_ops
    match_gap = [-1] * n_gaps
    for g0 in range(n_gaps):
        # BFS for an augmenting path from g0
        parent = {}
        seen = set()
        frontier = [g0]
        found = -1
        while frontier and found < 0:
            nxt = []
            for g in frontier:
                for o in elig[g]:
                    if o in seen:
                        continue
                    seen.add(o)
                    parent[o] = g
                    if match_op[o] < 0:
                        found = o
                        break
                    nxt.append(match_op[o])
                if found >= 0:
                    break
            frontier = nxt
        if found < 0:
            return None  # Hall violated: g0 cannot be filled
        o = found
        while True:
            g = parent[o]
            prev = match_gap[g]
            match_gap[g] = o
            match_op[o] = g
            if prev < 0:
                break
            o = prev
    return match_gap


def _setup(recs, v0, init, cutoff):
    """Split one key's records into the pinned skeleton and the optional ops.
    Raises _NA when the procedure does not apply; returns None when the
    skeleton is already inconsistent."""
    pinned = {}          # position -> (f, value, expected, call, ret)
    optional = []        # (f, value, expected, call, pos or None)
    a = {}               # version index k -> max read call
    b = {}               # position k -> min read ret (reads of version V0+k+1)
    claim = {}           # version index k -> value
    max_read = -1
    for ri, (f, value, expected, ver, call, ret) in enumerate(recs):
        if f not in (0, 1, 2):
            raise _NA
        if cutoff is not None:
            if call > cutoff:
                continue
            if ret > cutoff:
                ret = INF  # pending at the cut: optional
        if f == 0:
            if ret == INF or (ver == -1 and value == -1):
                continue  # an optional read never has to be placed
            if ver == -1:
                raise _NA
            k = ver - v0
            if k < 0:
                return None
            max_read = max(max_read, k)
            a[k] = max(a.get(k, -1), call)
            if k > 0:
                b[k - 1] = min(b.get(k - 1, INF), ret)
            if value != -1:
                if claim.get(k, value) != value:
                    return None
                claim[k] = value
        elif ret == INF:
            pos = None if ver == -1 else ver - v0 - 1
            if pos is not None and pos < 0:
                continue  # can never be linearized: leave it out
            optional.append((f, value, expected if f == 2 else None, call, pos, ri))
        else:
            if ver == -1:
                raise _NA
            pos = ver - v0 - 1
            if pos < 0 or pos in pinned:
                return None
            pinned[pos] = (f, value, expected if f == 2 else None, call, ret, ri)
    m = max(max(pinned) + 1 if pinned else 0, max_read)
    return pinned, optional, a, b, claim, m


def decide(recs, v0=0, init=-1, cutoff=None, budget=10000, witness=False):
    if not witness:
        return _decide(recs, v0, init, cutoff, budget, None)
    w = [-1] * len(recs)
    return _decide(recs, v0, init, cutoff, budget, w), w


def _decide(recs, v0, init, cutoff, budget, wit):
    try:
        st = _setup(recs, v0, init, cutoff)
    except _NA:
        return None
    if st is None:
        return 0
    pinned, optional, a, b, claim, m = st
    if wit is not None:
        for k, p in pinned.items():
            wit[p[5]] = k
    # suffix-min deadlines
    u = [min(b.get(k, INF), pinned[k][4] if k in pinned else INF) for k in range(m)]
    uh = [INF] * (m + 1)
    for k in range(m - 1, -1, -1):
        uh[k] = min(u[k], uh[k + 1])
    gaps = [k for k in range(m) if k not in pinned]
    for k in range(m):
        lo = a.get(k, -1)
        if k in pinned:
            lo = max(lo, pinned[k][3])
        if lo >= uh[k]:
            return 0
    # value requirements: claims of version V0+k+1 and the next pinned CAS
    req = {}
    if claim.get(0, init) != init:
        return 0
    if 0 in pinned and pinned[0][0] == 2 and pinned[0][2] != init:
        return 0
    for k in range(m):
        r = claim.get(k + 1, ANY)
        nxt = pinned.get(k + 1)
        if nxt is not None and nxt[0] == 2:
            if r is not ANY and r != nxt[2]:
                return 0
            r = nxt[2]
        if k in pinned:
            if r is not ANY and r != pinned[k][1]:
                return 0
        else:
            req[k] = r
    if not gaps:
        return 1
    if len(gaps) > len(optional):
        return 0
    nodes = [0]

    def val_before(k, req):
        """Known value at version V0+k (before position k), or ANY."""
        if k == 0:
            return init
        if k - 1 in pinned:
            return pinned[k - 1][1]
        return req[k - 1]

    def solve(req):
        nodes[0] += 1
        if nodes[0] > budget:
            raise _NA
        elig = []
        for k in gaps:
            before = val_before(k, req)
            lst = []
            for i, (f, value, exp, call, pos, _) in enumerate(optional):
                if call >= uh[k] or (pos is not None and pos != k):
                    continue
                if req[k] is not ANY and value != req[k]:
                    continue
                if f == 2 and before is not ANY and exp != before:
                    continue
                lst.append(i)
            elig.append(lst)
        mg = _matching(len(gaps), elig, len(optional))
        if mg is None:
            return False
        # the relaxation ignored CAS expectations after free gaps: check them
        for gi, k in enumerate(gaps):
            f, _, exp, _, _, _ = optional[mg[gi]]
            if f != 2 or val_before(k, req) is not ANY:
                continue
            # k-1 is a free gap; the op placed there fixes the value
            placed = optional[mg[gi - 1]][1]
            if placed == exp:
                continue
            # branch on the value of gap k-1
            cands = sorted({optional[o][1] for o in elig[gi - 1]})
            for v in cands:
                r2 = dict(req)
                r2[k - 1] = v
                if solve(r2):
                    return True
            return False
        if wit is not None:
            for gi, k in enumerate(gaps):
                wit[optional[mg[gi]][5]] = k
        return True

    try:
        return 1 if solve(req) else 0
    except _NA:
        return None


def first_failure(recs, v0=0, init=-1, budget=10000):
    """(fail_op, ret) of the canonical counterexample, or None if valid /
    not applicable.  Bisection over the :ok returns."""
    if decide(recs, v0, init, budget=budget) != 0:
        return None
    rets = sorted((ret, i) for i, (_, _, _, _, _, ret) in enumerate(recs) if ret != INF)
    lo, hi = 0, len(rets) - 1  # prefix at rets[hi] fails (the whole history)
    while lo < hi:
        mid = (lo + hi) // 2
        d = decide(recs, v0, init, cutoff=rets[mid][0], budget=budget)
        if d is None:
            return None
        if d == 0:
            hi = mid
        else:
            lo = mid + 1
    return rets[lo][1], rets[lo][0]
