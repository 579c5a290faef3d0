"""Python restatement of the GPU's version-order decision procedure
(check_kernel.hip, "Version-order fast tier") — test infrastructure, used to
check the procedure itself against the oracle's searches on the CPU.

Returns 1 (valid), 0 (invalid), or None (not decidable: a crashed write/CAS,
a nil version on an :ok write/CAS, or a read [nil x])."""
INF = (1 << 63) - 1


def decide(recs, v0=0, init=-1):
    n = len(recs)
    lm, um, val, exp = {}, {}, {}, {}
    rl, ru, claim = {}, {}, {}
    for (f, value, expected, ver, call, ret) in recs:
        if f not in (0, 1, 2):
            return None
        if f == 0:
            if ret == INF or (ver == -1 and value == -1):
                continue
            if ver == -1:
                return None
            k = ver - v0
            if k < 0 or k > n:
                return 0
            rl[k] = max(rl.get(k, -1), call)
            ru[k] = min(ru.get(k, INF), ret)
            if value != -1:
                if k in claim and claim[k] != value:
                    return 0
                claim[k] = value
        else:
            if ret == INF or ver == -1:
                return None
            pos = ver - v0 - 1
            if pos < 0 or pos >= n or pos in lm:
                return 0
            lm[pos], um[pos], val[pos] = call, ret, value
            exp[pos] = expected if f == 2 else None
    m = len(lm)
    if m and max(lm) != m - 1:
        return 0
    pm = -1
    for k in range(m):
        pm = max(pm, lm[k], rl.get(k, -1))
        if pm >= min(um[k], ru.get(k + 1, INF)):
            return 0
        before = init if k == 0 else val[k - 1]
        if exp[k] is not None and exp[k] != before:
            return 0
    for k, v in claim.items():
        if k > m or v != (init if k == 0 else val[k - 1]):
            return 0
    if any(k > m for k in list(rl) + list(ru)):
        return 0
    return 1


def first_failure(recs, v0=0, init=-1):
    """The GPU's first-failure rule (check_kernel.hip, `first_failure`) for
    a key the version order decides invalid: the canonical fail op (the :ok
    op whose return empties knossos.linear's frontier) in O(n) instead of a
    bisection over prefixes.

    Returns (fail_op, witness) — witness[r] = the mutation position of record
    r in a linearization of the prefix just before the failing return, -1
    when r is not linearized as a mutation — or None where the rule does not
    decide (ineligible key, an ambiguous choice between two mutations that
    claim one version, or no violation found)."""
    n = len(recs)
    for (f, value, expected, ver, call, ret) in recs:
        if f not in (0, 1, 2):
            return None
        if f == 0 and ret != INF and ver == -1 and value != -1:
            return None
        if f != 0 and (ret == INF or ver == -1):
            return None
    mut = [i for i, r in enumerate(recs) if r[0] != 0]
    reads = [i for i, r in enumerate(recs) if r[0] == 0 and r[5] != INF and r[3] != -1]
    t = INF
    # m*: per position, the mutation returning first; the others of that
    # position return later and make two mutations required at once
    star = {}
    for i in mut:
        pos = recs[i][3] - v0 - 1
        if pos < 0 or pos >= n:
            t = min(t, recs[i][5])
            continue
        if pos not in star or recs[i][5] < recs[star[pos]][5]:
            star[pos] = i
    others = []
    for i in mut:
        pos = recs[i][3] - v0 - 1
        if 0 <= pos < n and star[pos] != i:
            t = min(t, recs[i][5])
            others.append((i, pos))
    # N(p): the first return at which position p is needed (suffix minimum
    # of the returns of the ops needing more than p positions)
    nr = [INF] * (n + 2)
    for i in mut:
        pos = recs[i][3] - v0 - 1
        if 0 <= pos < n:
            nr[pos + 1] = min(nr[pos + 1], recs[i][5])
    for i in reads:
        k = recs[i][3] - v0
        if k < 0 or k > n:
            t = min(t, recs[i][5])
        elif k >= 1:
            nr[k] = min(nr[k], recs[i][5])
    need = [INF] * (n + 1)
    run = INF
    for q in range(n, -1, -1):
        need[q] = run          # N(q) = min nr[q+1 ..]
        run = min(run, nr[q])
    # U side: B[k] = min(ret(m*_k), rets of reads of version v0+k+1); Uh its
    # suffix minimum
    b = [INF] * (n + 1)
    for pos, i in star.items():
        b[pos] = min(b[pos], recs[i][5])
    for i in reads:
        k = recs[i][3] - v0
        if 1 <= k <= n:
            b[k - 1] = min(b[k - 1], recs[i][5])
    uh = [INF] * (n + 2)
    for k in range(n, -1, -1):
        uh[k] = min(b[k], uh[k + 1])
    val = {pos: recs[i][1] for pos, i in star.items()}
    for p in range(n):
        if need[p] != INF and (p not in star or recs[star[p]][4] > need[p]):
            t = min(t, need[p])   # needed before any mutation of it was called
    for p, i in star.items():
        f, value, expected, ver, call, ret = recs[i]
        if f == 2:
            before = init if p == 0 else val.get(p - 1)
            if before is not None and before != expected:
                t = min(t, need[p])
        if call >= uh[p]:
            t = min(t, need[p])
    for i in reads:
        f, value, expected, ver, call, ret = recs[i]
        k = ver - v0
        if k < 0 or k > n:
            continue
        if value != -1:
            before = init if k == 0 else val.get(k - 1)
            if before is not None and before != value:
                t = min(t, ret)
        if k < n and call >= uh[k]:
            t = min(t, ret)
    if t == INF:
        return None
    for i, p in others:  # a choice between two called mutations at a needed position
        if recs[i][4] < t and need[p] <= t < recs[star[p]][5]:
            return None
    fo = [i for i, r in enumerate(recs) if r[5] == t]
    wit = [-1] * n
    for p, i in star.items():
        if need[p] < t:
            wit[i] = p
    return fo[0], wit
