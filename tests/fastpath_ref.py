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
