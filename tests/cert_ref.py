"""Python restatement of the device's certificate finder (cert_kernel in
jepsen/etcd_amd/csrc/cert.hip) — test infrastructure.  Given an invalid
key's records and its failing return `cut`, name facts that rule out every
linearization of the prefix at `cut` (the kinds of include/lincheck.h,
LC_CERT_*).  oracle/cert.c checks what either finder emits from the records
alone; a finder can only fail to find a certificate, never make a wrong one
pass.

find(recs, cut) -> (kind, a, b, c, positions)."""
INF = (1 << 63) - 1
NIL = -1
R, W, C = 0, 1, 2
NONE, DUP, UNREACH, CLAIMS, PAIR, ORDER, HALL, PROOF = range(8)
# PROOF tokens (include/lincheck.h LC_CERT_PROOF): kind << 30 | a << 15 | b
FORCE, BRANCH, EMPTY = 1, 2, 3
PROOF_NODES = 2048  # search budget (the device finder's, cert.hip)


def tok(kind, a, b=0):
    """One proof token as the int32 the certificate set holds."""
    x = (kind << 30) | (a << 15) | b
    return x - (1 << 32) if x >= (1 << 31) else x


def untok(t):
    t &= 0xFFFFFFFF
    return t >> 30, (t >> 15) & 0x7FFF, t & 0x7FFF


def find(recs, cut, v0=0, init=-1, proof=True, proof_budget=PROOF_NODES):
    n = len(recs)
    inp = [r[4] <= cut for r in recs]
    req = [inp[i] and recs[i][5] <= cut for i in range(n)]
    mut = [r[0] in (W, C) for r in recs]
    pin = [mut[i] and recs[i][3] != NIL for i in range(n)]
    n_mut = sum(1 for i in range(n) if inp[i] and mut[i])
    pos = [recs[i][3] - v0 - 1 if pin[i] else None for i in range(n)]
    held, claim, reads_at, m_need = {}, {}, {}, 0
    for i, (f, val, exp, ver, call, ret) in enumerate(recs):
        if not req[i]:
            continue
        if pin[i]:
            if pos[i] < 0 or ver - v0 > n_mut:
                return (UNREACH, i, -1, 0, [])
            if pos[i] in held:
                return (DUP, held[pos[i]], i, 0, [])
            held[pos[i]] = i
            m_need = max(m_need, pos[i] + 1)
        elif f == R and ver != NIL:
            k = ver - v0
            if k < 0 or k > n_mut or (k == 0 and val != NIL and val != init):
                return (UNREACH, i, -1, 0, [])
            m_need = max(m_need, k)
            reads_at.setdefault(k, []).append(i)
            if val != NIL:
                if k in claim and recs[claim[k]][1] != val:
                    return (CLAIMS, claim[k], i, 0, [])
                claim.setdefault(k, i)
    # fixed value pairs: a required holder and a required consumer
    for q, b in sorted(held.items()):
        if recs[b][0] != C:
            continue
        if q == 0 and recs[b][2] != init:
            return (PAIR, -1, b, q, [])
        if q >= 1 and q - 1 in held and recs[held[q - 1]][1] != recs[b][2]:
            return (PAIR, held[q - 1], b, q, [])
    for k, b in sorted(claim.items()):
        if k >= 1 and k - 1 in held and recs[held[k - 1]][1] != recs[b][1]:
            return (PAIR, held[k - 1], b, k, [])
    # timing: lower bound at index j (a mutation at j, a read of v0+j) after
    # the return of an op bounding index >= j from above
    lo = {}
    for i in range(n):
        if not req[i]:
            continue
        j = pos[i] if pin[i] else (recs[i][3] - v0 if recs[i][0] == R and recs[i][3] != NIL else None)
        if j is not None and (j not in lo or recs[i][4] > recs[lo[j]][4]):
            lo[j] = i
    up = {}
    for i in range(n):
        if not req[i]:
            continue
        k = pos[i] if pin[i] else (recs[i][3] - v0 - 1 if recs[i][0] == R and recs[i][3] != NIL else None)
        if k is not None and k >= 0 and (k not in up or recs[i][5] < recs[up[k]][5]):
            up[k] = i
    best = None
    for k in range(max(list(up) + [0]), -1, -1):   # suffix minimum of the upper bounds
        if k in up and (best is None or recs[up[k]][5] < recs[best][5]):
            best = up[k]
        if k in lo and best is not None and recs[lo[k]][4] > recs[best][5]:
            return (ORDER, lo[k], best, 0, [])
    # the open positions: needed, held by no required op
    gaps = [p for p in range(m_need) if p not in held]
    cands = {}

    def before(p):
        if p == 0:
            return True, init
        if p - 1 in held:
            return True, recs[held[p - 1]][1]
        if p in claim:
            return True, recs[claim[p]][1]
        return False, None

    for p in gaps:
        dl = INF
        for i in range(n):
            if not req[i]:
                continue
            if (pin[i] and pos[i] > p) or (recs[i][0] == R and recs[i][3] != NIL and
                                           recs[i][3] - v0 - 1 >= p):
                dl = min(dl, recs[i][5])
        wants = set()
        if p + 1 in claim:
            wants.add(recs[claim[p + 1]][1])
        if p + 1 in held and recs[held[p + 1]][0] == C:
            wants.add(recs[held[p + 1]][2])
        det, bv = before(p)
        cs = []
        if len(wants) <= 1:
            for x in range(n):
                if not inp[x] or not mut[x] or (req[x] and pin[x]):
                    continue
                if pin[x] and pos[x] != p:
                    continue
                if recs[x][4] >= dl:
                    continue
                if recs[x][0] == C and det and recs[x][2] != bv:
                    continue
                if wants and recs[x][1] not in wants:
                    continue
                cs.append(x)
        cands[p] = cs
        if not cs:
            return (HALL, -1, -1, 1, [p])
    # forced pairs: a CAS that is the only op able to hold q after the only
    # op able to hold q-1 (or a required one), with another value
    for q in gaps:
        if len(cands[q]) != 1 or recs[cands[q][0]][0] != C:
            continue
        b = cands[q][0]
        if q == 0:
            continue  # (the initial value is fixed: the filter above applies)
        a = held.get(q - 1)
        if a is None and q - 1 in cands and len(cands[q - 1]) == 1:
            a = cands[q - 1][0]
        if a is not None and recs[a][1] != recs[b][2]:
            return (PAIR, a, b, q, [])
    union = set()
    for p in gaps:
        union.update(cands[p])
    if len(union) < len(gaps):
        return (HALL, -1, -1, len(gaps), gaps)
    # Infeasibility that only a search finds (a choice at one open position
    # fixes the value or uses the op another one needs): a proof by forced
    # choices and case splits over the candidates (LC_CERT_PROOF), as the
    # device's finder searches for it (cert.hip, prove)
    toks = (prove(recs, gaps, held, claim, inp, req, mut, pin, pos, v0, init, proof_budget)
            if proof else None)
    if toks is not None and len(toks) <= n and max(gaps) < 1 << 15 and n <= 1 << 15:
        return (PROOF, -1, -1, len(toks), toks)
    return (NONE, -1, -1, 0, [])


def prove(recs, gaps, held, claim, inp, req, mut, pin, pos, v0, init, budget=PROOF_NODES):
    """The proof's tokens — one BRANCH(position, cases) per case split, in
    preorder — or None (a complete consistent assignment exists, or the
    search ran over its budget).  Between splits the open positions are
    propagated (the checker re-derives this): a position with no candidate
    closes the case, else the lowest one with exactly one is assumed held by
    it; a split is taken at the open position with the fewest candidates
    (the lowest among equals), its cases in increasing record order."""
    n = len(recs)
    dl, base_before, base_wants, S = {}, {}, {}, {}
    for p in gaps:
        d = INF
        for i in range(n):
            if req[i] and ((pin[i] and pos[i] > p) or (recs[i][0] == R and recs[i][3] != NIL and
                                                        recs[i][3] - v0 - 1 >= p)):
                d = min(d, recs[i][5])
        dl[p] = d
        if p == 0:
            base_before[p] = (True, init)
        elif p - 1 in held:
            base_before[p] = (True, recs[held[p - 1]][1])
        elif p in claim:
            base_before[p] = (True, recs[claim[p]][1])
        else:
            base_before[p] = (False, None)
        w = set()
        if p + 1 in claim:
            w.add(recs[claim[p + 1]][1])
        if p + 1 in held and recs[held[p + 1]][0] == C:
            w.add(recs[held[p + 1]][2])
        base_wants[p] = w
        S[p] = [x for x in range(n) if inp[x] and mut[x] and not (req[x] and pin[x]) and
                (not pin[x] or pos[x] == p) and recs[x][4] < d]

    def cands(p, asg, used):
        wants = set(base_wants[p])
        if p + 1 in asg and recs[asg[p + 1]][0] == C:
            wants.add(recs[asg[p + 1]][2])
        if len(wants) > 1:
            return []
        det, bv = base_before[p]
        if not det and p - 1 in asg:
            det, bv = True, recs[asg[p - 1]][1]
        return [x for x in S[p] if x not in used and not (recs[x][0] == C and det and recs[x][2] != bv)
                and not (wants and recs[x][1] not in wants)]

    nodes = [0]

    def search(asg, used):
        nodes[0] += 1
        if nodes[0] > budget:
            return None
        asg, used = dict(asg), set(used)
        while True:
            open_ = [p for p in gaps if p not in asg]
            if not open_:
                return None  # every open position held: no contradiction here
            cs = {p: cands(p, asg, used) for p in open_}
            if any(not cs[p] for p in open_):
                return []    # the case closes
            one = [p for p in open_ if len(cs[p]) == 1]
            if one:          # forced (the checker re-derives it)
                p = one[0]
                asg[p] = cs[p][0]
                used.add(cs[p][0])
                continue
            p = min(open_, key=lambda q: (len(cs[q]), q))
            out = [tok(BRANCH, p, len(cs[p]))]
            for o in cs[p]:
                a2 = dict(asg)
                a2[p] = o
                sub = search(a2, used | {o})
                if sub is None:
                    return None
                out += sub
            return out

    return search({}, set())
