"""Dev: broad differential fuzz, GPU vs the oracle, over random histories:
tiny random keys (brute-force sized), synthetic register keys across crash and
anomaly rates and concurrencies (each also as 24-byte records through lc_check32,
field for field against the 48-byte call), version-stripped keys (cas-register), mutex
and cas-register record generators, and the frontier exchange (one and three
ranks) on version-less keys.  Prints mismatches; exits 1 on any.
    python tools/fuzz_gpu.py [rounds]"""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import oracle  # noqa: E402
from helpers import pack_keys, random_casreg, random_mutex, tiny_batch  # noqa: E402
from jepsen.etcd_amd import abi  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
bad_total = 0
t_start = time.time()
# invalid version-pinned keys (PREFIX witness) and those the certificate
# finder left without a certificate (its PROOF search over its node or work
# cap, cert.hip; certified on the witness side only)
cert_totals = {"invalid_witnessed": 0, "no_certificate": 0}


def compare(tag, ops, off, opts=None, algo=oracle.JITC, budget=1 << 18):
    global bad_total
    with abi.Context(device_mask=1) as ctx:
        _, g = ctx.check(ops, off, opts)
        # the same batch as 24-byte records (lc_check32's native pass) and as
        # 16-byte records (lc_check16): every result field equal to the
        # 48-byte call's
        o32, b32 = abi.pack32(ops, off)
        _, g32 = ctx.check32(o32, off, b32, opts)
        p16 = abi.pack16(ops, off)
        g16 = ctx.check16(p16[0], off, p16[1], opts)[1] if p16 is not None else g
        # witnesses and certificates: every certificate the checker reads
        # must hold (never CERT_BAD); count the invalid keys left without one
        _, gc, _, kind, cert, cset = ctx.check(ops, off, opts, witness=True, certificate=True)
    n32 = int((g32 != g).sum()) + int((g16 != g).sum()) + int((gc != g).sum())
    st = oracle.check_certificate(ops, off, cert.reshape(-1), cset, gc, n_threads=16)
    n32 += int((st == oracle.CERT_BAD).sum())
    invw = (gc["verdict"] == 0) & (kind == abi.LC_WITNESS_PREFIX)
    cert_totals["invalid_witnessed"] += int(invw.sum())
    cert_totals["no_certificate"] += int((invw & (cert[:, 0] == abi.LC_CERT_NONE)).sum())
    _, o = oracle.check(ops, off, algo=algo, n_threads=16, max_configs=budget,
                        init_version=opts.init_version if opts is not None else 0,
                        init_value=opts.init_value if opts is not None else -1)
    known = (o["verdict"] != -1) & (g["verdict"] != -1)
    diff = g["verdict"] != o["verdict"]
    if algo != oracle.WGL:  # WGL gives verdicts only
        diff |= g["fail_op"] != o["fail_op"]
    bad = np.nonzero(known & diff)[0]
    gpu_unknown = int(((g["verdict"] == -1) & (o["verdict"] != -1)).sum())
    print("%-34s keys %5d decided %5d gpu-only-unknown %3d mismatches %d 32/16-bit+cert %d "
          "invalid-witnessed %d no-cert %d (%.0fs)"
          % (tag, len(off) - 1, int(known.sum()), gpu_unknown, len(bad), n32, int(invw.sum()),
             int((invw & (cert[:, 0] == abi.LC_CERT_NONE)).sum()), time.time() - t_start),
          flush=True)
    for k in bad[:5]:
        print("   key", int(k), "gpu", g[k].tolist(), "oracle", int(o["verdict"][k]), int(o["fail_op"][k]))
    bad_total += len(bad) + n32


for rd in range(rounds):
    base = 1000 * rd + 17
    ops, off = pack_keys(tiny_batch(base, 4000, max_ops=7))
    compare("tiny r%d" % rd, ops, off)
    for conc, pinf, pan, opk in ((4, 0.3, 0.5, 40), (8, 0.2, 0.4, 80), (12, 0.1, 0.3, 150),
                                 (20, 0.05, 0.3, 300), (6, 0.0, 0.5, 500)):
        ops, off, _, _ = abi.synth(300, opk, concurrency=conc, p_info=pinf, p_anomaly=pan,
                                   seed=base + conc)
        compare("synth c%d i%.2f a%.1f n%d r%d" % (conc, pinf, pan, opk, rd), ops, off)
        ops2 = ops.copy()
        ops2[:, 3] = -1
        if pinf <= 0.1 and conc <= 8:
            compare("unversioned c%d n%d r%d" % (conc, opk, rd), ops2, off, algo=oracle.WGL)
            compare("unversioned-jit c%d n%d r%d" % (conc, opk, rd), ops2, off)
    # few long crash-heavy keys: full-history decision + multisection probes
    # (beyond the oracle: checked against the restated procedure)
    import gapmatch_ref as gm
    ops, off, _, _ = abi.synth(6, 1500, concurrency=24, p_info=0.1, p_anomaly=0.7, seed=base + 99)
    with abi.Context(device_mask=1) as ctx:
        _, g = ctx.check(ops, off)
    nbad = 0
    for k in range(6):
        recs = [tuple(r) for r in ops[off[k]:off[k + 1]].tolist()]
        want = gm.decide(recs)
        got = (int(g["verdict"][k]), int(g["fail_op"][k]), int(g["fail_prefix_end"][k]))
        exp = (want,) + (gm.first_failure(recs) if want == 0 else (-1, -1))
        if want is not None and got != exp:
            nbad += 1
            print("   long key", k, "gpu", got, "restated", exp)
    print("%-34s keys %5d mismatches %d" % ("long crash-heavy r%d" % rd, 6, nbad), flush=True)
    bad_total += nbad
    # the cooperative tier (LDS pool, value table, packed rounds, deferred
    # frontier updates) against the one-wave tier (HBM tables, serial
    # worklist) on version-less keys: every result field
    for conc, opk, pan in ((10, 300, 0.0), (14, 400, 0.01), (18, 600, 0.0)):
        ops, off, _, _ = abi.synth(96, opk, concurrency=conc, seed=base + 31 * conc)
        ops = ops.copy()
        ops[:, 3] = -1
        if pan:
            rr = np.random.default_rng(base + conc)
            reads = np.nonzero((ops[:, 0] == abi.LC_F_READ) & (ops[:, 5] != abi.LC_INF))[0]
            ops[rr.choice(reads, int(len(reads) * pan), replace=False), 1] = 12345
        co = abi.default_opts(flags=abi.LC_FLAG_NO_GAP_TIER, time_budget_ms=5000)
        res = {}
        for mode in ("0", "1"):
            os.environ["LC_HBM_COOP"] = mode
            with abi.Context(device_mask=1) as ctx:
                res[mode] = ctx.check(ops, off, co)[1]
        del os.environ["LC_HBM_COOP"]
        a, b = res["0"], res["1"]
        done = (a["verdict"] != -1) & (b["verdict"] != -1)
        nbad = 0
        for f in ("verdict", "reason", "fail_op", "fail_prefix_end", "configs_explored", "max_frontier"):
            nbad = max(nbad, int((a[f][done] != b[f][done]).sum()))
        print("%-34s keys %5d decided %5d mismatches %d" % ("coop vs one-wave c%d n%d r%d" % (conc, opk, rd),
                                                            len(off) - 1, int(done.sum()), nbad), flush=True)
        bad_total += nbad
    rng = random.Random(base)
    keys = [random_mutex(rng, rng.randrange(1, 24)) for _ in range(1500)]
    ops, off = pack_keys(keys)
    compare("mutex r%d" % rd, ops, off, abi.default_opts(init_value=0))
    keys = [random_casreg(rng, rng.randrange(1, 24)) for _ in range(1500)]
    ops, off = pack_keys(keys)
    compare("casreg r%d" % rd, ops, off)
    # the frontier exchange (one key at a time): every field against JITC,
    # one rank and three in-process ranks with every level partitioned
    from jepsen.etcd_amd.fx import FrontierExchange
    keys = [random_casreg(rng, rng.randrange(1, 40), p_info=0.1) for _ in range(200)]
    ops, off, _, _ = abi.synth(40, 150, concurrency=8, p_info=0.02, p_anomaly=0.5, seed=base + 7)
    ops = ops.copy()
    ops[:, 3] = -1
    keys += [ops[off[k]:off[k + 1]].tolist() for k in range(40)]
    kops, koff = pack_keys(keys)
    _, o = oracle.check(kops, koff, algo=oracle.JITC, n_threads=16, max_configs=1 << 20)
    fields = ("verdict", "fail_op", "configs_explored", "max_frontier")
    for ranks, pa in ((1, -1), (3, 0)):
        nbad = ndec = 0
        with FrontierExchange(device=0, virtual_ranks=ranks, part_above=pa, table_log2=20) as fx:
            for k in range(len(keys)):
                r = fx.check(kops[koff[k]:koff[k + 1]])
                if (r["verdict"] == -1 and o["verdict"][k] != -1
                        and r["reason"] != abi.LC_REASON_WINDOW_OVERFLOW):
                    # a spurious :unknown is a mismatch too (only the window
                    # bound, which the oracle lacks, may leave a key undecided)
                    nbad += 1
                    print("   fx-only unknown key", k, "reason", int(r["reason"]))
                    continue
                if r["verdict"] == -1 or o["verdict"][k] == -1:
                    continue
                ndec += 1
                if any(int(r[f]) != int(o[f][k]) for f in fields):
                    nbad += 1
                    print("   fx key", k, [int(r[f]) for f in fields], [int(o[f][k]) for f in fields])
        print("%-34s keys %5d decided %5d mismatches %d" % ("fx ranks %d r%d" % (ranks, rd),
                                                            len(keys), ndec, nbad), flush=True)
        bad_total += nbad
    # crash-heavy mutex keys (more crashed acquires / releases than the window
    # holds): counted classes, on one rank and on two with every level partitioned
    from helpers import FREE
    keys = [random_mutex(rng, rng.randrange(100, 300), p_info=0.4, p_perturb=0.5) for _ in range(10)]
    kops, koff = pack_keys(keys)
    _, o = oracle.check(kops, koff, algo=oracle.JITC, n_threads=16, init_value=FREE)
    mo = abi.default_opts(init_value=FREE)
    for ranks, pa in ((1, -1), (2, 0)):
        nbad = ndec = 0
        with FrontierExchange(device=0, virtual_ranks=ranks, part_above=pa, table_log2=18) as fx:
            for k in range(len(keys)):
                r = fx.check(kops[koff[k]:koff[k + 1]], mo)
                if r["verdict"] == -1 or o["verdict"][k] == -1:
                    nbad += int(r["verdict"] != o["verdict"][k])
                    continue
                ndec += 1
                if any(int(r[f]) != int(o[f][k]) for f in fields):
                    nbad += 1
                    print("   fx class key", k, [int(r[f]) for f in fields], [int(o[f][k]) for f in fields])
        print("%-34s keys %5d decided %5d mismatches %d" % ("fx classes ranks %d r%d" % (ranks, rd),
                                                            len(keys), ndec, nbad), flush=True)
        bad_total += nbad
print("certificates: %d invalid witnessed keys, %d left without a certificate (the PROOF search over "
      "its cap)" % (cert_totals["invalid_witnessed"], cert_totals["no_certificate"]))
print("TOTAL mismatches", bad_total)
sys.exit(1 if bad_total else 0)
