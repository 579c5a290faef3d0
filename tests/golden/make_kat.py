"""Writes tests/golden/kat.json: hand-derived known-answer histories for the
VersionedRegister model (register.clj:59-96) under the linearizability
definition of SURVEY.md §8a.  Every expected verdict / fail op below was
derived by hand from the step rules, NOT computed by any checker; the tests
check all oracles (brute force, JIT, WGL) and the GPU against them.

Record = [f, value, expected, version, call, ret]; f 0 read / 1 write / 2 cas;
-1 = nil; INF = never returned (:info).  fail_op = index (by call order) of
the :ok op whose return empties the frontier (the canonical counterexample).
"""
import json
import os

R, W, C = 0, 1, 2
N = -1
INF = (1 << 63) - 1

KATS = [
    # name, records, valid, fail_op, note
    ("kat1_sequential", [[W, 1, N, 1, 0, 1], [R, 1, N, 1, 2, 3], [C, 3, 1, 2, 4, 5], [R, 3, N, 2, 6, 7]],
     True, -1, "w1 ok [1 1]; r ok [1 1]; cas(1->3) ok [2 [1 3]]; r ok [2 3] (SURVEY KAT1)"),
    ("kat2_stale_read", [[W, 1, N, 1, 0, 1], [W, 2, N, 2, 2, 3], [R, 1, N, 1, 4, 5]],
     False, 2, "read invoked after w2 returned sees version 1 (KAT2)"),
    ("kat3_concurrent_read", [[R, 1, N, 1, 0, 2], [W, 1, N, 1, 1, 3]],
     True, -1, "read overlaps the write it observes (KAT3)"),
    ("kat4a_info_fills_gap", [[W, 1, N, N, 0, INF], [W, 2, N, 2, 1, 2]],
     True, -1, "crashed w1 supplies version 1 before w2 [2 2] (KAT4)"),
    ("kat4b_info_too_late", [[W, 2, N, 2, 0, 1], [W, 1, N, N, 2, INF]],
     False, 0, "w2 [2 2] returns before the crashed write is invoked (KAT4)"),
    ("kat5_nil_read", [[R, N, N, N, 0, 1], [W, 1, N, 1, 2, 3], [R, N, N, N, 4, 5]],
     True, -1, "[nil nil] reads are unconstrained (KAT5, register.clj:26-27)"),
    ("kat6_cas_on_nil", [[C, 1, 0, 1, 0, 1]],
     False, 0, "cas(0->1) on a fresh key: value nil != 0 (KAT6, register.clj:77)"),
    ("kat7_lost_cas", [[W, 0, N, 1, 0, 1], [C, 3, 0, 2, 2, 3], [R, 0, N, 2, 4, 5]],
     False, 2, "read [2 0] after cas(0->3) ok [2 ...] (KAT7)"),
    ("kat8_fail_dropped", [[W, 1, N, 1, 0, 1], [R, 1, N, 1, 4, 5]],
     True, -1, "a :fail cas between them was dropped by history completion (KAT8)"),
    ("kat9_duplicate_version", [[W, 1, N, 1, 0, 1], [W, 2, N, 1, 2, 3]],
     False, 1, "two sequential writes both report version 1 (KAT9)"),
    ("kat11_cas_nil_expected", [[C, 1, N, 1, 0, 1]],
     True, -1, "cas(nil->1): (not= nil nil) is false, so it applies (register.clj:77)"),
    ("kat12_version_only_read", [[W, 3, N, 1, 0, 1], [R, N, N, 1, 2, 3]],
     True, -1, "read [1 nil] checks the version only (register.clj:84-93)"),
    ("kat13_versions_order_writes", [[W, 5, N, 2, 0, 3], [W, 7, N, 1, 1, 2], [R, 5, N, 2, 4, 5]],
     True, -1, "w7 [1 7] must precede w5 [2 5] although invoked later"),
    ("kat14_read_overwritten", [[W, 5, N, 2, 0, 3], [W, 7, N, 1, 1, 2], [R, 7, N, 1, 4, 5]],
     False, 2, "read [1 7] invoked after both writes returned"),
    ("kat15_info_cas_applies", [[W, 0, N, 1, 0, 1], [C, 4, 0, N, 2, INF], [R, 4, N, 2, 3, 4]],
     True, -1, "crashed cas(0->4) took effect"),
    ("kat16_info_cas_cannot", [[W, 1, N, 1, 0, 1], [C, 4, 0, N, 2, INF], [R, 4, N, 2, 3, 4]],
     False, 2, "crashed cas(0->4) cannot apply to value 1"),
    ("kat17_read_from_future", [[R, 1, N, 1, 0, 1], [W, 1, N, 1, 2, 3]],
     False, 0, "read returns a value whose write is invoked later"),
    ("kat19_empty", [], True, -1, "empty subhistory"),
    ("kat20_concurrent_dup_version", [[W, 1, N, 1, 0, 3], [W, 2, N, 1, 1, 2]],
     False, 0, "overlapping writes both claim version 1: w2 returns first, w1 cannot follow"),
    ("kat21_info_read_ignored", [[W, 1, N, 1, 0, 1], [R, 3, N, 7, 2, INF]],
     True, -1, "a crashed read never constrains (its completion value is unknown)"),
    ("kat22_cas_chain", [[W, 0, N, 1, 0, 1], [C, 1, 0, 2, 2, 5], [C, 2, 1, 3, 3, 6], [R, 2, N, 3, 7, 8]],
     True, -1, "overlapping cas chain 0->1->2"),
    ("kat23_cas_chain_wrong_order", [[W, 0, N, 1, 0, 1], [C, 2, 1, 2, 2, 3], [C, 1, 0, 3, 4, 5]],
     False, 1, "cas(1->2) [2 ...] returns before cas(0->1) is invoked"),
]

if __name__ == "__main__":
    out = [{"name": n, "ops": ops, "valid": v, "fail_op": f, "note": note,
            "fail_prefix_end": (ops[f][5] if f >= 0 else -1)}
           for (n, ops, v, f, note) in KATS]
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat.json")
    with open(p, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", p, len(out))
