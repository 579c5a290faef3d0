"""Dev: where a frontier-exchange check's wall time goes, from a rocprofv3
--kernel-trace CSV of tools/fx_once.py: per kernel the dispatches, busy time
and the idle gap before each dispatch (GPU idle: the host's round trips),
over the last check (the dispatches after the last long idle gap > 5 ms,
which separates the checks).  Empty expand levels are the dispatches
shorter than --empty-ns.

    python tools/fx_gaps.py gpurun_out/fxkt/<pid>_kernel_trace.csv
"""
import argparse
import csv
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--empty-ns", type=int, default=2500)
    ap.add_argument("--split-ms", type=float, default=5.0)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # the checks: runs of dispatches separated by > split-ms idle
    start = 0
    for i in range(1, len(rows)):
        if rows[i][0] - rows[i - 1][1] > a.split_ms * 1e6:
            start = i
    gaps = sorted(((rows[i][0] - rows[i - 1][1]) / 1e6, i) for i in range(1, len(rows)))[-5:]
    print("largest idle gaps (ms, at dispatch):", ["%.2f@%d" % g for g in gaps])
    rows = rows[start:]
    wall = (rows[-1][1] - rows[0][0]) / 1e6
    busy = collections.Counter()
    calls = collections.Counter()
    gap = collections.Counter()
    empty = 0
    empty_ns = 0
    prev_end = rows[0][0]
    hist = collections.Counter()
    for s, e, n in rows:
        k = n.replace("(anonymous namespace)::", "").split("(")[0]
        calls[k] += 1
        busy[k] += e - s
        gap[k] += max(0, s - prev_end)
        prev_end = max(prev_end, e)
        if k.endswith("fx_expand_kernel"):
            hist[min((e - s) // 1000, 40)] += 1
            if e - s < a.empty_ns:
                empty += 1
                empty_ns += e - s
    print("last check: %d dispatches, wall %.2f ms, busy %.2f ms, idle %.2f ms" %
          (len(rows), wall, sum(busy.values()) / 1e6, sum(gap.values()) / 1e6))
    for k in sorted(busy, key=lambda x: -busy[x]):
        print("  %-40s %6d  busy %8.3f ms (avg %6.2f us)  idle before %8.3f ms" %
              (k, calls[k], busy[k] / 1e6, busy[k] / calls[k] / 1e3, gap[k] / 1e6))
    print("expand launches < %d ns: %d, %.3f ms" % (a.empty_ns, empty, empty_ns / 1e6))
    print("expand duration histogram (us: count):",
          " ".join("%d:%d" % (b, hist[b]) for b in sorted(hist)))


if __name__ == "__main__":
    main()
