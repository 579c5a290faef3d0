"""Per-dispatch duration histogram of one kernel from a rocprofv3 kernel trace.
  python tools/kt_hist.py TRACE.csv KERNEL_SUBSTRING"""
import csv
import sys

d = []
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        d.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
d.sort()
n = len(d)
print("dispatches", n, "total_ms %.1f" % (sum(d) / 1e3))
for q in (0.1, 0.25, 0.5, 0.75, 0.9, 0.99):
    print("p%d %.1f us" % (q * 100, d[int(q * (n - 1))]))
for lo, hi in ((0, 5), (5, 10), (10, 20), (20, 40), (40, 80), (80, 160), (160, 1e9)):
    s = [x for x in d if lo <= x < hi]
    print("[%g, %g) us: %d dispatches, %.1f ms" % (lo, hi, len(s), sum(s) / 1e3))
