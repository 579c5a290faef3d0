"""Per-grid-size durations of one kernel in a rocprofv3 kernel-trace csv:
count, mean, p10, p50, p90 (us) for each grid size (in workgroups).
  python tools/kt_grid.py TRACE.csv KERNEL_SUBSTRING [skip_per_grid]"""
import collections
import csv
import sys

import numpy as np

skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
by = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        wg = max(1, int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 1)) or 1))
        g = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0) // wg
        by[g].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for g in sorted(by):
    t = np.array(by[g][skip:])
    if len(t):
        print("grid %6d n %5d mean %8.2f p10 %8.2f p50 %8.2f p90 %8.2f us"
              % (g, len(t), t.mean(), np.percentile(t, 10), np.median(t), np.percentile(t, 90)))
