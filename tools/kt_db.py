"""Summarise a rocprofv3 results.db kernel trace: per kernel count, total,
mean, p50, p90, and for one kernel the durations by grid size."""
import collections
import sqlite3
import sys

import numpy as np

db = sys.argv[1]
focus = sys.argv[2] if len(sys.argv) > 2 else None
c = sqlite3.connect(db)
rows = c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
d = collections.defaultdict(list)
for n, s, e, g, wg in rows:
    d[n.split("(")[0][-40:]].append((e - s) / 1e3)
for n, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    t = np.array(v)
    print("%-40s n %6d total ms %8.2f mean us %7.2f p50 %7.2f p90 %7.2f max %8.1f"
          % (n, len(t), t.sum() / 1e3, t.mean(), np.median(t), np.percentile(t, 90), t.max()))
if focus:
    sel = [(s, e, g // max(wg, 1)) for n, s, e, g, wg in rows if focus in n]
    if sel:
        st = np.array([x[0] for x in sel]); en = np.array([x[1] for x in sel]); gs = np.array([x[2] for x in sel])
        dur = (en - st) / 1e3
        gaps = (st[1:] - en[:-1]) / 1e3
        print("%s: idle gap between launches mean us %.1f p50 %.1f total ms %.1f"
              % (focus, gaps.mean(), np.median(gaps), gaps.sum() / 1e3))
        for lo, hi in ((1, 1), (2, 8), (9, 32), (33, 64), (65, 256), (257, 1 << 20)):
            m = (gs >= lo) & (gs <= hi)
            if m.any():
                print("  grid %4d-%-7d n %5d mean us %7.1f total ms %7.1f"
                      % (lo, hi, m.sum(), dur[m].mean(), dur[m].sum() / 1e3))
