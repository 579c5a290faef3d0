"""Dev: the last --n dispatches of a rocprofv3 --kernel-trace CSV in order,
with each one's start (µs from the first listed), duration and the idle gap
before it.

    python tools/kt_timeline.py gpurun_out/.../kt_kernel_trace.csv [--n 40]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--n", type=int, default=40)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
                         .replace("lcdev::", ""),
                         r.get("Grid_Size", ""), r.get("Workgroup_Size", "")))
    rows.sort()
    rows = rows[-a.n:]
    t0 = rows[0][0]
    prev = t0
    for s, e, n, g, w in rows:
        print("%9.1f  %8.1f us  gap %7.1f  %-36s grid %s wg %s" %
              ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, n[:36], g, w))
        prev = max(prev, e)


if __name__ == "__main__":
    main()
