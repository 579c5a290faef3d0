"""Summarise tools/pmc_kernel.sh output for one kernel into profiles/.

  python tools/pmc_summary.py gpurun_out/pmc_TAG KERNEL_SUBSTRING OUT.json [ALGO_BYTES]

Per-dispatch medians of every counter over the dispatches of KERNEL (the
largest grid when several grids occur), the kernel-trace average duration,
and derived figures: HBM bytes (FETCH_SIZE x 2 per the gfx950 wide-read
correction + WRITE_SIZE, MI355X_MICROARCH.md "HBM"), achieved GB/s, L2 hit
rate, waits per busy cycle, LDS bank conflicts per LDS instruction.
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict


def main():
    src, kern, dst = sys.argv[1], sys.argv[2], sys.argv[3]
    algo = float(sys.argv[4]) if len(sys.argv) > 4 else None
    vals = defaultdict(list)
    grids = defaultdict(int)
    for f in glob.glob(os.path.join(src, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                grids[int(r["Grid_Size"])] += 1
                vals[(r["Counter_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    grid = max(grids, key=lambda g: (grids[g], g)) if grids else None
    ctr = {k[0]: statistics.median(v) for k, v in vals.items() if k[1] == grid}
    kt = None
    for f in glob.glob(os.path.join(src, "kt", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            if kern in r["Name"]:
                kt = {"name": r["Name"], "calls": int(r["Calls"]),
                      "avg_ns": float(r["AverageNs"]), "total_ns": float(r["TotalDurationNs"])}
    out = {"kernel": kern, "grid_size": grid, "dispatches_per_pass": grids.get(grid),
           "counters_median_per_dispatch": ctr, "kernel_trace": kt}
    d = {}
    if "FETCH_SIZE" in ctr and "WRITE_SIZE" in ctr:
        d["hbm_bytes"] = ctr["FETCH_SIZE"] * 1024 * 2 + ctr["WRITE_SIZE"] * 1024
        if kt:
            d["hbm_gb_per_s"] = d["hbm_bytes"] / kt["avg_ns"]
            d["hbm_frac_of_8tbs"] = d["hbm_gb_per_s"] / 8000.0
    if "TCC_HIT_sum" in ctr and ctr.get("TCC_HIT_sum", 0) + ctr.get("TCC_MISS_sum", 0) > 0:
        d["l2_hit_rate"] = ctr["TCC_HIT_sum"] / (ctr["TCC_HIT_sum"] + ctr["TCC_MISS_sum"])
    if ctr.get("SQ_BUSY_CYCLES"):
        d["wait_any_per_busy_cycle"] = ctr.get("SQ_WAIT_ANY", 0) / ctr["SQ_BUSY_CYCLES"]
    if ctr.get("SQ_WAVE_CYCLES"):
        d["wait_any_frac_of_wave_cycles"] = ctr.get("SQ_WAIT_ANY", 0) / ctr["SQ_WAVE_CYCLES"]
        d["active_inst_frac_of_wave_cycles"] = ctr.get("SQ_ACTIVE_INST_ANY", 0) / ctr["SQ_WAVE_CYCLES"]
    if ctr.get("SQ_INSTS_LDS"):
        d["lds_bank_conflict_cycles_per_lds_inst"] = ctr.get("SQ_LDS_BANK_CONFLICT", 0) / ctr["SQ_INSTS_LDS"]
    if algo and kt:
        d["algorithmic_bytes"] = algo
        d["algorithmic_gb_per_s"] = algo / kt["avg_ns"]
    out["derived"] = d
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
