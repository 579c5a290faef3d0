"""Summarise rocprofv3 outputs of tools/gpu_profile.sh into profiles/.

HBM traffic per launch of the dominant kernel from separate FETCH_SIZE and
WRITE_SIZE passes (MI355X_MICROARCH.md, HBM / rocprofv3 PMC slots: the two
do not fit one pass; both are in KiB; on gfx950 FETCH_SIZE reports half the
bytes of a wide coalesced read (16 B/lane) — our record loads are 16-B
dwordx4 per lane, so the read side is doubled).

usage: python tools/pmc_traffic.py gpurun_out/prof_r01 profiles r01 N_OPS [KERNEL]
"""
import csv
import json
import os
import shutil
import statistics
import sys

KERNEL = sys.argv[5] if len(sys.argv) > 5 else "fast_tier_kernel"


def counter(path, name):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == name]
    return statistics.median(vals), len(vals)


def main():
    src, dst, tag, n_ops = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    os.makedirs(os.path.join(dst, tag), exist_ok=True)
    fetch_kib, nf = counter(os.path.join(src, "fetch", "fetch_counter_collection.csv"), "FETCH_SIZE")
    write_kib, nw = counter(os.path.join(src, "write", "write_counter_collection.csv"), "WRITE_SIZE")
    read_b = fetch_kib * 1024 * 2      # gfx950 correction for 16-B/lane reads
    write_b = write_kib * 1024
    l2 = os.path.join(src, "l2", "l2_counter_collection.csv")
    hit = miss = None
    if os.path.exists(l2):
        hit, _ = counter(l2, "TCC_HIT_sum")
        miss, _ = counter(l2, "TCC_MISS_sum")
    stats = list(csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))))
    k = [r for r in stats if KERNEL in r["Name"]][0]
    out = {
        "kernel": KERNEL,
        "n_ops": n_ops,
        "launches_fetch": nf, "launches_write": nw,
        "fetch_size_kib_raw": fetch_kib, "write_size_kib_raw": write_kib,
        "read_bytes_corrected": read_b, "write_bytes": write_b,
        "hbm_bytes_per_launch": read_b + write_b,
        "hbm_bytes_per_op": (read_b + write_b) / n_ops,
        "rocprof_avg_ns": float(k["AverageNs"]), "rocprof_calls": int(k["Calls"]),
        "l2_hits": hit, "l2_misses": miss,
        "l2_hit_rate": (hit / (hit + miss)) if hit is not None and hit + miss > 0 else None,
        "note": "FETCH_SIZE doubled (gfx950 wide-read undercount); WRITE_SIZE as reported",
    }
    json.dump(out, open(os.path.join(dst, "traffic_%s.json" % tag), "w"), indent=1)
    for sub, f in (("kt", "kt_kernel_stats.csv"), ("kt", "kt_domain_stats.csv"),
                   ("fetch", "fetch_counter_collection.csv"),
                   ("write", "write_counter_collection.csv"),
                   ("l2", "l2_counter_collection.csv"),
                   ("kt_all", "kt_all_kernel_stats.csv")):
        p = os.path.join(src, sub, f)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, tag, f))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
