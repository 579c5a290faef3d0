#!/bin/bash
# SQ / TA / TCC counters for one kernel (KERNEL env, default fast_tier_kernel);
# one PMC pass per counter group, kernel dispatch only.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ctr_${1:-x}
K=${KERNEL:-fast_tier_kernel}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
run() {  # name, counters...
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $O/$n -o $n --output-format csv -- \
    python3 $R/bench.py --steps 3 --warmup 1 --bare > $O/$n.log 2>&1
}
run a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run b SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE
run c TA_TA_BUSY_sum TCC_HIT_sum TCC_MISS_sum
run d FETCH_SIZE
python3 - "$O" "$K" "${GRID:-2560000}" <<'PY'
import csv, glob, sys, statistics, collections
o, k, grid = sys.argv[1], sys.argv[2], sys.argv[3]
vals = collections.defaultdict(list)
for f in glob.glob(o + "/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if k in r["Kernel_Name"] and int(r["Grid_Size"]) >= int(grid):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, v in sorted(vals.items()):
    print("%-24s %16.0f  (n=%d)" % (name, statistics.median(v), len(v)))
PY
