#!/bin/bash
# SQ instruction-mix / stall counters for lds_tier_kernel (one PMC pass per
# counter group; no tracing domains besides kernel dispatch).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ctr_${1:-x}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  -d $O/a -o a --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/a.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE \
  -d $O/b -o b --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/b.log 2>&1
python3 - "$O" <<'PY'
import csv, glob, sys, statistics, collections
o = sys.argv[1]
vals = collections.defaultdict(list)
for f in glob.glob(o + "/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "lds_tier_kernel" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(vals.items()):
    print("%-24s %16.0f  (n=%d)" % (k, statistics.median(v), len(v)))
PY
