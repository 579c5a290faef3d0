#!/bin/bash
# Dev: LDS / issue counters of the fused pass on the crash leg (in-tree build).
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pmc_fused
mkdir -p $O
export TMPDIR=/tmp LC_FUSED=1
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/a -o a --output-format csv -- python3 $R/tools/leg.py crashdev 3 > $O/a.log 2>&1
echo pass a
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT -d $O/b -o b --output-format csv -- python3 $R/tools/leg.py crashdev 3 > $O/b.log 2>&1
echo pass b
python3 - <<'PY'
import csv,glob,collections
R='gpurun_out/pmc_fused'
for p in ('a','b'):
    fs=glob.glob(f'{R}/{p}/**/*counter_collection.csv',recursive=True)
    agg=collections.defaultdict(list)
    for f in fs:
        for r in csv.DictReader(open(f)):
            if 'fused_tier' in r['Kernel_Name']:
                agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for k,v in sorted(agg.items()):
        print(p,k,'per-launch',sum(v)/max(1,len(set(range(len(v))))) if False else v[-1], 'n',len(v))
PY
