#!/bin/bash
# Instruction-mix PMC passes (two groups) for the gap tier on C4 (tools/leg.py hot),
# raw CSVs under gpurun_out/pmc_$TAG/, summarised by tools/pmc_summary.py.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-hot}; LEG=${2:-hot}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- \
  python3 $R/tools/leg.py $LEG 3 > $O/kt.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES -d $O/sqa -o sqa --output-format csv -- python3 $R/tools/leg.py $LEG 3 > $O/sqa.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_WAIT_INST_LDS -d $O/sqb -o sqb --output-format csv -- python3 $R/tools/leg.py $LEG 3 > $O/sqb.log 2>&1
echo done
