#!/bin/bash
# PMC passes for one kernel of one workload (run on the GPU box, repo root):
#   tools/pmc_kernel.sh TAG LEG [REPS]
# One rocprofv3 run per counter group (MI355X_MICROARCH.md: FETCH_SIZE and
# WRITE_SIZE never share a pass), plus a kernel-trace/stats run; raw CSVs
# under gpurun_out/pmc_TAG/, summarised by tools/pmc_summary.py.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; LEG=$2; REPS=${3:-3}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/$n -o $n --output-format csv -- \
    python3 $R/tools/leg.py $LEG $REPS > $O/$n.log 2>&1
  echo "pass $n done"
}
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- \
  python3 $R/tools/leg.py $LEG $REPS > $O/kt.log 2>&1
echo "kernel trace done"
run sqa SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES
run sqb SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH GRBM_GUI_ACTIVE
run l2 TCC_HIT_sum TCC_MISS_sum
run fetch FETCH_SIZE
run write WRITE_SIZE
