#!/bin/bash
# Round 6: interleaved A/B of variant builds on one leg (tools/leg.py),
# V="a b ..." LEG=crashdev REPS=20
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
OUT=gpurun_out/ab_${TAG:-leg}.txt
timeout -k 10 170 python3 -c "import torch; print(torch.__version__, flush=True)" || exit $?
for r in 1 2 3; do
  for v in $V; do
    echo "== $v" >> $OUT
    LINCHECK_LIB=tools/variants/$v/liblincheck.so timeout -k 10 100 python3 -u tools/leg.py ${LEG:-crashdev} ${REPS:-20} >> $OUT 2>&1 || exit $?
  done
done
