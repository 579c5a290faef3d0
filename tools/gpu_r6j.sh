#!/bin/bash
# Round 6: model leg A/B of the cooperative tier's legality test (by state vs
# by slot), interleaved, then the phase clocks of the by-slot build
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 170 python3 -c "import torch; print(torch.__version__, flush=True)" || exit $?
for r in 1 2; do
  for v in d0 d64 d16; do
    echo "== $v" >> gpurun_out/ab_direct.txt
    LINCHECK_LIB=tools/variants/$v/liblincheck.so timeout -k 10 100 python3 -u tools/leg.py model 5 >> gpurun_out/ab_direct.txt 2>&1 || exit $?
  done
done
LINCHECK_LIB=tools/variants/cprof/liblincheck.so timeout -k 10 100 python3 -u tools/leg.py model 2 > gpurun_out/cprof_direct.txt 2>&1
