#!/bin/bash
# Round 6 (dropped; record in profiles/r06/fx_report_ab.txt): the frontier exchange's reports — system-scope report stores
# without the release fence, and reports folded into the batches' last
# launches: FX GPU tests both ways, then the oversized key interleaved
# (rr1 build: the release fence; norelease: LC_FX_FOLD=0; fold: default)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
OUT=gpurun_out/ab_fxfold.txt
timeout -k 10 170 python3 -c "import torch; print(torch.__version__, flush=True)" || exit $?
LC_FX_FOLD=0 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fx.py tests/test_frontiers.py -m gpu > gpurun_out/fxrel_tests.log 2>&1 || { tail -30 gpurun_out/fxrel_tests.log; exit 1; }
tail -1 gpurun_out/fxrel_tests.log
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fx.py tests/test_frontiers.py -m gpu > gpurun_out/fxfold_tests.log 2>&1 || { tail -30 gpurun_out/fxfold_tests.log; exit 1; }
tail -1 gpurun_out/fxfold_tests.log
for r in 1 2 3; do
  echo "== release" >> $OUT
  LC_FX_FOLD=0 LINCHECK_LIB=tools/variants/rr1/liblincheck.so timeout -k 10 100 python3 -u tools/leg.py fx 4 >> $OUT 2>&1 || exit $?
  echo "== norelease" >> $OUT
  LC_FX_FOLD=0 timeout -k 10 100 python3 -u tools/leg.py fx 4 >> $OUT 2>&1 || exit $?
  echo "== fold" >> $OUT
  timeout -k 10 100 python3 -u tools/leg.py fx 4 >> $OUT 2>&1 || exit $?
done
