#!/bin/bash
# Round 6: the value-indexed legality table of the cooperative tier: its GPU
# tests, then model-leg A/B against the previous build (interleaved), then
# the phase clocks
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 170 python3 -c "import torch; print(torch.__version__, flush=True)" || exit $?
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py tests/test_models.py tests/test_frontiers.py -m gpu > gpurun_out/df_tests.log 2>&1 || { tail -30 gpurun_out/df_tests.log; exit 1; }
tail -2 gpurun_out/df_tests.log
for r in 1 2; do
  for v in fl df; do
    echo "== $v" >> gpurun_out/ab_df.txt
    LINCHECK_LIB=tools/variants/$v/liblincheck.so timeout -k 10 100 python3 -u tools/leg.py model 5 >> gpurun_out/ab_df.txt 2>&1 || exit $?
  done
done
LINCHECK_LIB=tools/variants/cprof/liblincheck.so timeout -k 10 100 python3 -u tools/leg.py model 2 > gpurun_out/cprof_df.txt 2>&1
