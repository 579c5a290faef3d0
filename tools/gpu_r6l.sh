#!/bin/bash
# Round 6: cooperative tier A/B (LDS hash, queue sleep) on the model leg,
# interleaved, after the tier's GPU tests on the in-tree build
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-"h0 h1 h1s2 h1s4"}
OUT=gpurun_out/ab_${TAG:-coop}.txt
timeout -k 10 170 python3 -c "import torch; print(torch.__version__, flush=True)" || exit $?
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py tests/test_models.py tests/test_frontiers.py -m gpu > gpurun_out/${TAG:-coop}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG:-coop}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG:-coop}_tests.log
for r in 1 2; do
  for v in $V; do
    echo "== $v" >> $OUT
    LINCHECK_LIB=tools/variants/$v/liblincheck.so timeout -k 10 100 python3 -u tools/leg.py model 5 >> $OUT 2>&1 || exit $?
  done
done
