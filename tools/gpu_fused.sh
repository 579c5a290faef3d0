#!/bin/bash
# fused version-order + crash-light pass: tests, then the crash leg's kernel times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_witness.py tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu -k "fused or crash or gap or golden or witness" > gpurun_out/fused_test.log 2>&1
rc=$?; tail -5 gpurun_out/fused_test.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1; do
  echo "LC_FUSED=$m"; LC_FUSED=$m timeout -k 10 120 python tools/leg.py crash 4 || exit $?
done
