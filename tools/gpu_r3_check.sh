#!/bin/bash
# round-3 dev loop: new GPU tests (frontier, checker configs) + queue sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fx.py tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu -k "frontier" > gpurun_out/r3_check.log 2>&1
rc=$?; tail -8 gpurun_out/r3_check.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_fxq_sweep.sh
