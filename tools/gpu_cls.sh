#!/bin/bash
# counted classes: the frontier-exchange suite + frontier/witness tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fx.py tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu -k "fx or whole_gpu or frontier or model" > gpurun_out/cls_test.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR" gpurun_out/cls_test.log | tail -40; tail -3 gpurun_out/cls_test.log; exit $rc
