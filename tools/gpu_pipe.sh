#!/bin/bash
# Dev: GPU suites on the in-tree build, then the crash-leg / C2 variant A/B.
set -o pipefail
mkdir -p gpurun_out/pipe
timeout -k 10 700 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/pipe/test.log 2>&1 || { tail -40 gpurun_out/pipe/test.log; exit 1; }
tail -1 gpurun_out/pipe/test.log
bash tools/crash_var.sh
