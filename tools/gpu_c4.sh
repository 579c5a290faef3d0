#!/bin/bash
# C4 dev loop: the gap-tier GPU tests (verdicts vs the restatement and the
# oracle, witnesses certified), then C4 / C4x timings (tools/gap_probe.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_witness.py -x -q --timeout 200 --timeout-method thread -m gpu -k "gap or c4 or crash or witness or fused or mixed or golden" > gpurun_out/c4_test.log 2>&1
rc=$?; tail -3 gpurun_out/c4_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/gap_probe.py 4 C4,C4x,C4x1004,C5 || exit $?
if [ -n "$GAPPROF" ]; then
  LINCHECK_LIB=tools/variants/prof/liblincheck.so timeout -k 10 120 python tools/gap_probe.py 2 C4,C4x > gpurun_out/gapprof.log 2>&1 || exit $?
  grep -E "matching wg 0|gap_decide wg 0" gpurun_out/gapprof.log | head -6 | cut -c1-250
fi
if [ -n "$GAPAB" ]; then
  for v in $GAPAB; do echo "variant $v"; LINCHECK_LIB=tools/variants/$v/liblincheck.so timeout -k 10 120 python tools/gap_probe.py 3 C4,C4x,C4x1004 | tail -7 || exit $?; done
fi
if [ -n "$GAPTESTV" ]; then  # the gap suites again on a variant build (e.g. budget2: every branching decision reruns)
  LINCHECK_LIB=tools/variants/$GAPTESTV/liblincheck.so timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_witness.py -x -q --timeout 200 --timeout-method thread -m gpu -k "gap or c4 or crash or witness or mixed or golden" > gpurun_out/c4_test_v.log 2>&1
  rc=$?; tail -3 gpurun_out/c4_test_v.log; [ $rc -eq 0 ] || exit $rc
fi
