#!/bin/bash
# C4 stage clocks: the GAP_PROFILE variant (tools/build_variants.sh prof -DGAP_PROFILE)
set -o pipefail
mkdir -p gpurun_out
LINCHECK_LIB=tools/variants/prof/liblincheck.so timeout -k 10 120 python tools/gap_probe.py 2 C4,C4x > gpurun_out/gapprof.log 2>&1
rc=$?; grep -v "^  matching\|^gap_decide" gpurun_out/gapprof.log | tail -4; grep -E "matching wg 0|gap_decide wg 0" gpurun_out/gapprof.log | head -6 | cut -c1-250; exit $rc
