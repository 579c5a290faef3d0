#!/bin/bash
# Dev tool: each variant in tools/variants on the crash leg (fused pass
# forced) and on C2 (version-order tier), interleaved twice: median kernel ms.
set -uo pipefail
for rep in 1 2; do
  for v in $(ls tools/variants); do
    c=$(LC_FUSED=1 LINCHECK_LIB=tools/variants/$v/liblincheck.so timeout -k 10 120 python tools/leg.py crash 7 2>/dev/null | python -c "
import sys,json,statistics
r=[json.loads(l) for l in sys.stdin if l.startswith('{')]
print('%.4f' % statistics.median(x['fast_ms'] for x in r[1:]), r[-1]['verdicts'])") || exit 1
    b=$(LINCHECK_LIB=tools/variants/$v/liblincheck.so timeout -k 10 120 python bench.py --bare --steps 30 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4f' % d['roofline']['kernel_ms'])") || exit 1
    echo "$v rep $rep crash_fused_ms $c c2_fast_ms $b"
  done
done
