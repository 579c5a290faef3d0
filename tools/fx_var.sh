#!/bin/bash
# Dev: the frontier-exchange suite on the in-tree build, then the oversized
# key (bench.py's fx leg) under each variant in tools/variants, interleaved.
set -o pipefail
mkdir -p gpurun_out/fxv
timeout -k 10 400 python -u -m pytest tests/test_fx.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/fxv/test.log 2>&1 || { tail -30 gpurun_out/fxv/test.log; exit 1; }
tail -1 gpurun_out/fxv/test.log
for rep in 1 2 3; do
  for v in $(ls tools/variants); do
    LINCHECK_LIB=tools/variants/$v/liblincheck.so timeout -k 10 120 python tools/leg.py fx 4 2>/dev/null | python -c "
import sys,json
r=[json.loads(l) for l in sys.stdin if l.startswith('{')]
print('$v', [round(x['wall_ms'],1) for x in r], r[-1]['configs'], r[-1]['stats']['levels'], r[-1]['stats']['max_local_frontier'])" || exit 1
  done
done
