#!/bin/bash
# Dev tool: bench each variant in tools/variants twice, interleaved.
set -uo pipefail
for rep in 1 2; do
  for v in $(ls tools/variants); do
    LINCHECK_LIB=tools/variants/$v/liblincheck.so timeout -k 10 120 python bench.py --bare --steps 30 2>gpurun_out/ab_$v.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', 'rep $rep', 'kernel_ms %.4f step %.4f' % (d['roofline']['kernel_ms'], d['ms_per_step']), d['verdicts'])"
  done
done
