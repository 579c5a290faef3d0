#!/bin/bash
# Dev tool: fast-tier kernel time vs number of keys (1 key = 1 workgroup),
# for each variant in tools/variants: per-workgroup latency at low load.
set -uo pipefail
for v in ${VARIANTS:-$(ls tools/variants)}; do
  for k in ${KEYS:-256 512 1792 3584 10000}; do
    LINCHECK_LIB=tools/variants/$v/liblincheck.so timeout -k 10 120 python bench.py --bare --steps 30 --keys $k 2>gpurun_out/ls_$v.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', 'keys $k', 'kernel_ms %.4f' % d['roofline']['kernel_ms'])" || exit 1
  done
done
