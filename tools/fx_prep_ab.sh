#!/bin/bash
# Dev A/B (GPU box): the frontier-exchange GPU tests, then the oversized key
# (tools/leg.py fx) with the return preparation on / off (LC_FX_PREP),
# interleaved; one line per run in gpurun_out/r4b/fxab.txt.
set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fx.py -m gpu > gpurun_out/r4b/fx3.txt 2>&1 || exit 1
for v in 1 0 1 0 1 0; do
  LC_FX_PREP=$v timeout -k 10 120 python tools/leg.py fx 5 > gpurun_out/r4b/fxab_$v.txt 2>&1 || exit 1
  echo "prep=$v $(python -c "
import json
r=[json.loads(l) for l in open('gpurun_out/r4b/fxab_$v.txt') if l.startswith('{')]
print([round(x['wall_ms'],1) for x in r], r[-1]['configs'], r[-1]['stats']['levels'], r[-1]['stats']['max_local_frontier'])")" >> gpurun_out/r4b/fxab.txt
done
