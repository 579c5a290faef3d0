#!/bin/bash
# Dev tool: bench variant/env combinations twice, interleaved.
# usage: tools/ab_env.sh "name|LIB|ENV=..." ...
set -uo pipefail
for rep in 1 2; do
  for spec in "$@"; do
    IFS='|' read -r name lib envs <<< "$spec"
    env LINCHECK_LIB=$lib $envs timeout -k 10 120 python bench.py --bare --steps 30 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$name', 'rep $rep', 'kernel_ms %.4f step %.4f' % (d['roofline']['kernel_ms'], d['ms_per_step']), d['verdicts'])" || exit 1
  done
done
