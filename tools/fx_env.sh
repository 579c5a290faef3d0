#!/bin/bash
# Dev: the oversized key under several values of one environment switch
# (in-tree build), interleaved:  EVAR=LC_FX_SPEC_PAD EVALS="0 1 2" tools/fx_env.sh
set -o pipefail
for rep in 1 2; do
  for v in ${EVALS}; do
    env ${EVAR}=$v timeout -k 10 120 python tools/leg.py fx 4 2>/dev/null | python -c "
import sys,json
r=[json.loads(l) for l in sys.stdin if l.startswith('{')]
print('${EVAR}=$v', [round(x['wall_ms'],1) for x in r], r[-1]['configs'], r[-1]['stats']['levels'], r[-1]['stats']['redos'])" || exit 1
  done
done
