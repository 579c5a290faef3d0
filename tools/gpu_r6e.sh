#!/bin/bash
# Round 6: resident-grid A/B at C3 sizes: in-tree vs poll/sleep/claims
# variants, interleaved twice (wall per step and device time per request).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6e
mkdir -p $O
cd $R
for rep in 1 2; do
  for v in tree sl32 p1s8 res1p; do
    if [ $v = tree ]; then lib=""; else lib=$R/tools/variants/$v/liblincheck.so; fi
    LINCHECK_LIB=$lib timeout -k 10 120 python3 tools/shard_probe.py 300 1,625,1250 > $O/$v.$rep.json 2> $O/$v.$rep.err || { tail -5 $O/$v.$rep.err; exit 1; }
    echo "$v $rep $(tr '\n' ' ' < $O/$v.$rep.json | sed 's/"lib": "[^"]*"//g')"
  done
done
