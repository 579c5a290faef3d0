#!/bin/bash
set -o pipefail
for cfg in "LC_FXQ_LOCAL=0" "LC_FXQ_LOCAL=16" "LC_FXQ_LOCAL=0 LC_FXQ_MAXG=64"; do
  echo "== $cfg"
  env $cfg LC_FXQ_TIME=1 timeout -k 10 120 python tools/fx_probe.py --ops 2000 --conc 50 --info 0 --reps 1 --no-tiers 2>&1 | grep -E "fxq:|ms" | cut -c1-200 || exit $?
done
