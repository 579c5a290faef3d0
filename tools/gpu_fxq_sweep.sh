#!/bin/bash
# queue-path knob sweep on the bench's oversized key (dev A/B)
set -o pipefail
timeout -k 10 300 python tools/fxq_debug.py || exit $?
run() { env "$@" timeout -k 10 120 python tools/fx_probe.py --ops 2000 --conc 50 --info 0 --reps 2 --no-tiers > gpurun_out/sweep.json 2>gpurun_out/sweep.err || exit $?;
  echo "$* -> $(python -c "import json;d=json.load(open('gpurun_out/sweep.json'))['fx'];print(round(d['ms'],1),d['explored'],d['max_frontier'])") $(grep fxq gpurun_out/sweep.err | tail -1)"; }
run LC_FX_QUEUE=0
run LC_FX_QUEUE=1 LC_FXQ_TIME=1 LC_FXQ_ATOMIC=1 LC_FXQ_LOCAL=0
run LC_FX_QUEUE=1 LC_FXQ_TIME=1 LC_FXQ_LOCAL=0
run LC_FX_QUEUE=1 LC_FXQ_TIME=1 LC_FXQ_LOCAL=16
run LC_FX_QUEUE=1 LC_FXQ_TIME=1 LC_FXQ_LOCAL=64
run LC_FX_QUEUE=1 LC_FXQ_TIME=1 LC_FXQ_LOCAL=0 LC_FXQ_MAXG=128
