#!/bin/bash
# round 3, re-entry: kernel trace of the bench's timed region (profiles/r03),
# then the frontier exchange's level path vs queue path on the oversized key
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3b
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b/kt_bench -o kt -- python3 bench.py --bare --steps 20 --warmup 3 > gpurun_out/r3b/bench_bare.json || exit $?
for q in 0 1 0 1; do
  LC_FX_QUEUE=$q LC_FXQ_TIME=1 timeout -k 10 120 python tools/fx_probe.py --ops 2000 --conc 50 --info 0 --reps 3 --no-tiers > gpurun_out/r3b/fxq_$q.json 2> gpurun_out/r3b/fxq_$q.err || exit $?
  echo "queue=$q $(python -c "import json;d=json.load(open('gpurun_out/r3b/fxq_$q.json'))['fx'];print(round(d['ms'],1),d['explored'],d['max_frontier'],d['verdict'],d['stats']['redos'])") $(grep fxq gpurun_out/r3b/fxq_$q.err | tail -1 | cut -c1-300)"
done
