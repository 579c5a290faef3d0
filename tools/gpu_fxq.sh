#!/bin/bash
# frontier-exchange tests, then the bench's oversized key on the queue path
# and on the level path (A/B)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fx.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/fxq_test.log 2>&1
rc=$?; tail -25 gpurun_out/fxq_test.log; [ $rc -eq 0 ] || exit $rc
for q in 1 0 1 0; do
  LC_FX_QUEUE=$q timeout -k 10 120 python tools/fx_probe.py --ops 2000 --conc 50 --info 0 --reps 3 --no-tiers > gpurun_out/fxq_probe_$q.json || exit $?
  echo "queue=$q $(python -c "import json;d=json.load(open('gpurun_out/fxq_probe_$q.json'))['fx'];print(d['ms'],d['explored'],d['max_frontier'],d['verdict'],d['stats']['redos'])")"
done
