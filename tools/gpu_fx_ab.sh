#!/bin/bash
# frontier exchange: GPU tests, then the oversized key on this build vs
# tools/variants/$FXAB builds (interleaved)
set -o pipefail
mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_fx.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/fx_test.log 2>&1
  rc=$?; tail -3 gpurun_out/fx_test.log; [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2 3; do
  for v in default $FXAB; do
    if [ $v = default ]; then L=""; else L=tools/variants/$v/liblincheck.so; fi
    LINCHECK_LIB=$L timeout -k 10 120 python tools/fx_probe.py --ops 2000 --conc 50 --info 0 --reps 3 --no-tiers > gpurun_out/fxab.json || exit $?
    echo "$v run $i $(python -c "import json;d=json.load(open('gpurun_out/fxab.json'))['fx'];print(round(d['ms'],1),d['explored'],d['max_frontier'],d['stats']['levels'],d['stats']['redos'])")"
  done
done
