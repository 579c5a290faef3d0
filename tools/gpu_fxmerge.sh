# Dev: merged split+levels launch A/B on the oversized key, the crashed-ops
# variant's counts, and the frontier-exchange GPU tests
set -o pipefail
mkdir -p gpurun_out/fx
bash tools/fx_sweep.sh LC_FX_MERGE=0 LC_FX_MERGE=1 LC_FX_MERGE_PAD=0 LC_FX_MERGE=0 LC_FX_MERGE=1 LC_FX_MERGE_PAD=0 || exit 1
LC_FX_HOSTPROF=1 timeout -k 10 100 python tools/fx_once.py --reps 1 2>&1 | grep hostprof | tail -1
for cfg in LC_FX_MERGE=0 LC_FX_MERGE=1; do
  timeout -k 10 120 env $cfg python -u tools/fx_probe.py --ops 2000 --conc 50 --info 0.002 --no-tiers > gpurun_out/fx/var.txt 2>&1 || { tail -20 gpurun_out/fx/var.txt; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/fx/var.txt | cut -c1-220)"
done
timeout -k 10 400 python -u -m pytest tests/test_fx.py tests/test_frontiers.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fx/t.log 2>&1; rc=$?; tail -2 gpurun_out/fx/t.log; exit $rc
