# Dev: the crashed-ops variant of the oversized key (fx_probe) with one
# level per launch (LC_FX_HOPS=0) and with the default hops: same counts
for cfg in LC_FX_HOPS=0 LC_FX_HOPS=8; do
  timeout -k 10 120 env $cfg python -u tools/fx_probe.py --ops 2000 --conc 50 --info 0.002 --no-tiers > gpurun_out/fx/var.txt 2>&1 || { tail -20 gpurun_out/fx/var.txt; exit 1; }
  echo "$cfg $(tail -1 gpurun_out/fx/var.txt)"
done
