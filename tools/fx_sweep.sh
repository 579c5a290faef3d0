# Dev: the oversized key under each env setting given as an argument
# ("LC_FX_HOP2=16,LC_FX_HOPS=2"; commas separate assignments), 5 checks each
mkdir -p gpurun_out/fx
for cfg in "$@"; do
  timeout -k 10 120 env ${cfg//,/ } python -u tools/fx_once.py --reps 5 > gpurun_out/fx/sweep.txt 2>&1 || { tail -20 gpurun_out/fx/sweep.txt; exit 1; }
  python -c "import json; a=json.loads(open('gpurun_out/fx/sweep.txt').read().strip().splitlines()[-1]); print('$cfg', ' '.join('%.1f'%x for x in a['ms']), a['explored'], a['max_frontier'], a['stats']['levels'])"
done
