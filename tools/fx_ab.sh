# Dev: interleaved A/B of the oversized key, 3 rounds: default vs the env
# assignment in $1 (e.g. LC_FX_COPY_SYNC=1), 5 checks each (min reported)
mkdir -p gpurun_out/fx
for i in 1 2 3; do
  timeout -k 10 120 python -u tools/fx_once.py --reps 5 > gpurun_out/fx/a$i.txt 2>&1 || { tail -20 gpurun_out/fx/a$i.txt; exit 1; }
  env $1 timeout -k 10 120 python -u tools/fx_once.py --reps 5 > gpurun_out/fx/b$i.txt 2>&1 || { tail -20 gpurun_out/fx/b$i.txt; exit 1; }
  python -c "import json,sys; a=json.loads(open('gpurun_out/fx/a$i.txt').read().strip().splitlines()[-1]); b=json.loads(open('gpurun_out/fx/b$i.txt').read().strip().splitlines()[-1]); print('A', ' '.join('%.1f'%x for x in a['ms']), a['explored'], a['max_frontier'], '| B($1)', ' '.join('%.1f'%x for x in b['ms']), b['explored'], b['max_frontier'])"
done
