# A/B of the frontier exchange's table-prefix multiplier (LC_FX_TABLE_MUL) on
# bench.py's oversized key, interleaved (run on the GPU box, repo root).
set -e
for i in 1 2; do
  for m in 4 8 16 2; do
    LC_FX_TABLE_MUL=$m timeout -k 10 120 python tools/leg.py fx 4 > gpurun_out/abfx_${m}_$i.log 2>&1
    python -c "
import json,statistics
r=[json.loads(l) for l in open('gpurun_out/abfx_${m}_$i.log') if l.startswith('{')][1:]
print('mul $m run $i wall_ms med %.1f min %.1f' % (statistics.median(x['wall_ms'] for x in r), min(x['wall_ms'] for x in r)), 'redos', r[-1]['stats']['redos'], 'configs', r[-1]['configs'])"
  done
done
