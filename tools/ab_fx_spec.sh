# A/B of the frontier exchange's speculative level padding (LC_FX_SPEC_PAD:
# levels launched per batch = the last return's levels + pad) on bench.py's
# oversized key, interleaved (run on the GPU box, repo root).
set -e
for i in 1 2 3; do
  for m in 1 0 2; do
    LC_FX_SPEC_PAD=$m timeout -k 10 120 python tools/leg.py fx 4 > gpurun_out/abspec_${m}_$i.log 2>&1
    python -c "
import json,statistics
r=[json.loads(l) for l in open('gpurun_out/abspec_${m}_$i.log') if l.startswith('{')][1:]
print('pad $m run $i wall_ms med %.1f min %.1f' % (statistics.median(x['wall_ms'] for x in r), min(x['wall_ms'] for x in r)), 'levels', r[-1]['stats']['levels'], 'configs', r[-1]['configs'])"
  done
done
