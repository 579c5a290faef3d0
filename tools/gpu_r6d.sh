#!/bin/bash
# Round 6: the bench line at HEAD (resident grid for C3 shards), then the
# doorbell probe's fix variants (whole-wave poll: masks 32, 47).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6d
mkdir -p $O
cd $R
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value %.4g ms %.4f frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))
for c in d['c3_shards']: print(c['n_gpus'], 'implied ms %.4f speedup %.2f' % (c['implied_ms_per_step'], c['implied_speedup']), [round(x['kernel_ms']*1e3,1) for x in c['shards']])
"
LINCHECK_LIB=$R/tools/variants/fprof/liblincheck.so LC_RESIDENT=0 timeout -k 10 120 python3 tools/shard_probe.py 30 1,1250,10000 > $O/fprof.txt 2> $O/fprof.err || exit $?
grep fastprof $O/fprof.txt | awk '{print $3}' | uniq -c
for m in 32 47; do
  timeout -k 10 30 $R/tools/doorbell_probe2_bin 500 $m > $O/r5mask_$m.txt 2>&1
  rc=$?
  tail -3 $O/r5mask_$m.txt
  [ $rc = 0 ] || { echo "mask $m rc $rc: stop"; exit 0; }
done
