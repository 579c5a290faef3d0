#!/bin/bash
# Round 6: branch-free version-order passes — fast-tier parity tests, phase
# clocks, shard steps (resident and launched) and the bench's timed region,
# in-tree (branch-free pass 1 and 2) against p1br (pass 1 as the case
# analysis), interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6h
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu.py tests/test_resident.py tests/test_op32.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
LINCHECK_LIB=$R/tools/variants/fprof/liblincheck.so LC_RESIDENT=0 timeout -k 10 120 python3 tools/shard_probe.py 30 1,1250,10000 > $O/fprof.txt 2> $O/fprof.err || exit $?
for rep in 1 2; do
  for v in tree p1br; do
    if [ $v = tree ]; then lib=""; else lib=$R/tools/variants/$v/liblincheck.so; fi
    LINCHECK_LIB=$lib timeout -k 10 120 python3 tools/shard_probe.py 300 1,1250,2500,10000 > $O/shard_$v$rep.json 2> $O/shard_$v$rep.err || exit $?
    echo "$v $rep $(tr '\n' ' ' < $O/shard_$v$rep.json | sed 's/, "lib": "[^"]*"//g; s/"valid": [0-9]*, //g')"
    LINCHECK_LIB=$lib timeout -k 10 200 python3 bench.py --bare --steps 50 --warmup 5 > $O/bare_$v$rep.json 2> $O/bare_$v$rep.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/bare_$v$rep.json').read().strip().splitlines()[-1])
print('   bare ms %.4f kernel %.4f frac %.3f' % (d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac']))"
  done
done
