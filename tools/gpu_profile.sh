#!/bin/bash
# Run on the GPU box (via gpurun) from the repo root:
#   bench.py JSON line, rocprofv3 kernel-trace stats, and FETCH_SIZE /
#   WRITE_SIZE PMC passes (separate runs, per MI355X_MICROARCH.md), all
#   under gpurun_out/.  Every GPU step has its own time limit; a failing step
#   ends the script.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-r01}
STEPS=${STEPS:-20}
mkdir -p $O $O/prof_$TAG
cd $R
timeout -k 10 400 python3 bench.py --steps $STEPS --warmup 3 > $O/bench_$TAG.json 2> $O/bench_$TAG.err
echo "bench done"; cat $O/bench_$TAG.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG/kt -o kt --output-format csv -- \
  python3 $R/bench.py --steps $STEPS --warmup 3 --bare > $O/prof_$TAG/kt.log 2>&1
echo "kernel trace done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/prof_$TAG/fetch -o fetch --output-format csv -- \
  python3 $R/bench.py --steps 5 --warmup 1 --bare > $O/prof_$TAG/fetch.log 2>&1
echo "fetch done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/prof_$TAG/write -o write --output-format csv -- \
  python3 $R/bench.py --steps 5 --warmup 1 --bare > $O/prof_$TAG/write.log 2>&1
echo "write done"
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/prof_$TAG/l2 -o l2 --output-format csv -- \
  python3 $R/bench.py --steps 5 --warmup 1 --bare > $O/prof_$TAG/l2.log 2>&1
echo "l2 done"
# every leg of the bench line (gap, JIT, HBM tiers, compaction, narrowing)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$TAG/kt_all -o kt_all --output-format csv -- \
  python3 $R/bench.py --steps $STEPS --warmup 3 --no-cpu-baseline > $O/prof_$TAG/kt_all.log 2>&1
echo "all-legs kernel trace done"
find $O/prof_$TAG -name '*.csv' | head -50
