#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats, csv): the bench's timed
# region (--bare) and each secondary leg on its own (tools/leg.py), under
# gpurun_out/prof_$ROUND/<name>/ (ROUND defaults to r04; LEGS to every leg).
# Every step has its own time limit; a failing step ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_${ROUND:-r04}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/bench -o kt --output-format csv -- \
  python3 $R/bench.py --steps 20 --warmup 3 --bare > $O/bench.json 2> $O/bench.err || exit $?
echo "bench trace done"
for leg in ${LEGS:-model hot hotx crash mixed fx}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$leg -o kt --output-format csv -- \
    python3 $R/tools/leg.py $leg 4 > $O/$leg.log 2>&1 || exit $?
  echo "$leg trace done"
done
find $O -name '*kernel_stats.csv' | sort
