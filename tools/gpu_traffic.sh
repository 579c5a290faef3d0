#!/bin/bash
# HBM traffic of the bench's dominant kernel: FETCH_SIZE, WRITE_SIZE and the
# L2 hit counters in passes of their own over bench.py --bare (summarised by
# tools/pmc_traffic.py into profiles/<tag>/traffic_fast_tier.json)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_${1:-r03}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" "l2 TCC_HIT_sum TCC_MISS_sum"; do
  set -- $pass
  n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/$n -o $n --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 1 --bare > $O/$n.log 2>&1 || exit $?
  echo "$n done"
done
