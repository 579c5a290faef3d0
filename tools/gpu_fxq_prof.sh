#!/bin/bash
# kernel trace of the oversized key on the queue path (dev)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fxq_prof
LC_FXQ_MAXG=64 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fxq_prof/q -o q -- python tools/fx_probe.py --ops 2000 --conc 50 --info 0 --reps 1 --no-tiers > gpurun_out/fxq_prof/q.json || exit $?
find gpurun_out/fxq_prof -name "*kernel_stats.csv" | head
for f in $(find gpurun_out/fxq_prof -name "*kernel_stats.csv"); do head -8 $f | cut -c1-200; done
