#!/bin/bash
# Round 6, first GPU look: the version-order pass at C3 shard sizes under a
# kernel trace (in-tree library and the loads-only dev build), then the
# bounded doorbell probe (last: it is the one step that may time out).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6a
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt_tree -o kt --output-format csv -- \
  python3 $R/tools/shard_probe.py 200 > $O/shard_tree.json 2> $O/shard_tree.err || exit $?
echo "in-tree shard trace done"
LINCHECK_LIB=$R/tools/variants/loads/liblincheck.so timeout -k 10 240 rocprofv3 --kernel-trace --stats \
  -d $O/kt_loads -o kt --output-format csv -- \
  python3 $R/tools/shard_probe.py 200 > $O/shard_loads.json 2> $O/shard_loads.err || exit $?
echo "loads-only shard trace done"
timeout -k 10 60 python3 $R/tools/shard_probe.py 300 > $O/shard_wall.json 2> $O/shard_wall.err || exit $?
echo "wall done"
timeout -k 10 60 $R/tools/doorbell_probe2_bin 2000 > $O/doorbell2.txt 2>&1
echo "doorbell rc $?"
