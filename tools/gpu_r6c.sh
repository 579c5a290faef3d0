#!/bin/bash
# Round 6: resident-grid parity tests after the tagged-word protocol, the
# shard probe (resident / launched), then round 5's hung kernel split into
# its constructs (doorbell_probe2 mask runs; the first one that hangs ends
# the script: it leaves on its own bound with exit code 3).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6c
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_resident.py \
  tests/test_gpu.py::test_check_device_path_with_torch > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python3 tools/shard_probe.py 300 > $O/shard_res.json 2> $O/shard_res.err || exit $?
LC_RESIDENT=0 timeout -k 10 120 python3 tools/shard_probe.py 300 > $O/shard_launch.json 2> $O/shard_launch.err || exit $?
paste -d' ' $O/shard_res.json $O/shard_launch.json | cut -c1-200
for m in 0 1 2 4 8; do
  timeout -k 10 30 $R/tools/doorbell_probe2_bin 500 $m > $O/r5mask_$m.txt 2>&1
  rc=$?
  tail -3 $O/r5mask_$m.txt
  [ $rc = 0 ] || { echo "mask $m rc $rc: stop"; exit 0; }
done
