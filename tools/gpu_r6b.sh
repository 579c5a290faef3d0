#!/bin/bash
# Round 6: the resident grid's parity tests, then the shard probe (wall time
# per step by key count, resident on / off) and a kernel trace of it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6b
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_resident.py \
  tests/test_gpu.py::test_check_device_path_with_torch tests/test_gpu_witness.py::test_proof_search_over_its_cap_leaves_no_certificate > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 python3 tools/shard_probe.py 300 > $O/shard_res.json 2> $O/shard_res.err || exit $?
LC_RESIDENT=0 timeout -k 10 120 python3 tools/shard_probe.py 300 > $O/shard_launch.json 2> $O/shard_launch.err || exit $?
cat $O/shard_res.json $O/shard_launch.json
timeout -k 10 60 $R/tools/doorbell_probe2_bin 2000 > $O/doorbell2.txt 2>&1; echo "doorbell rc $?"; cat $O/doorbell2.txt
