#!/bin/bash
# Round 6: the 16-byte record path's parity tests and its host leg.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6f
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_op16.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python3 tools/host_probe.py > $O/host.json 2> $O/host.err || { tail -5 $O/host.err; exit 1; }
cat $O/host.json
