#!/bin/bash
# Round 6: the GPU fuzz at HEAD (48/24/16-byte records, certificates checked,
# the PROOF search's cap hits counted).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6g
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u tools/fuzz_gpu.py ${ROUNDS:-6} > $O/fuzz.log 2>&1
rc=$?
tail -4 $O/fuzz.log
exit $rc
