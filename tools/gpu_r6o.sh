#!/bin/bash
# Round 6 evidence at HEAD: PMC passes of the crash leg's fused pass and of
# C4's gap tier (profiles/r06/pmc_crash_fused.json, pmc_hot_gap_tier.json)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 170 python3 -c "import torch; print(torch.__version__, flush=True)" || exit $?
timeout -k 10 600 bash tools/pmc_kernel.sh crash6 crashdev 3 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_crash6 fused_tier_kernel gpurun_out/pmc_crash_fused.json > /dev/null || exit $?
timeout -k 10 600 bash tools/pmc_kernel.sh hot6 hot 3 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_hot6 gap_tier_kernel gpurun_out/pmc_hot_gap_tier.json > /dev/null || exit $?
echo pmc done
