#!/bin/bash
# Round 6 evidence at HEAD: kernel traces of the bench and each leg, the
# fast tier's traffic passes, the model leg's PMC passes (profiles/r06)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 170 python3 -c "import torch; print(torch.__version__, flush=True)" || exit $?
ROUND=r06 LEGS="model hot hotx crashdev mixed fx" bash tools/gpu_prof.sh || exit $?
bash tools/gpu_traffic.sh r06 || exit $?
cd $R
timeout -k 10 600 bash tools/pmc_kernel.sh model_r6 model 2 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_model_r6 hbm_coop_kernel gpurun_out/pmc_model_hbm_coop4.json > /dev/null || exit $?
echo evidence done
