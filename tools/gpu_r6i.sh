#!/bin/bash
# Round 6: PMC passes of the model leg's hbm_coop_kernel<4> (profiles/r06)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 600 bash tools/pmc_kernel.sh model_r6 model 2 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_model_r6 hbm_coop_kernel gpurun_out/pmc_model_hbm_coop4.json > /dev/null || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_model_hbm_coop4.json')); print(json.dumps(d['derived'])); print(d['kernel_trace'])"
