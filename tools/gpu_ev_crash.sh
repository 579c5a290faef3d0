# Evidence: the crash leg's fused pass as bench.py runs it (resident records,
# one launch per call): kernel trace and the fused PMC passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ev
mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_crashdev -o kt --output-format csv -- \
  python3 $R/tools/leg.py crashdev 3 > $O/kt_crashdev.log 2>&1 || { tail -5 $O/kt_crashdev.log; exit 1; }
cd $R
GRAFT_REPO_ROOT=$R bash tools/fused_pmc.sh > $O/fused_pmc.txt 2>&1 || { tail -5 $O/fused_pmc.txt; exit 1; }
echo done
