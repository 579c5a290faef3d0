#!/bin/bash
# Round evidence at HEAD, in two calls (each under gpurun's 1,200 s):
#   bash tools/gpu_evidence.sh tests   -> the whole GPU suite, smoke, GPU fuzz
#   bash tools/gpu_evidence.sh prof    -> kernel traces (bench --bare, every leg),
#                                         HBM traffic + L2 passes, fused / gap PMC,
#                                         then the full bench line with that traffic
# Outputs under gpurun_out/ev/ (copied into profiles/<round>/ afterwards).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ev
mkdir -p $O
cd $R
if [ "$1" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1
  rc=$?; tail -3 $O/gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
  timeout -k 10 200 python -u tools/fuzz_gpu.py 3 > $O/fuzz_gpu.log 2>&1 || { tail -5 $O/fuzz_gpu.log; exit 1; }
  tail -3 $O/fuzz_gpu.log
  exit 0
fi
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_bench -o kt --output-format csv -- \
  python3 $R/bench.py --steps 20 --warmup 3 --bare > $O/kt_bench.log 2>&1 || { tail -5 $O/kt_bench.log; exit 1; }
echo "kt bench done"
for leg in crash hot hotx mixed model fx; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_$leg -o kt --output-format csv -- \
    python3 $R/tools/leg.py $leg 3 > $O/kt_$leg.log 2>&1 || { tail -5 $O/kt_$leg.log; exit 1; }
  echo "kt $leg done"
done
mkdir -p $O/prof/kt
cp $O/kt_bench/kt_kernel_stats.csv $O/prof/kt/kt_kernel_stats.csv
for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" "l2 TCC_HIT_sum TCC_MISS_sum"; do
  set -- $pass
  n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $O/prof/$n -o $n --output-format csv -- \
    python3 $R/bench.py --steps 5 --warmup 1 --bare > $O/prof/$n.log 2>&1 || exit 1
  echo "pmc $n done"
done
cd $R
python tools/pmc_traffic.py $O/prof $O/ptraffic r05 10000000 > $O/traffic.log 2>&1 || { tail -5 $O/traffic.log; exit 1; }
GRAFT_REPO_ROOT=$R bash tools/fused_pmc.sh > $O/fused_pmc.txt 2>&1 || { tail -5 $O/fused_pmc.txt; exit 1; }
GRAFT_REPO_ROOT=$R bash tools/gap_pmc.sh hot hot > $O/gap_pmc.txt 2>&1 || { tail -5 $O/gap_pmc.txt; exit 1; }
echo "pmc done"
timeout -k 10 900 python bench.py --traffic-json $O/ptraffic/traffic_r05.json > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('value %.4g ms %.4f frac %.3f traffic %s' % (d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic']))"
