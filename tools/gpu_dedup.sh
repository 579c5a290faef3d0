# Dev: pass-1 read dedup A/B on the crash leg (in-tree vs tools/variants/nodedup),
# the fused pass's LDS counters, and the fast-path GPU tests
set -o pipefail
mkdir -p gpurun_out/dd
for rep in 1 2 3; do
  echo "dedup   $(timeout -k 10 120 python tools/crash_call.py 3 2>/dev/null | tr '\n' ' ')" || exit 1
  echo "nodedup $(LINCHECK_LIB=tools/variants/nodedup/liblincheck.so timeout -k 10 120 python tools/crash_call.py 3 2>/dev/null | tr '\n' ' ')" || exit 1
done
echo "C2 dedup   $(timeout -k 10 120 python bench.py --bare --steps 200 --warmup 20 2>/dev/null | tail -1 | cut -c1-200)"
echo "C2 nodedup $(LINCHECK_LIB=tools/variants/nodedup/liblincheck.so timeout -k 10 120 python bench.py --bare --steps 200 --warmup 20 2>/dev/null | tail -1 | cut -c1-200)"
bash tools/fused_pmc.sh > gpurun_out/dd/pmc.txt 2>&1 || { tail -5 gpurun_out/dd/pmc.txt; exit 1; }
grep -E "LDS|VALU|WAVE_CYCLES" gpurun_out/dd/pmc.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_witness.py tests/test_op32.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/dd/t.log 2>&1; rc=$?; tail -2 gpurun_out/dd/t.log; exit $rc
