set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_witness.py -x -q --timeout 200 --timeout-method thread -m gpu -k "gap or c4 or crash or witness or fused or mixed or golden" > gpurun_out/r4b/c4_test.log 2>&1 || { tail -30 gpurun_out/r4b/c4_test.log; exit 1; }
tail -1 gpurun_out/r4b/c4_test.log
for w in ${WVALS:-1 0 1 0}; do
  echo "${WVAR:-LC_GAP_WIDE}=$w"
  env ${WVAR:-LC_GAP_WIDE}=$w timeout -k 10 120 python tools/gap_probe.py 3 C4,C4x,C4x1004 2>/dev/null | python -c "
import sys,json
r={}
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); r.setdefault(d['cfg'],[]).append((round(d['gap_ms'],3),d['nodes']))
print(r)" || exit 1
done
