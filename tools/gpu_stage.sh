# Dev: the pinned staging of small lc_check calls — the GPU suite, then the
# small calls with and without it (LC_STAGE=0), interleaved
set -o pipefail
mkdir -p gpurun_out/stage
[ "$1" = notests ] || { timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/stage/t.log 2>&1 || { tail -30 gpurun_out/stage/t.log; exit 1; }; }
[ "$1" = notests ] || tail -2 gpurun_out/stage/t.log
for i in 1 2 3 4; do
  for s in 0 1; do
    timeout -k 10 200 env LC_STAGE=$s python -u tools/stage_ab.py > gpurun_out/stage/s.txt 2>&1 || { tail -20 gpurun_out/stage/s.txt; exit 1; }
    tail -1 gpurun_out/stage/s.txt
  done
done
