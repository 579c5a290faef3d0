# Dev: the native 24-byte pass — op32 parity tests (incl. the no-aux native
# path), the resident32 leg against the 48-byte step, the crash leg through
# lc_check32 vs lc_check
set -o pipefail
mkdir -p gpurun_out/r32
timeout -k 10 600 python -u -m pytest tests/test_op32.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r32/t.log 2>&1 || { tail -30 gpurun_out/r32/t.log; exit 1; }
tail -2 gpurun_out/r32/t.log
timeout -k 10 300 python -u tools/resident32.py 2 2>&1 | grep -v amdgpu.ids
