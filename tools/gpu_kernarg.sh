# Dev: HIP_FORCE_DEV_KERNARG 0 / 1 on the launch-heavy paths (oversized key,
# bench --bare step), interleaved
set -o pipefail
mkdir -p gpurun_out/ka
for rep in 1 2; do
  for v in 0 1; do
    fx=$(HIP_FORCE_DEV_KERNARG=$v LC_FX_HOSTPROF=1 timeout -k 10 100 python tools/fx_once.py --reps 3 2>&1 | grep -v amdgpu | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(' '.join('%.1f'%x for x in d['ms']))") || exit 1
    b=$(HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python bench.py --bare --steps 200 --warmup 20 2>/dev/null | tail -1 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('%.4f'%d['ms_per_step'])") || exit 1
    echo "kernarg=$v fx_ms $fx bare_ms_per_step $b"
  done
done
