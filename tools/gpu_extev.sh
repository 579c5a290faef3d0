# Dev: dispatch-bound timing events (hipExtLaunchKernel) — the bench's event
# kernel time against rocprofv3's, the step time, and the fast-path tests
set -o pipefail
mkdir -p gpurun_out/xe
for i in 1 2; do
  timeout -k 10 300 python bench.py --bare --steps 200 --warmup 20 > gpurun_out/xe/bare$i.json 2>gpurun_out/xe/bare.err || { tail -5 gpurun_out/xe/bare.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/xe/bare$i.json').read().strip().splitlines()[-1]); print('value %.4g ms/step %.4f frac %.3f fast %.4f' % (d['value'], d['ms_per_step'], d['roofline']['frac'], d['tiers']['fast_kernel_ms']))"
done
timeout -k 10 300 python -u tools/step_floor.py 300 > gpurun_out/xe/step_floor.jsonl 2>&1; grep -v amdgpu gpurun_out/xe/step_floor.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_op32.py tests/test_gpu_single_pass.py tests/test_gpu_witness.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/xe/t.log 2>&1; rc=$?; tail -2 gpurun_out/xe/t.log; exit $rc
