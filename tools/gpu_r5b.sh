# completion-signal round: the GPU suite's fast-path tests, the step floor, a bare bench
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_op32.py tests/test_gpu_single_pass.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r5/t2.log 2>&1 || { tail -30 gpurun_out/r5/t2.log; exit 1; }
tail -2 gpurun_out/r5/t2.log
timeout -k 10 300 python -u tools/step_floor.py 300 > gpurun_out/r5/step_floor.jsonl 2>&1; cat gpurun_out/r5/step_floor.jsonl
timeout -k 10 300 python bench.py --bare --steps 50 > gpurun_out/r5/bare.json 2>gpurun_out/r5/bare.err && python -c "
import json; d=json.load(open('gpurun_out/r5/bare.json')); print('value %.4g ms/step %.4f frac %.3f fast %.4f' % (d['value'], d['ms_per_step'], d['roofline']['frac'], d['tiers']['fast_kernel_ms']))"
timeout -k 10 600 python -u -m pytest tests/test_gpu_witness.py tests/test_frontiers.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5/t3.log 2>&1 || { tail -30 gpurun_out/r5/t3.log; exit 1; }
tail -2 gpurun_out/r5/t3.log
