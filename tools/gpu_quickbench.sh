#!/bin/bash
# GPU tests + one bench line (no CPU baseline) — dev loop.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo pytest_exit=$rc; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc   # nothing more on the GPU after a failure
timeout -k 10 300 python bench.py --no-cpu-baseline 2>/dev/null > gpurun_out/bench.json
rc=$?; echo bench_exit=$rc; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('value %.4g ms/step %.3f kernel_ms %.3f frac %.4f' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac']), d['verdicts'])"
