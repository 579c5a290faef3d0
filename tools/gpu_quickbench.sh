#!/bin/bash
# GPU tests + one bench line (no CPU baseline) — dev loop.
set -uo pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
echo pytest_exit=$?; tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline 2>/dev/null > gpurun_out/bench.json
echo bench_exit=$?
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print('value %.4g ms/step %.3f kernel_ms %.3f frac %.4f' % (d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac']), d['verdicts'])"
