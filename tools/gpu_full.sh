#!/bin/bash
# the round-end checks: every GPU test, smoke, then the full bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_full.err; exit $rc; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/bench_full.json"))
print("value %.4g ms/step %.4f frac %.3f" % (d["value"], d["ms_per_step"], d["roofline"]["frac"]))
print("crash_leg", {k: d["crash_leg"][k] for k in ("call_ms", "fast_kernel_ms", "gap_kernel_ms")})
print("hot_key", d["hot_key"])
print("oversized", {k: d["oversized_key"][k] for k in ("fx_ms", "configs_explored", "max_frontier")})
print("c3", [(x["n_gpus"], round(x["implied_ms_per_step"], 4), round(x["implied_speedup"], 2)) for x in d["c3_shards"]])
print("model", {k: d["model_leg"].get(k) for k in ("call_ms", "hbm_kernel_ms")})
print("cpu", d["cpu_baseline"]["value"] if d.get("cpu_baseline") else None)
PY
