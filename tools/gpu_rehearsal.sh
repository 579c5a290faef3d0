# The 2-rank rehearsal of the driver's N = 2 run on one GPU: two ranks over
# gloo, both on device 0 (LC_BENCH_DEVICE), the fan-out leg with two virtual
# device contexts, the oversized key over both ranks through gloo callbacks
# (RCCL needs one GPU per rank).  Output: gpurun_out/r6/gloo2.json.
set -o pipefail
mkdir -p gpurun_out/r6
LC_BENCH_BACKEND=gloo LC_BENCH_DEVICE=0 LC_BENCH_FX_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 > gpurun_out/r6/gloo2.json 2> gpurun_out/r6/gloo2.err || { tail -30 gpurun_out/r6/gloo2.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r6/gloo2.json').read().strip().splitlines()[-1]); f=d.get('fanout_leg') or {}; print(d['value'], d['ms_per_step']); print(json.dumps({k: (v.get('call_ms'), [x.get('total_ms') for x in v.get('devices', [])]) for k, v in f.items() if isinstance(v, dict) and 'call_ms' in v}))"
