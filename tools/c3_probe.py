"""Dev probe: bench.py's c3_shards leg alone, `reps` times (the C2 batch cut
into 1/2/4/8 shards, each timed as lc_check_device steps on this GPU)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from jepsen.etcd_amd import abi  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
dev = torch.device("cuda", 0)
ops, off, _, _ = abi.synth(10000, 1000, concurrency=20, seed=0x5EED0002)
d_ops = torch.from_numpy(np.ascontiguousarray(ops)).to(dev)
d_off = torch.from_numpy(np.ascontiguousarray(off)).to(dev)
stream = torch.cuda.current_stream(dev)
with abi.Context(device_mask=1) as ctx:
    for r in range(reps):
        out = bench.c3_shards(ctx, abi, ops, off, d_ops, d_off, dev, stream)
        print(json.dumps([{"n": c["n_gpus"], "implied_us": round(c["implied_ms_per_step"] * 1e3, 1),
                           "speedup": round(c["implied_speedup"], 2),
                           "shards_us": [round(x["ms_per_step"] * 1e3, 1) for x in c["shards"]],
                           "kernel_us": [round(x["kernel_ms"] * 1e3, 1) for x in c["shards"]]}
                          for c in out]), flush=True)
