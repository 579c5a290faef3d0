"""Dev: bench.py's resident32_leg alone (the C2 batch as 24-byte records
resident in HBM through lc_check_device32), with the main loop's 48-byte
step beside it for comparison.

    python tools/resident32.py [reps]
"""
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
stream = torch.cuda.Stream(device=dev)
ops, key_off, _, _ = abi.synth(10000, 1000, concurrency=20, p_info=0.0, seed=0x5EED0002)
d_ops = torch.from_numpy(np.ascontiguousarray(ops)).to(dev)
d_off = torch.from_numpy(np.ascontiguousarray(key_off)).to(dev)
with abi.Context(device_mask=1) as ctx:
    for _ in range(reps):
        r = bench.resident32_leg(ctx, abi, ops, key_off, d_ops, d_off, dev, stream)
        c = bench.c3_shards(ctx, abi, ops, key_off, d_ops, d_off, dev, stream)[0]
        print(json.dumps({"resident32": {k: r[k] for k in ("ms_per_step", "ops_per_s", "kernel_ms",
                                                            "frac_of_hbm_peak", "valid",
                                                            "result_mismatches_vs_48_byte")},
                          "resident48_ms_per_step": c["implied_ms_per_step"],
                          "resident48_kernel_ms": c["shards"][0]["kernel_ms"]}), flush=True)
