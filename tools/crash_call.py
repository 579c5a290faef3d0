"""Dev: bench.py's crash_leg alone (call_ms and the fused kernel's), N times."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from jepsen.etcd_amd import abi  # noqa: E402

dev = torch.device("cuda:0")
stream = torch.cuda.Stream(device=dev)
with abi.Context(device_mask=1) as ctx:
    for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
        r = bench.crash_leg(ctx, abi, dev, stream)
        print(json.dumps({k: r[k] for k in ("call_ms", "fast_kernel_ms", "valid")}), flush=True)
