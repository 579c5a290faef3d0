"""Dev probe: fast-tier kernel time against the number of keys (1,000-op
keys), to see the workgroup-round quantization (7 workgroups per CU x 256
CUs = 1,792 keys per round)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402

dev = torch.device("cuda:0")
ops, off, _, _ = abi.synth(12544, 1000, concurrency=20, seed=0x5EED0001)
d_ops = torch.from_numpy(ops).to(dev)
stream = torch.cuda.current_stream(dev)
with abi.Context(device_mask=1) as ctx:
    for n in (1792, 3584, 5376, 7168, 8960, 9500, 10000, 10752, 11000, 12544):
        d_off = torch.from_numpy(off[:n + 1].copy()).to(dev)
        d_out = torch.zeros(n * abi.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        st = abi.LcStats()
        call = ctx.bind_check_device(d_ops.data_ptr(), d_off.data_ptr(), n, d_out.data_ptr(),
                                     stream=stream.cuda_stream, stats=st)
        f = []
        for _ in range(30):
            call()
            f.append(st.fast_kernel_ms)
        t = float(np.median(f[5:]))
        print(json.dumps({"keys": n, "rounds": round(n / 1792, 2), "fast_ms": round(t, 4),
                          "us_per_1k_keys": round(t * 1e3 / n * 1e3, 3),
                          "tb_s": round((48 * 1000 * n + 40 * n) / (t * 1e-3) / 1e12, 3)}), flush=True)
