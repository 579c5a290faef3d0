"""Dev: repeat the c5 golden fixture (device path, key slice) and report any
verdict / fail-op mismatch in detail."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402

z = np.load(os.path.join(ROOT, "tests", "golden", "c5.npz"))
dev = torch.device("cuda", 0)
ctx = abi.Context(device_mask=1)
bad_runs = 0
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 30):
    for a, b in ((50, 250), (0, len(z["key_off"]) - 1)):
        d_ops = torch.from_numpy(np.ascontiguousarray(z["ops"][z["key_off"][a]:])).to(dev)
        d_off = torch.from_numpy(np.ascontiguousarray(z["key_off"][a:b + 1])).to(dev)
        d_out = torch.zeros((b - a) * 40, dtype=torch.uint8, device=dev)
        s = torch.cuda.current_stream(dev)
        ctx.check_device(d_ops.data_ptr(), d_off.data_ptr(), b - a, d_out.data_ptr(),
                         stream=s.cuda_stream)
        r = np.frombuffer(d_out.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)
        st = ctx.stats()
        bad = np.nonzero((r["verdict"] != z["verdict"][a:b]) | (r["fail_op"] != z["fail_op"][a:b]))[0]
        if len(bad):
            bad_runs += 1
            for k in bad[:5]:
                print("rep", rep, "slice", a, b, "key", a + k, "got", r[k], "want",
                      z["verdict"][a + k], z["fail_op"][a + k], "n_gap", st["n_gap_keys"],
                      "n_jit", st["n_jit_keys"], flush=True)
print("bad runs", bad_runs)
