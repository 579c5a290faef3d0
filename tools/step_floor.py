"""Dev probe: where a bench step's time goes at C3 shard sizes (1,250 -
10,000 keys of the C2 batch): Python wall per step, the C call's own time
(lc_stats.total_ms), and the fast tier's HIP-event time, for a run of
back-to-back lc_check_device steps on one GPU."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    ops, off, _, _ = abi.synth(10000, 1000, concurrency=20, seed=0x5EED0002)
    d_ops = torch.from_numpy(ops).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    stream = torch.cuda.current_stream(dev)
    with abi.Context(device_mask=1) as ctx:
        for nk in (1, 1250, 2500, 5000, 10000):
            out = torch.zeros(nk * abi.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            for every in (1, 4, 0):  # timed steps: every step, every 4th, none
                fl = [0, abi.LC_FLAG_NO_TIMING]
                steps_ = [ctx.bind_check_device(d_ops.data_ptr(), d_off.data_ptr(), nk, out.data_ptr(),
                                                stream=stream.cuda_stream, opts=abi.default_opts(flags=f))
                          for f in fl]
                pick = (lambda i: 0 if i % every == 0 else 1) if every else (lambda i: 1)
                for i in range(20):
                    steps_[pick(i)]()
                torch.cuda.synchronize()
                ctx.totals(reset=True)
                wall = []
                t_all = time.perf_counter()
                for i in range(steps):
                    t0 = time.perf_counter()
                    steps_[pick(i)]()
                    wall.append((time.perf_counter() - t0) * 1e6)
                t_all = (time.perf_counter() - t_all) * 1e6 / steps
                tot = ctx.totals(reset=True)
                print(json.dumps({"keys": nk, "timed_every": every, "us_per_step": round(t_all, 2),
                                  "wall_us_med": round(float(np.median(wall)), 2),
                                  "kernel_us_mean": round(tot["fast_kernel_ms"] * 1e3 /
                                                          max(1, tot["timed_calls"]), 2)}),
                      flush=True)


if __name__ == "__main__":
    main()
