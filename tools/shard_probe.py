"""Dev probe (round 6): the version-order pass at C3 shard sizes.  For each
key count (a prefix of the C2 batch) STEPS back-to-back lc_check_device
calls, untimed (LC_FLAG_NO_TIMING), so a rocprofv3 kernel trace of this
process holds the kernel's own durations by grid size (tools/kt_grid.py),
and the wall time per step is printed.
  python tools/shard_probe.py [steps] [sizes,comma,separated]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from jepsen.etcd_amd import abi  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    sizes = ([int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2
             else [1, 157, 313, 625, 1250, 2500, 5000, 10000])
    dev = torch.device("cuda", 0)
    ops, off, _, _ = abi.synth(10000, 1000, concurrency=20, seed=0x5EED0002)
    d_ops = torch.from_numpy(ops).to(dev)
    d_off = torch.from_numpy(off).to(dev)
    stream = torch.cuda.current_stream(dev)
    with abi.Context(device_mask=1) as ctx:
        for nk in sizes:
            out = torch.zeros(nk * abi.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
            call = ctx.bind_check_device(d_ops.data_ptr(), d_off.data_ptr(), nk, out.data_ptr(),
                                         stream=stream.cuda_stream,
                                         opts=abi.default_opts(flags=abi.LC_FLAG_NO_TIMING))
            for _ in range(20):
                call()
            torch.cuda.synchronize()
            ctx.totals(reset=True)
            t0 = time.perf_counter()
            for _ in range(steps):
                call()
            ctx.quiesce()
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) * 1e6 / steps
            tot = ctx.totals(reset=True)
            dev_us = tot["fast_kernel_ms"] * 1e3 / max(1, tot["timed_calls"])
            res = np.frombuffer(out.cpu().numpy().tobytes(), dtype=abi.RESULT_DTYPE)[:nk]
            print(json.dumps({"keys": nk, "us_per_step": round(us, 2),
                              "device_us": round(dev_us, 2), "timed": tot["timed_calls"],
                              "valid": int((res["verdict"] == 1).sum()),
                              "lib": os.environ.get("LINCHECK_LIB", "in-tree")}), flush=True)


if __name__ == "__main__":
    main()
