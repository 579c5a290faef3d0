"""The drop-in's host path on C2: lc_check (48-byte records) against
lc_check32 (24-byte, ABI 4), pageable and page-locked, one device context
and LC_VIRTUAL_DEVICES contexts, with lc_call_profile per call.  JSON lines.
  python tools/host32_probe.py [virtual_devices ...]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jepsen.etcd_amd import abi  # noqa: E402


def run(ctx, fn, reps=5):
    rows = []
    for _ in range(reps):
        t0 = time.perf_counter()
        _, r = fn()
        ms = (time.perf_counter() - t0) * 1e3
        rows.append((ms, ctx.call_profile(), ctx.device_stats(), r))
    rows = rows[1:]
    rows.sort(key=lambda x: x[0])
    return rows[len(rows) // 2]


def main():
    ops, off, _, _ = abi.synth(10000, 1000, concurrency=20, seed=0x5EED0002)
    t0 = time.perf_counter()
    o32, base = abi.pack32(ops, off)
    print(json.dumps({"pack32_ms": (time.perf_counter() - t0) * 1e3}), flush=True)
    want = None
    for nv in [1] + [int(x) for x in sys.argv[1:]]:
        if nv > 1:
            os.environ["LC_VIRTUAL_DEVICES"] = str(nv)
        else:
            os.environ.pop("LC_VIRTUAL_DEVICES", None)
        with abi.Context(device_mask=1) as ctx:
            for name, buf, fn in (("lc_check", ops, lambda: ctx.check(ops, off)),
                                  ("lc_check32", o32, lambda: ctx.check32(o32, off, base))):
                for reg in (False, True):
                    if reg:
                        ctx.host_register(buf)
                    try:
                        ms, prof, devs, r = run(ctx, fn)
                    finally:
                        if reg:
                            ctx.host_unregister(buf)
                    if want is None:
                        want = r
                    print(json.dumps({"devices": nv, "call": name, "registered": reg, "ms": ms,
                                      "same": bool((r == want).all()),
                                      "profile": {k: round(v, 3) if isinstance(v, float) else v
                                                  for k, v in prof.items()},
                                      "dev": [{"h2d_ms": round(d["h2d_ms"], 3),
                                               "kernel_ms": round(d["kernel_ms"], 3),
                                               "total_ms": round(d["total_ms"], 3),
                                               "keys": [d["key_begin"], d["key_end"]]}
                                              for d in devs]}), flush=True)


if __name__ == "__main__":
    main()
