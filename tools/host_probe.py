"""Dev probe: bench.py's host legs alone — C2 from host memory as 24-byte
(lc_check32) and 16-byte (lc_check16) records, pageable and page-locked."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from jepsen.etcd_amd import abi  # noqa: E402

ops, off, _, _ = abi.synth(10000, 1000, concurrency=20, seed=0x5EED0002)
with abi.Context(device_mask=1) as ctx:
    for leg in sys.argv[1:] or ["host_leg32", "host_leg16"]:
        r = getattr(bench, leg)(ctx, abi, ops, off)
        print(json.dumps({"leg": leg, **{k: v for k, v in r.items() if k not in ("pageable", "registered")},
                          **{m: {k: r[m][k] for k in ("call_ms", "h2d_ms", "h2d_gb_per_s",
                                                      "result_mismatches_vs_lc_check")}
                             for m in ("pageable", "registered") if m in r}}), flush=True)
