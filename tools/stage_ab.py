"""Dev: the small host-buffer calls (C1, C4 valid / invalid, the C5 drop-in
with witnesses, certificates and :configs) as bench.py times them; run once
with LC_STAGE=0 and once without to compare the pageable copies with the
pinned staging buffer.
    LC_STAGE=0 python tools/stage_ab.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from jepsen.etcd_amd import abi  # noqa: E402

with abi.Context(device_mask=1) as ctx:
    c1 = bench.c1_leg(ctx, abi)
    hk = bench.hot_key(ctx, abi)
    dr = bench.dropin_leg(ctx, abi)
print(json.dumps({"stage": os.environ.get("LC_STAGE", "1"),
                  "c1": [c1["gpu_call_ms"], c1["gpu_call32_ms"], c1["check32_result_mismatches"],
                         c1["verdict_mismatches_vs_oracle"]],
                  "c4": [hk["call_ms"], hk["gap_kernel_ms"], hk["invalid"]["call_ms"],
                         hk["invalid"]["fail_op"]],
                  "dropin": [dr["check32_with_witness_and_certificates_ms"], dr["configs_ms"],
                             dr["total_ms"], dr["certified_kinds"],
                             dr["configs_mismatches_vs_oracle_frontier"]]}))
