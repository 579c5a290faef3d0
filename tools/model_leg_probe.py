"""Dev probe: bench.py's model_leg alone (its JSON)."""
import json, sys, os
sys.path.insert(0, os.getcwd())
import bench
from jepsen.etcd_amd import abi
with abi.Context(device_mask=1) as ctx:
    print(json.dumps(bench.model_leg(ctx, abi), default=str))
