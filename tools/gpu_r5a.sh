mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest tests/test_frontiers.py tests/test_op32.py "tests/test_gpu.py::test_register_checker_end_to_end" "tests/test_gpu.py::test_register_checker_frontier_configs" -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/r5/t1.log 2>&1 || { tail -40 gpurun_out/r5/t1.log; exit 1; }
tail -3 gpurun_out/r5/t1.log
timeout -k 10 200 python -u -c "
import json, bench
from jepsen.etcd_amd import abi
with abi.Context(device_mask=1) as ctx:
    print(json.dumps(bench.dropin_leg(ctx, abi)))
" > gpurun_out/r5/dropin.json 2>gpurun_out/r5/dropin.err && cat gpurun_out/r5/dropin.json
timeout -k 10 300 python -u tools/host32_probe.py 2 > gpurun_out/r5/host32e.jsonl 2>gpurun_out/r5/host32.err
timeout -k 10 300 python -u -m pytest tests/test_edn.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/r5/edn.log 2>&1; tail -2 gpurun_out/r5/edn.log
