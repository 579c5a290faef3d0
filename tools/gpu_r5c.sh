mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests/test_gpu_witness.py tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/r5/t4.log 2>&1 || { tail -40 gpurun_out/r5/t4.log; exit 1; }
tail -2 gpurun_out/r5/t4.log
