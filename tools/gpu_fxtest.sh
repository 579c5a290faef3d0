set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_fx.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/fxtest.log 2>&1
rc=$?; tail -30 gpurun_out/fxtest.log; exit $rc
