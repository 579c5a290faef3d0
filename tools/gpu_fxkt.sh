# Dev: the oversized key's wall time (3 checks, LC_FX_DEBUG counters) and a
# kernel trace of one check for tools/fx_gaps.py
mkdir -p gpurun_out/fx
LC_FX_DEBUG=1 timeout -k 10 120 python -u tools/fx_once.py --reps 3 > gpurun_out/fx/once.txt 2>&1 || { tail -20 gpurun_out/fx/once.txt; exit 1; }
tail -3 gpurun_out/fx/once.txt
timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/fx/kt -o kt --output-format csv -- python3 tools/fx_once.py --reps 1 > gpurun_out/fx/kt.log 2>&1 || { tail -20 gpurun_out/fx/kt.log; exit 1; }
tail -1 gpurun_out/fx/kt.log
