# Dev: C4 call timings (tools/c4_probe.py), and a kernel trace of each history's calls
mkdir -p gpurun_out/c4
timeout -k 10 120 python -u tools/c4_probe.py > gpurun_out/c4/probe.txt 2>&1 || { tail -20 gpurun_out/c4/probe.txt; exit 1; }
tail -1 gpurun_out/c4/probe.txt
for t in valid invalid; do
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/c4/kt_$t -o kt --output-format csv -- python3 tools/c4_probe.py --reps 2 --only $t > gpurun_out/c4/kt_$t.log 2>&1 || { tail -20 gpurun_out/c4/kt_$t.log; exit 1; }
done
