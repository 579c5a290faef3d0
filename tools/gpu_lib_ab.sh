# Dev: bench.py --bare (the C2 step) with the in-tree library and with a
# variant build (LINCHECK_LIB=$1), interleaved 3 times each
set -o pipefail
mkdir -p gpurun_out/ab
for i in 1 2 3; do
  for lib in "" "$1"; do
    timeout -k 10 200 env ${lib:+LINCHECK_LIB=$PWD/$lib} python bench.py --bare --steps 50 --warmup 5 > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err || { tail -5 gpurun_out/ab/b.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/ab/b.json').read().strip().splitlines()[-1]); print('${lib:-default}', 'ms %.4f kernel %.4f value %.4g' % (d['ms_per_step'], d['roofline']['kernel_ms'], d['value']))"
  done
done
