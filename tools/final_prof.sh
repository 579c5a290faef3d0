set -euo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r02final
mkdir -p $O
timeout -k 10 300 python3 -u $R/bench.py > $O/bench.json 2> $O/bench.err
echo bench done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --bare --steps 20 > $O/kt.log 2>&1
echo kt done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 $R/bench.py --bare --steps 5 > $O/fetch.log 2>&1
echo fetch done
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o write --output-format csv -- python3 $R/bench.py --bare --steps 5 > $O/write.log 2>&1
echo write done
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/l2 -o l2 --output-format csv -- python3 $R/bench.py --bare --steps 5 > $O/l2.log 2>&1
echo l2 done
