set -e
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$PWD
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_BRANCH -d $R/gpurun_out/pmc/a -o a --output-format csv -- python3 $R/tools/gap_probe.py 2 C4 > $R/gpurun_out/pmc/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d $R/gpurun_out/pmc/b -o b --output-format csv -- python3 $R/tools/gap_probe.py 2 C4 > $R/gpurun_out/pmc/b.log 2>&1
