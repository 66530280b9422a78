#!/bin/bash
# Counters of the stride-1 pool sweeps at the Mixed_3 shapes (tools/pool_bench.py):
# bash tools/gpu/pool_pmc.sh TAG  -> gpurun_out/TAG/{a,b,c}/ + summary.txt (tools/pmc_kernels.py)
set -o pipefail
D=gpurun_out/${1:-pool_pmc}
mkdir -p $D
RUN="python tools/pool_bench.py --only 0,1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU -d $D/a -o run --output-format csv -- $RUN > $D/a.log 2>&1 || { tail -5 $D/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum -d $D/b -o run --output-format csv -- $RUN > $D/b.log 2>&1 || { tail -5 $D/b.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d $D/c -o run --output-format csv -- $RUN > $D/c.log 2>&1 || { tail -5 $D/c.log; exit 1; }
python tools/pmc_kernels.py $D > $D/summary.txt
