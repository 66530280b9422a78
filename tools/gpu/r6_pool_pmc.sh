# Counter passes over tools/pool_bench.py (one shape, given impls) -> tools/pmc_kernels.py summary.
# bash tools/gpu/r6_pool_pmc.sh TAG "SHAPE_IDX" "IMPLS"
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-r6poolpmc}
mkdir -p $D
RUN="python tools/pool_bench.py --only ${2:-1} --impls ${3:-2,1}"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $D/a -o run --output-format csv -- $RUN > $D/a.log 2>&1 || { tail -5 $D/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS FETCH_SIZE -d $D/b -o run --output-format csv -- $RUN > $D/b.log 2>&1 || { tail -5 $D/b.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_INSTS_VMEM SQ_WAIT_INST_ANY -d $D/c -o run --output-format csv -- $RUN > $D/c.log 2>&1 || { tail -5 $D/c.log; exit 1; }
python tools/pmc_kernels.py $D > $D/summary.txt
find $D -name "*.csv" -size +20M -delete
cat $D/summary.txt
