# Counter passes over one flagship training step (the last of bench.py --steps 1 --warmup 1):
# bash tools/gpu/step_pmc.sh TAG   -> gpurun_out/TAG/{a,b,c}/ + table.txt (tools/pmc_step.py)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${1:-step_pmc}
mkdir -p $D
RUN="python bench.py --steps 1 --warmup 1"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $D/a -o run --output-format csv -- $RUN > $D/a.log 2>&1 || { tail -5 $D/a.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $D/b -o run --output-format csv -- $RUN > $D/b.log 2>&1 || { tail -5 $D/b.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_LDS_IDX_ACTIVE -d $D/c -o run --output-format csv -- $RUN > $D/c.log 2>&1 || { tail -5 $D/c.log; exit 1; }
python tools/pmc_step.py --trace $D/a/run_kernel_trace.csv --pmc $D/a/run_counter_collection.csv $D/b/run_counter_collection.csv $D/c/run_counter_collection.csv --top 60 > $D/table.txt
find $D -name "*.csv" -size +20M -delete
head -60 $D/table.txt
