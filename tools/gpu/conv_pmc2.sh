# PMC passes (one counter group per run) over tools/conv_impls.py-style single-layer runs of the
# given implementation list: bash tools/gpu/conv_pmc2.sh TAG "--cin 192 --cout 192 --k 3 1 1" "4 8 12"
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/$1
mkdir -p $D
ARGS="$2 --impls $3"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $D/t -o run --output-format csv -- python tools/conv_impls.py $ARGS > $D/t.log 2>&1 || { tail -5 $D/t.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS -d $D/a -o run --output-format csv -- python tools/conv_impls.py $ARGS > $D/a.log 2>&1 || { tail -5 $D/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $D/b -o run --output-format csv -- python tools/conv_impls.py $ARGS > $D/b.log 2>&1 || { tail -5 $D/b.log; exit 1; }
find $D -name "*.csv" -size +20M -delete
python tools/pmc_kernels.py $D > $D/summary.txt
grep -E "==|wait|mfma busy|valu/mfma|clock" $D/summary.txt
