# Counter passes over the temporal box wgrad vs the im2col wgrad (tools/twgrad_probe.py).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${TW_PMC_TAG:-tw_pmc}
mkdir -p $D
ARGS="${@:-}"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $D/t -o run --output-format csv -- python tools/twgrad_probe.py $ARGS > $D/t.log 2>&1 || { tail -5 $D/t.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS -d $D/a -o run --output-format csv -- python tools/twgrad_probe.py $ARGS > $D/a.log 2>&1 || { tail -5 $D/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $D/b -o run --output-format csv -- python tools/twgrad_probe.py $ARGS > $D/b.log 2>&1 || { tail -5 $D/b.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $D/c -o run --output-format csv -- python tools/twgrad_probe.py $ARGS > $D/c.log 2>&1 || { tail -5 $D/c.log; exit 1; }
find $D -name "*.csv" -size +20M -delete
python tools/pmc_kernels.py $D > $D/summary.txt
cat $D/summary.txt
