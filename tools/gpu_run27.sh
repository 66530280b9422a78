cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc27
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc27/a -o run --output-format csv -- python tools/stem_probe.py > gpurun_out/pmc27/a.log 2>&1 || { tail -5 gpurun_out/pmc27/a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM -d gpurun_out/pmc27/c -o run --output-format csv -- python tools/stem_probe.py > gpurun_out/pmc27/c.log 2>&1 || { tail -5 gpurun_out/pmc27/c.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc27/t -o run --output-format csv -- python tools/stem_probe.py > gpurun_out/pmc27/t.log 2>&1 || { tail -5 gpurun_out/pmc27/t.log; exit 1; }
echo ok
