set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 -L > gpurun_out/counters_avail.txt 2>&1 || true
timeout -k 10 600 python tools/conv_bench.py > gpurun_out/conv_bench.txt 2>&1 || { tail -20 gpurun_out/conv_bench.txt; exit 1; }
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "conv_" -d gpurun_out/pmc2 -o run --output-format csv -- python tools/conv_bench.py --batch 64 > gpurun_out/pmc2.log 2>&1 || { tail -20 gpurun_out/pmc2.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "conv_" -d gpurun_out/pmc3 -o run --output-format csv -- python tools/conv_bench.py --batch 64 > gpurun_out/pmc3.log 2>&1 || { tail -20 gpurun_out/pmc3.log; exit 1; }
