set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --kernel-include-regex "conv_" -d gpurun_out/pmc6 -o run --output-format csv -- python tools/conv_bench.py --batch 128 > gpurun_out/pmc6.log 2>&1 || { tail -20 gpurun_out/pmc6.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_MISC --kernel-include-regex "conv_" -d gpurun_out/pmc7 -o run --output-format csv -- python tools/conv_bench.py --batch 128 > gpurun_out/pmc7.log 2>&1 || { tail -20 gpurun_out/pmc7.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py -q -m gpu -x -k "maxpool or fused" > gpurun_out/pytest_pool.log 2>&1 || { tail -30 gpurun_out/pytest_pool.log; exit 1; }
tail -2 gpurun_out/pytest_pool.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bs256 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --batch_per_gpu 256 > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
