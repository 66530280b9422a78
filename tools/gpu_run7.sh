set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -q -m gpu -s > gpurun_out/pytest_gpu.log 2>&1 || true
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --batch_per_gpu 256 > gpurun_out/bench_bs256.json 2> gpurun_out/bench_bs256.err || { tail -30 gpurun_out/bench_bs256.err; exit 1; }
cat gpurun_out/bench_bs256.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bs256 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --batch_per_gpu 256 > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-include-regex "conv_" -d gpurun_out/pmc1 -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --batch_per_gpu 128 > gpurun_out/pmc1.log 2>&1 || { tail -20 gpurun_out/pmc1.log; exit 1; }
