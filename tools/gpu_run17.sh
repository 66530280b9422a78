set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -q -m gpu -x > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --batch_per_gpu 256 > gpurun_out/bench_bs256.json 2> gpurun_out/bench_bs256.err || { tail -30 gpurun_out/bench_bs256.err; exit 1; }
cat gpurun_out/bench_bs256.json
timeout -k 10 600 python tools/conv_bench.py > gpurun_out/conv_bench.txt 2>&1 || { tail -20 gpurun_out/conv_bench.txt; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bs256 -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --batch_per_gpu 256 > gpurun_out/prof_bench.log 2>&1 || { tail -20 gpurun_out/prof_bench.log; exit 1; }
